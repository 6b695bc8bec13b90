"""OFDM receive FFT (ofdm.c restated in oracle/ofdm_oracle.py with numpy's float64 FFT — the
reference's FFTW backend is absent, so parity is pinned to numpy)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import ofdm_oracle as oo  # noqa: E402


def test_oracle_roundtrip_and_layout():
    """tx -> rx returns the grid times N (unnormalised DFTs, ofdm_test.c's round trip)"""
    rng = np.random.default_rng(0)
    for nof_prb, N in ((6, 128), (25, 384), (100, 1536), (100, 2048)):
        g = rng.standard_normal(14 * 12 * nof_prb) + 1j * rng.standard_normal(14 * 12 * nof_prb)
        x = oo.tx_sf(g, nof_prb, N)
        assert x.size == 15 * N
        assert np.allclose(oo.rx_sf(x, nof_prb, N), g * N, atol=1e-9 * N)
        assert np.allclose(oo.rx_sf(x, nof_prb, N, normalize=True), g * np.sqrt(N), atol=1e-9 * N)


def test_symbol_sizes():
    import srsgpu_phy as s
    exp = {6: (128, 128), 15: (256, 256), 25: (384, 512), 50: (768, 1024), 75: (1024, 1536),
           100: (1536, 2048)}
    for nprb, (ns, st) in exp.items():  # phy_common.c:227-275
        assert s.symbol_sz(nprb) == ns and s.symbol_sz(nprb, True) == st


@pytest.mark.gpu
@pytest.mark.parametrize("nof_prb,standard", [(100, True), (100, False), (25, False), (25, True),
                                              (6, False), (50, False), (75, False), (15, False)])
def test_ofdm_rx_gpu_vs_numpy(nof_prb, standard):
    import torch
    import srsgpu_phy as s
    N = s.symbol_sz(nof_prb, standard)
    rng = np.random.default_rng(nof_prb * 7 + N)
    n = 6
    x = (rng.standard_normal((n, 15 * N)) + 1j * rng.standard_normal((n, 15 * N))).astype(np.complex64)
    o = s.OfdmRx(nof_prb, N, normalize=(nof_prb == 25))
    d_x = torch.from_numpy(x.reshape(-1)).cuda()
    gsz = 14 * 12 * nof_prb
    d_g = torch.zeros(n * gsz, dtype=torch.complex64, device="cuda")
    assert o.rx_dev(n, d_x.data_ptr(), 15 * N, d_g.data_ptr(), gsz) == 0
    torch.cuda.synchronize()
    got = d_g.cpu().numpy().reshape(n, -1)
    for i in range(n):
        ref = oo.rx_sf(x[i], nof_prb, N, normalize=(nof_prb == 25))
        rms = np.sqrt(np.mean(np.abs(ref) ** 2))
        assert np.max(np.abs(got[i] - ref)) / rms < 1e-4, (i, np.max(np.abs(got[i] - ref)) / rms)
    o.close()


@pytest.mark.gpu
def test_ofdm_rx_gpu_generic_size():
    """a 2^a 3^b size outside the LTE table (1152 = 2^7 3^2) takes the run-time-planned kernel"""
    import torch
    import srsgpu_phy as s
    nof_prb, N, n = 75, 1152, 3
    rng = np.random.default_rng(11)
    x = (rng.standard_normal((n, 15 * N)) + 1j * rng.standard_normal((n, 15 * N))).astype(np.complex64)
    o = s.OfdmRx(nof_prb, N)
    d_x = torch.from_numpy(x.reshape(-1)).cuda()
    gsz = 14 * 12 * nof_prb
    d_g = torch.zeros(n * gsz, dtype=torch.complex64, device="cuda")
    assert o.rx_dev(n, d_x.data_ptr(), 15 * N, d_g.data_ptr(), gsz) == 0
    torch.cuda.synchronize()
    got = d_g.cpu().numpy().reshape(n, -1)
    for i in range(n):
        ref = oo.rx_sf(x[i], nof_prb, N)
        rms = np.sqrt(np.mean(np.abs(ref) ** 2))
        assert np.max(np.abs(got[i] - ref)) / rms < 1e-4
    o.close()
