"""End-to-end downlink receive on the GPU: time-domain subframes -> OFDM FFT -> CRS channel
estimation -> PDSCH (RE extraction, MMSE with the estimator's noise, demap, descramble) ->
DL-SCH decode, against a transmitter built from the oracles (DL-SCH encoder, scrambling, 36.211
modulation, CRS, OFDM modulator) over a smooth fading channel with AWGN. Intermediate grids are
checked against the numpy oracles within float tolerances (frequency-selective, time-flat channel), the final TBs bit-exactly against the
transmitted bytes."""
import os
import sys

import numpy as np
import pytest

from srsgpu_testlib import DlschOracle, PdschOracle

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import chest_oracle as co  # noqa: E402
import ofdm_oracle as oo  # noqa: E402
from test_pdsch_gpu import _modulate  # noqa: E402

pytestmark = pytest.mark.gpu


def build_subframe(po, dl, rng, nof_prb, cell_id, N, sf_idx, tbs, rnti, snr_db, phase):
    idx = po.re_map(nof_prb, cell_id, 1, 1, sf_idx, np.ones((2, nof_prb), np.uint8))
    nbits = idx.size * 6
    data = rng.integers(0, 256, tbs // 8).astype(np.uint8)
    e = dl.encode(tbs, 0, 6, nbits, data)
    c = po.sequence(po.seed(rnti, 0, 2 * sf_idx, cell_id), nbits)
    grid = np.zeros(14 * 12 * nof_prb, np.complex128)
    grid[idx] = _modulate(e ^ c, 3)
    g2 = grid.reshape(14, -1)
    pil = co.crs_pilots(nof_prb, cell_id, sf_idx)
    for l, s in enumerate(co.SYMS):
        g2[s, co.fidx(cell_id, l) + 6 * np.arange(2 * nof_prb)] = pil[l]
    k = np.arange(12 * nof_prb)
    h = np.tile((1 + 0.3 * np.cos(2 * np.pi * k / k.size + phase)) * np.exp(1j * (phase + 0.5 * np.sin(2 * np.pi * k / k.size))), 14)
    x = oo.tx_sf(grid * h, nof_prb, N) / N  # per-subcarrier channel applied in frequency
    sig = 10 ** (-snr_db / 20) / np.sqrt(2 * N)
    x = x + sig * (rng.standard_normal(x.size) + 1j * rng.standard_normal(x.size))
    return x.astype(np.complex64), data, idx


def test_time_domain_to_transport_blocks(oracle):
    import torch
    import srsgpu_phy as s
    po, dl = PdschOracle(oracle), DlschOracle(oracle)
    rng = np.random.default_rng(2024)
    nof_prb, cell_id, tbs, rnti = 100, 1, 75376, 1234
    N = s.symbol_sz(nof_prb, True)
    n = 8
    xs, datas, sfs = [], [], []
    for i in range(n):
        sf_idx = [1, 2, 3, 4, 6, 7, 8, 9][i]
        x, data, idx = build_subframe(po, dl, rng, nof_prb, cell_id, N, sf_idx, tbs, rnti, 30.0,
                                      rng.uniform(0, 6.28))
        xs.append(x)
        datas.append(data)
        sfs.append((sf_idx, idx.size))
    gsz = 14 * 12 * nof_prb
    stream = torch.cuda.current_stream().cuda_stream
    ofdm = s.OfdmRx(nof_prb, N, stream=stream)
    chest = s.Chest(nof_prb, cell_id, max_grids=n, stream=stream)
    pd = s.Pdsch(nof_prb, cell_id, nof_softbuffers=n, max_sf=n, stream=stream)
    d_x = torch.from_numpy(np.stack(xs).reshape(-1)).cuda()
    d_grid = torch.zeros(n * gsz, dtype=torch.complex64, device="cuda")
    d_ce = torch.zeros_like(d_grid)
    d_noise = torch.zeros(n, dtype=torch.float32, device="cuda")
    assert ofdm.rx_dev(n, d_x.data_ptr(), 15 * N, d_grid.data_ptr(), gsz) == 0
    assert chest.estimate_dev([sf for sf, _ in sfs], d_grid.data_ptr(), gsz, d_ce.data_ptr(),
                              d_noise.data_ptr()) == 0
    pd.set_noise_dev(d_noise.data_ptr())
    dlen = tbs // 8 + 6
    sfl = []
    for i, (sf_idx, nre) in enumerate(sfs):
        pd.reset_softbuffer(i)
        sfl.append(s.make_sf(sf_idx=sf_idx, lstart=1, nof_prb=nof_prb, mod=3, nof_re=nre, rnti=rnti,
                             tbs=tbs, softbuffer=i, grid_offset=i * gsz, data_offset=i * dlen))
    d_data = torch.zeros(n * dlen, dtype=torch.uint8, device="cuda")
    d_ret = torch.full((n,), 9, dtype=torch.int32, device="cuda")
    d_noi = torch.zeros(n, dtype=torch.int32, device="cuda")
    assert pd.decode_dev(sfl, d_grid.data_ptr(), d_ce.data_ptr(), gsz, d_data.data_ptr(), 8,
                         d_ret.data_ptr(), d_noi.data_ptr()) == 0
    torch.cuda.synchronize()
    # intermediate stages vs the numpy oracles
    grid = d_grid.cpu().numpy().reshape(n, -1)
    ce = d_ce.cpu().numpy().reshape(n, -1)
    for i in range(n):
        rg = oo.rx_sf(xs[i], nof_prb, N)
        assert np.max(np.abs(grid[i] - rg)) / np.sqrt(np.mean(np.abs(rg) ** 2)) < 1e-4
        rce, rn = co.estimate(grid[i].astype(np.complex128), nof_prb, cell_id, sfs[i][0])
        assert np.max(np.abs(ce[i] - rce)) / np.max(np.abs(rce)) < 1e-4
    ret = d_ret.cpu().numpy()
    out = d_data.cpu().numpy().reshape(n, dlen)
    assert (ret == 0).all(), ret
    for i in range(n):
        assert (out[i][:tbs // 8] == datas[i]).all(), i
    for o in (ofdm, chest, pd):
        o.close()
