"""Channel estimation (chest_dl.c restated in oracle/chest_oracle.py, GPU in chest_kernels.hip).

CPU: the CRS table and pilot extraction of the oracle equal the reference's refsignal_dl.c
(compiled into oracle/_ref); the estimator reproduces the reference's own chest_test_dl check on
its smooth synthetic channel. The rest of chest_dl.c needs the FFTW-backed DFT through
pss.c/convolution.c and cannot be built here: parity of smoothing/interpolation/noise is
unpinned restatement, compared on the GPU with a float tolerance.
"""
import ctypes
import os
import sys

import numpy as np
import pytest

from srsgpu_testlib import Ref, have_ref

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import chest_oracle as co  # noqa: E402

f32 = ctypes.POINTER(ctypes.c_float)


def smooth_channel(nof_prb):
    """chest_test_dl.c:158-164 channel: h = (3 + x) exp(jx), x = -1 + i/7 + cos(2 pi j / (12 nprb))"""
    i = np.arange(14)[:, None]
    j = np.arange(12 * nof_prb)[None, :]
    x = -1 + i / 7 + np.cos(2 * np.pi * j / nof_prb / 12)
    return ((3 + x) * np.exp(1j * x)).reshape(-1)


def crs_grid(nof_prb, cell_id, sf_idx, rng, port=0):
    """random data REs with the CRS of `port` placed (refsignal_cs_put_sf)"""
    g = ((0.5 - rng.random((14, 12 * nof_prb))) + 1j * (0.5 - rng.random((14, 12 * nof_prb))))
    pil = co.crs_pilots(nof_prb, cell_id, sf_idx)
    for l, s in enumerate(co.SYMS):
        g[s, co.fidx(cell_id, l, port) + 6 * np.arange(2 * nof_prb)] = pil[l]
    return g.reshape(-1)


@pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built (build container only)")
def test_crs_and_pilot_extraction_vs_reference():
    L = Ref().lib
    L.ref_crs_pilots.argtypes = [ctypes.c_uint32] * 3 + [f32]
    L.ref_crs_get_sf.argtypes = [ctypes.c_uint32] * 3 + [f32, f32]
    rng = np.random.default_rng(0)
    for nof_prb, cid in ((100, 1), (6, 0), (25, 503), (50, 17), (75, 254)):
        for sf in (0, 3, 9):
            out = np.zeros(4 * 2 * nof_prb, np.complex64)
            assert L.ref_crs_pilots(nof_prb, cid, sf, out.ctypes.data_as(f32)) == 0
            assert np.allclose(out.reshape(4, -1), co.crs_pilots(nof_prb, cid, sf), atol=1e-7)
        grid = (rng.standard_normal(14 * 12 * nof_prb) + 1j * rng.standard_normal(14 * 12 * nof_prb)).astype(np.complex64)
        for port in (0, 1):
            got = np.zeros(4 * 2 * nof_prb, np.complex64)
            assert L.ref_crs_get_sf(nof_prb, cid, port, grid.ctypes.data_as(f32), got.ctypes.data_as(f32)) == 0
            g = grid.reshape(14, -1)
            exp = np.stack([g[s, co.fidx(cid, l, port) + 6 * np.arange(2 * nof_prb)]
                            for l, s in enumerate(co.SYMS)])
            assert (got.reshape(4, -1) == exp).all(), port


def test_oracle_reference_test_property():
    """chest_test_dl.c: equalising the smooth channel with the estimate leaves a small error"""
    rng = np.random.default_rng(1)
    for nof_prb, cid in ((25, 1), (100, 7)):
        h = smooth_channel(nof_prb)
        x = crs_grid(nof_prb, cid, 0, rng)
        ce, _ = co.estimate(x * h, nof_prb, cid, 0)
        assert np.mean(np.abs(x - (x * h) / ce)) < 0.05


@pytest.mark.gpu
@pytest.mark.parametrize("nof_prb,cell_id,filt", [(100, 1, (0.1, 0.8, 0.1)), (25, 5, ()),
                                                  (50, 300, (0.05, 0.2, 0.5, 0.2, 0.05)),
                                                  (6, 2, (0.1, 0.8, 0.1))])
def test_chest_gpu_vs_oracle(nof_prb, cell_id, filt):
    import torch
    import srsgpu_phy as s
    rng = np.random.default_rng(nof_prb + cell_id)
    n = 10
    size = 14 * 12 * nof_prb
    grids, sfs = [], []
    for i in range(n):
        h = smooth_channel(nof_prb) * np.exp(1j * rng.uniform(0, 6.3))
        x = crs_grid(nof_prb, cell_id, i % 10, rng)
        noise = 0.05 * (rng.standard_normal(size) + 1j * rng.standard_normal(size))
        grids.append((x * h + noise).astype(np.complex64))
        sfs.append(i % 10)
    c = s.Chest(nof_prb, cell_id, max_grids=n)
    if len(filt) == 3:
        c.set_filter3(filt[0])
    else:
        c.set_filter(list(filt))
    d_g = torch.from_numpy(np.stack(grids).reshape(-1)).cuda()
    d_ce = torch.zeros_like(d_g)
    d_n = torch.zeros(n, dtype=torch.float32, device="cuda")
    assert c.estimate_dev(sfs, d_g.data_ptr(), size, d_ce.data_ptr(), d_n.data_ptr()) == 0
    torch.cuda.synchronize()
    ce = d_ce.cpu().numpy().reshape(n, -1)
    nz = d_n.cpu().numpy()
    for i in range(n):
        ref_ce, ref_n = co.estimate(grids[i].astype(np.complex128), nof_prb, cell_id, sfs[i], filt)
        scale = np.max(np.abs(ref_ce))
        assert np.max(np.abs(ce[i] - ref_ce)) / scale < 1e-4, i
        assert abs(nz[i] - ref_n) <= 1e-4 * ref_n + 1e-9, (i, nz[i], ref_n)
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("nof_prb,cell_id", [(100, 1), (25, 4), (15, 503)])
def test_chest_two_ports_gpu_vs_oracle(nof_prb, cell_id):
    """2 CRS ports: each grid carries both ports' CRS (different channels); estimates come out
    [grid][port] (srslte_chest_dl_estimate_multi order)"""
    import torch
    import srsgpu_phy as s
    rng = np.random.default_rng(7 * nof_prb + cell_id)
    n = 6
    size = 14 * 12 * nof_prb
    grids = []
    for i in range(n):
        g = np.zeros(size, np.complex128)
        for port in (0, 1):
            h = smooth_channel(nof_prb) * np.exp(1j * rng.uniform(0, 6.3)) * (0.5 + port)
            x = crs_grid(nof_prb, cell_id, i % 10, rng, port)
            # keep only this port's CRS REs (the other port's positions are empty, 36.211 6.10.1.2)
            mask = np.zeros((14, 12 * nof_prb), bool)
            for l, sy in enumerate(co.SYMS):
                mask[sy, co.fidx(cell_id, l, port) + 6 * np.arange(2 * nof_prb)] = True
            g += np.where(mask.reshape(-1), x * h, 0)
        g += 0.02 * (rng.standard_normal(size) + 1j * rng.standard_normal(size))
        grids.append(g.astype(np.complex64))
    sfs = [i % 10 for i in range(n)]
    c = s.Chest(nof_prb, cell_id, max_grids=n, nof_ports=2)
    d_g = torch.from_numpy(np.stack(grids).reshape(-1)).cuda()
    d_ce = torch.zeros(2 * n * size, dtype=torch.complex64, device="cuda")
    d_n = torch.zeros(2 * n, dtype=torch.float32, device="cuda")
    assert c.estimate_dev(sfs, d_g.data_ptr(), size, d_ce.data_ptr(), d_n.data_ptr()) == 0
    torch.cuda.synchronize()
    ce = d_ce.cpu().numpy().reshape(n, 2, -1)
    nz = d_n.cpu().numpy().reshape(n, 2)
    for i in range(n):
        for port in (0, 1):
            ref_ce, ref_n = co.estimate(grids[i].astype(np.complex128), nof_prb, cell_id, sfs[i],
                                        port=port)
            scale = np.max(np.abs(ref_ce))
            assert np.max(np.abs(ce[i, port] - ref_ce)) / scale < 1e-4, (i, port)
            assert abs(nz[i, port] - ref_n) <= 1e-4 * ref_n + 1e-9, (i, port, nz[i, port], ref_n)
    c.close()
