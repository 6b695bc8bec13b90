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
                                                  (50, 300, (0.05, 0.2, 0.5, 0.2, 0.05)), (75, 9, (0.1, 0.4, 0.4, 0.1)),
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


def _sync_grid(nof_prb, cell_id, sf_idx, nports, rng, sigma=0.02, flat=False):
    """every port's CRS through its own channel; in subframes 0 / 5 the PSS (symbol 6) and a random
    SSS (symbol 5) at the band centre with their 5 empty subcarriers either side (pss.c:386-392)"""
    size = 14 * 12 * nof_prb
    nsc = 12 * nof_prb
    g = np.zeros(size, np.complex128)
    hs = []
    for port in range(nports):
        h = smooth_channel(nof_prb) * np.exp(1j * rng.uniform(0, 6.3)) * (0.5 + port)
        if flat:
            h = np.tile(h.reshape(14, -1)[0], 14)
        hs.append(h)
        x = crs_grid(nof_prb, cell_id, sf_idx, rng, port)
        mask = np.zeros((14, nsc), bool)
        for l, sy in enumerate(co.SYMS):
            mask[sy, co.fidx(cell_id, l, port) + 6 * np.arange(2 * nof_prb)] = True
        g += np.where(mask.reshape(-1), x * h, 0)
    if sf_idx in (0, 5):
        k0 = nsc // 2 - 31
        for s, seq in ((6, co.pss_sequence(cell_id % 3)), (5, np.sign(rng.standard_normal(62)) + 0j)):
            k = s * nsc + k0
            g[k - 5:k] = 0
            g[k + 62:k + 67] = 0
            g[k:k + 62] = seq * hs[0][k:k + 62]
    g += sigma * (rng.standard_normal(size) + 1j * rng.standard_normal(size))
    return g.astype(np.complex64)


def _run_modes(nof_prb, cell_id, nports, sfs, filt, average, noise_alg, filt_auto, noise_in, rng):
    import torch
    import srsgpu_phy as s
    n = len(sfs)
    size = 14 * 12 * nof_prb
    grids = [_sync_grid(nof_prb, cell_id, sf, nports, rng, flat=average) for sf in sfs]
    c = s.Chest(nof_prb, cell_id, max_grids=n, nof_ports=nports)
    c.set_filter(list(filt))
    alg = {"refs": 0, "pss": 1, "empty": 2}[noise_alg]
    c.set_cfg(average_subframe=average, noise_alg=alg, smooth_filter_auto=filt_auto, rsrp_neighbour=True,
              cfo_enable=True, cfo_mask=0x3ff & ~(1 << 3))
    d_g = torch.from_numpy(np.stack(grids).reshape(-1)).cuda()
    d_ce = torch.zeros(nports * n * size, dtype=torch.complex64, device="cuda")
    d_n = torch.full((n * nports,), noise_in, dtype=torch.float32, device="cuda")
    d_m = torch.full((n * nports * 4,), -7.0, dtype=torch.float32, device="cuda")
    assert c.estimate_meas_dev(sfs, d_g.data_ptr(), size, d_ce.data_ptr(), d_n.data_ptr(), d_m.data_ptr()) == 0
    torch.cuda.synchronize()
    ce = d_ce.cpu().numpy().reshape(n, nports, -1)
    nz = d_n.cpu().numpy().reshape(n, nports)
    me = d_m.cpu().numpy().reshape(n, nports, 4)
    c.close()
    for i, sf in enumerate(sfs):
        g64 = grids[i].astype(np.complex128)
        for p in range(nports):
            ref_ce, ref_n = co.estimate_full(g64, nof_prb, cell_id, sf, filt, p, average, noise_alg, filt_auto,
                                             float(np.float32(noise_in)), nports)
            scale = np.max(np.abs(ref_ce))
            where = (nof_prb, sf, p, average, noise_alg, filt_auto, len(filt))
            assert np.max(np.abs(ce[i, p] - ref_ce)) / scale < 1e-4, where
            assert abs(nz[i, p] - ref_n) <= 1e-4 * abs(ref_n) + 1e-9, (where, nz[i, p], ref_n)
            rsrp, rssi, corr, cfo = co.measurements(g64, nof_prb, cell_id, sf, p, s.symbol_sz_of(nof_prb))
            assert abs(me[i, p, 0] - rsrp) <= 1e-4 * rsrp and abs(me[i, p, 1] - rssi) <= 1e-4 * rssi, where
            assert abs(me[i, p, 2] - corr) <= 1e-4 * rsrp, where
            if sf == 3:  # CFO masked off for subframe 3: left untouched
                assert me[i, p, 3] == -7.0
            else:
                assert abs(me[i, p, 3] - cfo) <= 1e-5 + 1e-4 * abs(cfo), (where, me[i, p, 3], cfo)


@pytest.mark.gpu
@pytest.mark.parametrize("nof_prb,cell_id,nports", [(6, 3, 1), (6, 10, 2), (25, 1, 1), (25, 2, 2),
                                                    (100, 7, 1), (100, 500, 2)])
def test_chest_srsue_default_gpu_vs_oracle(nof_prb, cell_id, nports):
    """srsUE's phch_worker configuration (srsue/src/main.cc:287-301, phch_worker.cc:148-150,
    553-565): average_subframe, Gaussian filter order 4 / std dev 1, REFS noise, neighbour RSRP,
    CFO estimation on every subframe (cfo_ref_mask 1023; subframe 3 masked here to check the mask)"""
    rng = np.random.default_rng(nof_prb * 3 + cell_id)
    _run_modes(nof_prb, cell_id, nports, list(range(10)), co.gauss_filter(4, 1.0), True, "refs", False, 0.0, rng)


@pytest.mark.gpu
@pytest.mark.parametrize("average", [False, True])
@pytest.mark.parametrize("noise_alg", ["refs", "pss", "empty"])
@pytest.mark.parametrize("filt_auto", [False, True])
def test_chest_modes_gpu_vs_oracle(average, noise_alg, filt_auto):
    """every combination of average_subframe x noise algorithm x smooth_filter_auto, 2 ports, with
    subframes 0 / 5 (PSS / EMPTY update the noise) and others (the caller's value stays)"""
    rng = np.random.default_rng(int(average) * 100 + len(noise_alg) * 10 + int(filt_auto))
    _run_modes(25, 11, 2, [0, 3, 5, 8], (0.1, 0.8, 0.1), average, noise_alg, filt_auto, 0.004, rng)


@pytest.mark.gpu
@pytest.mark.parametrize("filt", [(), (0.0, 1.0, 0.0), (0.05, 0.2, 0.5, 0.2, 0.05)])
def test_chest_average_filters_gpu_vs_oracle(filt):
    """average_subframe without smoothing interpolates the reference's raw pilot buffer
    (chest_dl.c:619-621): the quirk is reproduced"""
    rng = np.random.default_rng(len(filt))
    _run_modes(50, 301, 1, [1, 5], filt, True, "refs", False, 0.0, rng)


def test_oracle_average_subframe_property():
    """averaging is exact on a channel constant in time (chest_test_dl.c-style check)"""
    rng = np.random.default_rng(2)
    for nof_prb, cid in ((25, 1), (100, 8)):
        for port in (0, 1):
            j = np.arange(12 * nof_prb)
            xx = np.cos(2 * np.pi * j / nof_prb / 12)
            h = np.tile((3 + xx) * np.exp(1j * xx), 14)
            x = crs_grid(nof_prb, cid, 3, rng, port)
            ce, _ = co.estimate_full(x * h, nof_prb, cid, 3, co.gauss_filter(4, 1.0), port, average=True)
            assert np.mean(np.abs(x - (x * h) / ce)) < 1e-3
