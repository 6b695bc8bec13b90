"""Channel estimation: the reference's own chest_dl.c (oracle/_ref/ref_front), the numpy restatement
oracle/chest_oracle.py, and the GPU estimator (chest_kernels.hip).

Parity chain:
  - tests/golden/chest_golden.npz holds CE grids, noise, RSRP, RSSI, RSRP correlation and CFO recorded from
    the reference's chest_dl.c (compiled where it lies, tests/golden/make_chest_golden.py) in srsUE's
    configurations (average_subframe + Gaussian filter, per-symbol interpolation, REFS / PSS / EMPTY noise,
    smooth_filter_auto, no smoothing), 1-2 ports x 1-2 rx antennas, 6-100 PRB, one estimator object per
    subframe sequence (noise state carried as in srsUE);
  - CPU: the oracle equals the golden data (and, in the build container, fresh runs of the reference) within
    1e-4 relative; CRS generation and pilot extraction equal refsignal_dl.c bit for bit;
  - GPU: the estimator equals the golden data within 1e-4 relative (float stage, SURVEY.md 8(a) tolerance),
    and the oracle on further random cases.
"""
import ctypes
import os
import sys

import numpy as np
import pytest

import json

from srsgpu_testlib import Ref, have_ref, have_ref_front, ref_front_chest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import chest_oracle as co  # noqa: E402
from chest_synth import crs_grid, smooth_channel, sync_grid  # noqa: E402

f32 = ctypes.POINTER(ctypes.c_float)


@pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built (build container only)")
def test_crs_and_pilot_extraction_vs_reference():
    L = Ref().lib
    L.ref_crs_pilots.argtypes = [ctypes.c_uint32] * 3 + [f32]
    L.ref_crs_get_sf.argtypes = [ctypes.c_uint32] * 3 + [f32, f32]
    L.ref_crs_pilots23.argtypes = [ctypes.c_uint32] * 3 + [f32]
    rng = np.random.default_rng(0)
    for nof_prb, cid in ((100, 1), (6, 0), (25, 503), (50, 17), (75, 254)):
        for sf in (0, 3, 9):
            out = np.zeros(4 * 2 * nof_prb, np.complex64)
            assert L.ref_crs_pilots(nof_prb, cid, sf, out.ctypes.data_as(f32)) == 0
            assert np.allclose(out.reshape(4, -1), co.crs_pilots(nof_prb, cid, sf), atol=1e-7)
            out = np.zeros(2 * 2 * nof_prb, np.complex64)
            assert L.ref_crs_pilots23(nof_prb, cid, sf, out.ctypes.data_as(f32)) == 0
            assert np.allclose(out.reshape(2, -1), co.crs_pilots(nof_prb, cid, sf, port=2), atol=1e-7)
        grid = (rng.standard_normal(14 * 12 * nof_prb) + 1j * rng.standard_normal(14 * 12 * nof_prb)).astype(np.complex64)
        for port in (0, 1, 2, 3):
            sy = co.syms(port)
            got = np.zeros(len(sy) * 2 * nof_prb, np.complex64)
            assert L.ref_crs_get_sf(nof_prb, cid, port, grid.ctypes.data_as(f32), got.ctypes.data_as(f32)) == 0
            g = grid.reshape(14, -1)
            exp = np.stack([g[s, co.fidx(cid, l, port) + 6 * np.arange(2 * nof_prb)] for l, s in enumerate(sy)])
            assert (got.reshape(len(sy), -1) == exp).all(), port


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


def _run_modes(nof_prb, cell_id, nports, sfs, filt, average, noise_alg, filt_auto, noise_in, rng):
    import torch
    import srsgpu_phy as s
    n = len(sfs)
    size = 14 * 12 * nof_prb
    grids = [sync_grid(nof_prb, cell_id, sf, nports, rng, flat=average) for sf in sfs]
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
                                                    (100, 7, 1), (100, 500, 2), (25, 4, 4), (100, 9, 4)])
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
@pytest.mark.parametrize("average", [False, True])
@pytest.mark.parametrize("noise_alg", ["refs", "pss", "empty"])
def test_chest_four_ports_gpu_vs_oracle(average, noise_alg):
    """4 CRS ports: ports 2 / 3 from symbols 1 and 8 (2-symbol noise, averaging and time
    interpolation, chest_dl.c:285-299, 427-431, 538-550), with smoothing and smooth_filter_auto"""
    rng = np.random.default_rng(int(average) * 10 + len(noise_alg))
    _run_modes(50, 23, 4, [0, 2, 5, 9], (0.1, 0.8, 0.1), average, noise_alg, False, 0.004, rng)
    _run_modes(15, 200, 4, [1, 5], (), average, noise_alg, True, 0.004, rng)


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


# ------------------------------------------------------------------ reference golden data ----

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "chest_golden.npz")
ALG = ("refs", "pss", "empty")


def _gold():
    z = np.load(GOLD)
    return z, json.loads(bytes(z["manifest"]).decode())


def _case_filter(c):
    return co.gauss_filter(*c["gauss"]) if c["gauss"] else tuple(c["filt"])


def _check_against(c, got_ce, got_noise, got_meas, z, who):
    """got_*: [sf][rx][port] like the golden arrays (meas: [..., 4] rsrp, rssi, rsrp_corr, cfo)"""
    n = c["name"]
    ce, noise = z[n + "_ce"], z[n + "_noise"]
    for i, sf in enumerate(c["sfs"]):
        for a in range(c["nrx"]):
            for p in range(c["nports"]):
                where = (who, n, sf, a, p)
                scale = np.max(np.abs(ce[i, a, p]))
                assert np.max(np.abs(got_ce[i][a][p] - ce[i, a, p])) / scale < 1e-4, where
                rn = float(noise[i, a, p])
                assert abs(got_noise[i][a][p] - rn) <= 1e-4 * abs(rn) + 1e-9, (where, got_noise[i][a][p], rn)
                if got_meas is None:
                    continue
                rsrp, rssi, corr, cfo = (float(z[n + k][i, a, p]) for k in ("_rsrp", "_rssi", "_rsrp_corr", "_cfo"))
                m = got_meas[i][a][p]
                assert abs(m[0] - rsrp) <= 1e-4 * rsrp and abs(m[1] - rssi) <= 1e-4 * rssi, where
                assert abs(m[2] - corr) <= 1e-4 * rsrp, where
                assert abs(m[3] - cfo) <= 1e-5 + 1e-4 * abs(cfo), (where, m[3], cfo)


def test_oracle_vs_reference_golden():
    """the numpy restatement equals the reference's chest_dl.c on the recorded cases"""
    z, man = _gold()
    for c in man:
        g = z[c["name"] + "_grid"]
        nb = z[c["name"] + "_noise_before"]
        f = _case_filter(c)
        got_ce, got_n, got_m = [], [], []
        for i, sf in enumerate(c["sfs"]):
            rows_ce, rows_n, rows_m = [], [], []
            for a in range(c["nrx"]):
                pce, pn, pm = [], [], []
                for p in range(c["nports"]):
                    g64 = g[i, a].astype(np.complex128)
                    e, nz = co.estimate_full(g64, c["nof_prb"], c["cell_id"], sf, f, p, c["average"],
                                             ALG[c["noise_alg"]], c["smooth_auto"], float(nb[i, a, p]), c["nports"])
                    pce.append(e)
                    pn.append(nz)
                    pm.append(co.measurements(g64, c["nof_prb"], c["cell_id"], sf, p, symbol_sz_of(c["nof_prb"])))
                rows_ce.append(pce)
                rows_n.append(pn)
                rows_m.append(pm)
            got_ce.append(rows_ce)
            got_n.append(rows_n)
            got_m.append(rows_m)
        _check_against(c, got_ce, got_n, got_m, z, "oracle")


def symbol_sz_of(nof_prb):
    return next(sz for lim, sz in ((6, 128), (15, 256), (25, 384), (50, 768), (75, 1024), (110, 1536)) if nof_prb <= lim)


def test_golden_getters_follow_the_per_port_values():
    """srslte_chest_dl_get_noise_estimate / get_rsrp as recorded equal their formulas (chest_dl.c:741-846)
    over the recorded per-(rx, port) values: what the GPU queue computes from its per-grid outputs"""
    z, man = _gold()
    for c in man:
        n = c["name"]
        for i in range(len(c["sfs"])):
            nz = z[n + "_noise"][i].astype(np.float32)
            acc = np.float32(0)
            for a in range(c["nrx"]):
                s = np.float32(0)
                for p in range(c["nports"]):
                    s = np.float32(s + nz[a, p])
                acc = np.float32(acc + s / np.float32(c["nports"]))
            assert np.float32(acc / np.float32(c["nrx"])) == z[n + "_getters"][i][0], (n, i)


@pytest.mark.skipif(not have_ref_front(), reason="oracle/_ref/ref_front not built (build container only)")
@pytest.mark.parametrize("nof_prb,cell_id,nports,nrx,average,alg,auto", [
    (25, 11, 2, 2, False, 0, False), (50, 301, 1, 1, True, 1, False), (6, 3, 1, 2, False, 2, False),
    (75, 40, 2, 1, True, 0, True), (100, 7, 1, 1, False, 1, False), (25, 19, 4, 2, False, 0, False),
    (50, 6, 4, 1, True, 1, False), (15, 100, 4, 2, True, 0, True)])
def test_oracle_vs_reference_live(nof_prb, cell_id, nports, nrx, average, alg, auto):
    """fresh random cells through the reference's chest_dl.c and the oracle"""
    rng = np.random.default_rng(nof_prb * 7 + cell_id)
    sfs = [0, 1, 5, 6] if nof_prb < 75 else [4, 5]
    grids = [[sync_grid(nof_prb, cell_id, sf, nports, rng, flat=average) for _ in range(nrx)] for sf in sfs]
    gauss = (4, 1.0) if average else None
    filt = () if average else (0.1, 0.8, 0.1)
    res = ref_front_chest(nof_prb, cell_id, nports, nrx, sfs, grids, filt=filt, gauss=gauss, smooth_auto=auto,
                          average=average, noise_alg=alg, noise_init=0.003)
    f = co.gauss_filter(*gauss) if gauss else filt
    for i, sf in enumerate(sfs):
        for a in range(nrx):
            for p in range(nports):
                g64 = grids[i][a].astype(np.complex128)
                e, nz = co.estimate_full(g64, nof_prb, cell_id, sf, f, p, average, ALG[alg], auto,
                                         float(res[i]["noise_before"][a, p]), nports)
                ref_ce = res[i]["ce"][a, p]
                assert np.max(np.abs(e - ref_ce)) / np.max(np.abs(ref_ce)) < 1e-4, (sf, a, p)
                rn = float(res[i]["noise"][a, p])
                assert abs(nz - rn) <= 1e-4 * abs(rn) + 1e-9, (sf, a, p, nz, rn)


@pytest.mark.gpu
def test_chest_gpu_vs_reference_golden():
    """the GPU estimator against the reference's chest_dl.c recordings: one call per case (all subframes and
    rx antennas as separate grids), noise in/out from the recorded state before each subframe"""
    import torch
    import srsgpu_phy as s
    z, man = _gold()
    for c in man:
        n, nprb, npt, nrx = c["name"], c["nof_prb"], c["nports"], c["nrx"]
        size = 14 * 12 * nprb
        nsf = len(c["sfs"])
        grids = z[n + "_grid"].reshape(nsf * nrx, size)
        ch = s.Chest(nprb, c["cell_id"], max_grids=nsf * nrx, nof_ports=npt)
        if c["gauss"]:
            ch.set_filter_gauss(int(c["gauss"][0]), float(c["gauss"][1]))
        else:
            ch.set_filter(list(c["filt"]))
        ch.set_cfg(average_subframe=c["average"], noise_alg=c["noise_alg"], smooth_filter_auto=c["smooth_auto"],
                   rsrp_neighbour=True, cfo_enable=True, cfo_mask=0x3FF)
        d_g = torch.from_numpy(np.ascontiguousarray(grids).reshape(-1)).cuda()
        d_ce = torch.zeros(npt * nsf * nrx * size, dtype=torch.complex64, device="cuda")
        d_n = torch.from_numpy(z[n + "_noise_before"].reshape(-1).astype(np.float32)).cuda()
        d_m = torch.zeros(nsf * nrx * npt * 4, dtype=torch.float32, device="cuda")
        sfi = [sf for sf in c["sfs"] for _ in range(nrx)]
        assert ch.estimate_meas_dev(sfi, d_g.data_ptr(), size, d_ce.data_ptr(), d_n.data_ptr(), d_m.data_ptr()) == 0
        torch.cuda.synchronize()
        ce = d_ce.cpu().numpy().reshape(nsf, nrx, npt, size)
        nz = d_n.cpu().numpy().reshape(nsf, nrx, npt)
        me = d_m.cpu().numpy().reshape(nsf, nrx, npt, 4)
        ch.close()
        _check_against(c, ce, nz, me, z, "gpu")
