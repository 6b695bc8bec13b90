"""What srsUE's PHY worker reads after every subframe: the
estimator's measurements (srslte_chest_dl_get_cfo / _snr / _rsrp / _rsrq / _rssi / _rsrp_neighbour,
chest_dl.c:737-846; phch_worker.cc:226-241, 301, 313, 1618-1628) and the TM3 / TM4 feedback of
phch_worker::compute_ri (:522-540: srslte_ue_dl_ri_select's condition number and rank,
srslte_ue_dl_ri_pmi_select's rank / PMI / SINR, ue_dl.c:684-764, over precoding.c:2335-2930).

Pinned to the reference (oracle/_ref/ref_front ue_dl) on synthetic two-port cells
(tests/golden/make_feedback_golden.py): the CPU oracle restatement (oracle/pdsch_oracle.c orc_feedback)
equals the reference on the reference's own estimates — the one-layer SINRs and the condition number
exactly, the two-layer SINRs within the _mm256_rcp_ps tolerance; on the GPU, srsgpu_pdsch_feedback_dev
equals the oracle bit for bit on the GPU's estimates, and the queue's per-subframe results
(srsgpu_rxq_ue_dl_t.meas / .fb, from the time-domain samples) equal the reference's within 1e-4
(two-layer SINR: 3e-3), rank and PMI exactly (unless the reference's own choice is within that
tolerance of a tie)."""
import ctypes
import json
import os
import sys

import numpy as np
import pytest

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, "oracle"))
import ofdm_oracle as oo  # noqa: E402

GOLD = os.path.join(REPO, "tests", "golden", "feedback_golden.npz")
TOL, TOL_2L = 1e-4, 3e-3


def _load():
    z = np.load(GOLD)
    return z, json.loads(bytes(z["manifest"]).decode())


def orc_feedback(oracle, ce, noise, flags, nrx):
    """oracle/pdsch_oracle.c orc_feedback on estimate planes ce[port][rx][n] (2 ports)"""
    L = oracle.lib
    fp = ctypes.POINTER(ctypes.c_float)
    L.orc_feedback.argtypes = [fp, fp, fp, fp, ctypes.c_uint32, ctypes.c_float, ctypes.c_uint32, ctypes.c_int,
                               ctypes.c_int, fp, ctypes.POINTER(ctypes.c_int32), fp]
    pl = [[np.ascontiguousarray(ce[p][a], np.complex64) if a < nrx else None for a in range(2)] for p in range(2)]
    ptr = lambda v: v.ctypes.data_as(fp) if v is not None else None  # noqa: E731
    cn = np.zeros(1, np.float32)
    oi = np.zeros(7, np.int32)
    sinr = np.zeros(8, np.float32)
    n = pl[0][0].size
    assert L.orc_feedback(ptr(pl[0][0]), ptr(pl[1][0]), ptr(pl[0][1]), ptr(pl[1][1]), n, noise, flags, 2, nrx,
                          ptr(cn), oi.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), ptr(sinr)) == 0
    return dict(cn=float(cn[0]), ri_tm3=int(oi[0]), ret_cn=int(oi[1]), ri=int(oi[2]), pmi=int(oi[3]),
                pmi_l=[int(oi[4]), int(oi[5])], ret_pmi=int(oi[6]), sinr=sinr.reshape(2, 4))


def _choice_margin(sinr, nrx):
    """relative distance of the reference's rank / PMI decisions from a tie: the per-layer best codebook
    against the runner-up, and the rank comparison of ue_dl.c:701 (sinr * L^2 against best + 0.1)"""
    m = np.inf
    for L in range(min(nrx, 2)):
        s = np.sort(sinr[L][:4 if L == 0 else 2])[::-1]
        m = min(m, (s[0] - s[1]) / max(abs(s[0]), 1e-30))
    if nrx == 2:
        a, b = sinr[0].max(), 4.0 * sinr[1][:2].max()
        m = min(m, abs(b - (a + 0.1)) / max(abs(a), 1e-30))
    return m


def _close(a, b, tol):
    return abs(a - b) <= tol * max(abs(a), abs(b), 1e-12)


def _check_fb(got, ref, nrx, tag):
    assert got["ret_cn"] == ref["ret_cn"] and got["ret_pmi"] == ref["ret_pmi"], tag
    if ref["ret_cn"] == 0:
        assert _close(got["cn"], ref["cn"], TOL), (tag, got["cn"], ref["cn"])
        if abs(ref["cn"] - 17.0) > 1e-3:
            assert got["ri_tm3"] == ref["ri_tm3"], tag
    s, r = np.asarray(got["sinr"]), np.asarray(ref["sinr"])
    for c in range(4):
        assert _close(s[0][c], r[0][c], TOL), (tag, c, s[0], r[0])
    if nrx == 2:
        for c in range(2):
            assert _close(s[1][c], r[1][c], TOL_2L), (tag, c, s[1], r[1])
    else:
        assert np.all(np.isneginf(s[1])) and np.all(np.isneginf(r[1])), tag
    if _choice_margin(r, nrx) > TOL_2L:
        assert (got["ri"], got["pmi"], list(got["pmi_l"])) == (ref["ri"], ref["pmi"], list(ref["pmi_l"])), (tag, got, ref)


@pytest.mark.skipif(not os.path.exists(os.path.join(REPO, "oracle", "_ref", "ref_front")),
                    reason="needs the reference build (this container only)")
def test_oracle_feedback_equals_reference(oracle):
    """orc_feedback on the reference's own estimates: one-layer SINR and condition number bit-exact,
    two-layer SINR within the rcpps tolerance, rank / PMI equal; the golden fixture equals a live run"""
    from srsgpu_testlib import ref_front_ue_dl
    z, man = _load()
    for name, m in man.items():
        xs = z[name + "_x"]
        grids = [[oo.rx_sf(xs[i, a], m["nof_prb"], m["N"]).reshape(-1).astype(np.complex64) for a in range(m["nrx"])]
                 for i in range(len(m["ttis"]))]
        res = ref_front_ue_dl(m["nof_prb"], m["cell_id"], 2, m["nrx"], 0, 2, m["nof_prb"], m["rnti"], 3, m["ttis"],
                              grids, gauss=m["gauss"], filt=None if m["gauss"] else (0.1, 0.8, 0.1),
                              average=m["average"], rsrp_neighbour=m["rsrp_neighbour"],
                              cfo_enable=m["cfo_enable"], cfo_mask=m["cfo_mask"])
        for i, r in enumerate(res):
            assert np.array_equal(r["getters"], z[name + "_getters"][i]), (name, i)
            assert r["cn"] == z[name + "_cn"][i] and r["ri"] == z[name + "_ri"][i] and r["pmi"] == z[name + "_pmi"][i]
            o = orc_feedback(oracle, r["ce"], float(r["getters"][0]), 3, m["nrx"])
            assert o["ret_cn"] == r["ret_cn"] and o["ret_pmi"] == r["ret_pmi"], (name, i)
            assert o["cn"] == r["cn"] and o["ri_tm3"] == r["ri_tm3"], (name, i, o["cn"], r["cn"])
            assert np.array_equal(o["sinr"][0], r["sinr"][0]), (name, i, o["sinr"][0], r["sinr"][0])
            _check_fb(o, r, m["nrx"], (name, i))


def _gpu_estimates(s, torch, z, name, m):
    """GPU OFDM + estimation of a case's subframes with its estimator settings -> (d_ce, ce host
    [sf][port][rx][n], noise per subframe as srslte_chest_dl_get_noise_estimate)"""
    nof_prb, N, nrx = m["nof_prb"], m["N"], m["nrx"]
    nsf, n = len(m["ttis"]), 14 * 12 * nof_prb
    xs = np.ascontiguousarray(z[name + "_x"])
    ofdm = s.OfdmRx(nof_prb, N)
    ch = s.Chest(nof_prb, m["cell_id"], max_grids=nsf * nrx, nof_ports=2)
    ch.set_cfg(average_subframe=m["average"], rsrp_neighbour=m["rsrp_neighbour"], cfo_enable=m["cfo_enable"],
               cfo_mask=m["cfo_mask"])
    if m["gauss"]:
        ch.set_filter_gauss(*m["gauss"])
    d_x = torch.from_numpy(xs.reshape(-1)).cuda()
    d_grid = torch.zeros(nsf * nrx * n, dtype=torch.complex64, device="cuda")
    d_ce = torch.zeros(nsf * nrx * 2 * n, dtype=torch.complex64, device="cuda")
    d_noise = torch.zeros(nsf * nrx * 2, dtype=torch.float32, device="cuda")
    assert ofdm.rx_dev(nsf * nrx, d_x.data_ptr(), 15 * N, d_grid.data_ptr(), n) == 0
    sfi = [t % 10 for t in m["ttis"] for _ in range(nrx)]
    assert ch.estimate_meas_dev(sfi, d_grid.data_ptr(), n, d_ce.data_ptr(), d_noise.data_ptr()) == 0
    torch.cuda.synchronize()
    ce = d_ce.cpu().numpy().reshape(nsf, nrx, 2, n).transpose(0, 2, 1, 3)  # [sf][port][rx][n]
    nz = d_noise.cpu().numpy().reshape(nsf, nrx, 2)
    noise = []
    for i in range(nsf):  # chest_dl.c:741-750 in float
        acc = np.float32(0)
        for a in range(nrx):
            acc = np.float32(acc + np.float32(np.float32(nz[i, a, 0] + nz[i, a, 1]) / np.float32(2)))
        noise.append(float(np.float32(acc / np.float32(nrx))))
    ofdm.close()
    ch.close()
    return d_ce, ce, noise


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["tm4_25_2x2", "tm4_6_2x1", "tm3_50_2x2"])
def test_gpu_feedback_dev(oracle, name):
    """srsgpu_pdsch_feedback_dev on the GPU's estimates equals the oracle on the same estimates bit for
    bit (condition number up to the device log10f), and the reference within the tolerances"""
    import torch
    import srsgpu_phy as s
    z, man = _load()
    m = man[name]
    nsf, nrx, n = len(m["ttis"]), m["nrx"], 14 * 12 * m["nof_prb"]
    d_ce, ce, noise = _gpu_estimates(s, torch, z, name, m)
    pd = s.Pdsch(m["nof_prb"], m["cell_id"], nof_ports=2, nof_rx_ant=nrx, max_sf=nsf)
    d_out = torch.zeros(nsf * ctypes.sizeof(s.srsgpu_feedback_t), dtype=torch.uint8, device="cuda")
    items = [(i * nrx * 2 * n, noise[i], 3) for i in range(nsf)]
    assert pd.feedback_dev(items, d_ce.data_ptr(), n, d_out.data_ptr()) == 0
    torch.cuda.synchronize()
    fb = s.Pdsch.parse_feedback(d_out.cpu().numpy().tobytes(), nsf)
    for i in range(nsf):
        g = dict(cn=fb[i].cn, ri_tm3=fb[i].ri_tm3, ret_cn=fb[i].ret_cn, ri=fb[i].ri, pmi=fb[i].pmi,
                 pmi_l=list(fb[i].pmi_l), ret_pmi=fb[i].ret_pmi, sinr=fb[i].sinr_array())
        o = orc_feedback(oracle, ce[i], noise[i], 3, nrx)
        assert np.array_equal(g["sinr"], o["sinr"]), (name, i, g["sinr"], o["sinr"])
        assert _close(g["cn"], o["cn"], 1e-6) and (g["ri"], g["pmi"], g["pmi_l"]) == (o["ri"], o["pmi"], o["pmi_l"])
        ref = {k: z["%s_%s" % (name, k)][i] for k in ("cn", "ri_tm3", "ret_cn", "ri", "pmi", "ret_pmi", "sinr", "pmi_l")}
        ref = {k: (v.tolist() if k == "pmi_l" else v) for k, v in ref.items()}
        _check_fb(g, ref, nrx, (name, i))
    pd.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["tm4_25_2x2", "tm4_6_2x1", "tm3_50_2x2"])
def test_queue_returns_worker_reads(name):
    """one srsgpu_rxq_ue_dl_t per subframe through the queue (time-domain samples in, srsUE's or the init
    estimator settings, feedback on): noise, the six getters and the feedback equal the reference's; the
    CFO carries over the subframes that do not estimate it, across batches too"""
    import torch  # noqa: F401
    import srsgpu_phy as s
    z, man = _load()
    m = man[name]
    nsf, nrx = len(m["ttis"]), m["nrx"]
    xs = np.ascontiguousarray(z[name + "_x"])
    q = s.RxQueue(m["nof_prb"], m["cell_id"], m["N"], nof_ports=2, nof_rx_ant=nrx, nof_softbuffers=2 * nsf,
                  max_batch=2, max_wait_us=100000)
    q.set_chest_cfg(average_subframe=m["average"], rsrp_neighbour=m["rsrp_neighbour"], cfo_enable=m["cfo_enable"],
                    cfo_mask=m["cfo_mask"], gauss=m["gauss"])
    outs = [np.zeros(16, np.uint8) for _ in range(nsf)]
    items = [q.ue_item([xs[i, a] for a in range(nrx)], t, m["rnti"], [outs[i]], tm=3, softbuffer=(2 * i, 2 * i + 1),
                       feedback=s.FEEDBACK_CN | s.FEEDBACK_PMI) for i, t in enumerate(m["ttis"])]
    tickets = [q.submit_ue_dl(u) for u in items]  # batches of 2: the carried values cross batches
    q.flush()
    assert all(q.wait(t) == 0 for t in tickets)
    for i, u in enumerate(items):
        gref = z[name + "_getters"][i]  # noise snr rssi rsrq rsrp rsrp_neighbour cfo
        assert _close(u.noise, gref[0], TOL), (name, i, u.noise, gref[0])
        got = u.meas.values()  # cfo snr rsrp rsrq rssi rsrp_neighbour
        want = [gref[6], gref[1], gref[4], gref[3], gref[2], gref[5]]
        for k, (a, b) in enumerate(zip(got, want)):
            assert abs(a - b) <= TOL * max(abs(a), abs(b)) + (1e-6 if k == 0 else 0.0), (name, i, k, got, want)
        g = dict(cn=u.fb.cn, ri_tm3=u.fb.ri_tm3, ret_cn=u.fb.ret_cn, ri=u.fb.ri, pmi=u.fb.pmi, pmi_l=list(u.fb.pmi_l),
                 ret_pmi=u.fb.ret_pmi, sinr=u.fb.sinr_array())
        ref = {k: z["%s_%s" % (name, k)][i] for k in ("cn", "ri_tm3", "ret_cn", "ri", "pmi", "ret_pmi", "sinr", "pmi_l")}
        ref = {k: (v.tolist() if k == "pmi_l" else v) for k, v in ref.items()}
        _check_fb(g, ref, nrx, (name, i))
    q.close()
