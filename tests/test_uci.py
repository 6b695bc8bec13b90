"""UCI multiplexed on the PUSCH (SURVEY §8(f) rank 3 widening): HARQ-ACK, RI
and CQI decoded around the UL-SCH data as srslte_pusch_decode does it (pusch.c:626-657, sch.c:892-985,
uci.c:270-790).
  - CPU: the oracle restatement (oracle/pdsch_oracle.c orc_ulsch_uci) equals golden receptions recorded
    from the reference build (tests/golden/make_uci_golden.py) and, in the build container, fresh
    reference runs on random configurations;
  - GPU: srsgpu_ulsch_uci_decode_dev equals the golden receptions (ACK / RI / cqi_ack / CQI bits, the
    deinterleaved g bits, return value, data) and the oracle on a mixed batch in one call."""
import json
import os

import numpy as np
import pytest

from srsgpu_testlib import PdschOracle, Ref, have_ref, orc_ulsch_uci, uci_case, uci_rx

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def ugold():
    z = np.load(os.path.join(HERE, "golden", "uci_golden.npz"))
    return z, json.loads(bytes(z["manifest"]))


def test_oracle_vs_golden(oracle, ugold):
    z, man = ugold
    assert len(man) == 10
    for u in man:
        k = u["key"]
        r, out, g, qp = orc_ulsch_uci(oracle, u, z[k + "_q"], z[k + "_c"])
        assert r == 0, k
        assert (out == z[k + "_out"]).all(), (k, out, z[k + "_out"])
        assert (g == z[k + "_g"]).all(), k


@pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built")
def test_oracle_vs_live_reference(oracle):
    ref = Ref()
    po = PdschOracle(oracle)
    rng = np.random.default_rng(77)
    checked = 0
    for n in range(40):
        Qm = [2, 4, 6][n % 3]
        prb = int(rng.choice([2, 5, 9, 16, 25, 40]))
        O = (int(rng.integers(0, 3)), int(rng.integers(0, 3)), int(rng.choice([0, 3, 8, 11, 12, 25, 60])))
        tbs = int(rng.choice([0, 328, 1032, 2600])) if O != (0, 0, 0) else 1032
        I_off = (int(rng.integers(0, 15)), int(rng.integers(0, 13)), int(rng.integers(2, 16)))
        u = uci_case(tbs, Qm, prb, nof_symb=int(rng.choice([11, 12])), O=O, I_off=I_off,
                     ack=tuple(int(v) for v in rng.integers(0, 2, 2)), ri=int(rng.integers(0, 2)),
                     cqi=tuple(int(v) for v in rng.integers(0, 2, O[2])))
        if tbs and u["nof_bits"] < 3 * (tbs + 24):
            continue
        zq, zc = np.zeros(u["nof_bits"], np.int16), np.zeros(u["nof_bits"], np.uint8)
        r0, _o, _g, qp = orc_ulsch_uci(oracle, u, zq, zc)
        if r0 or (qp[0] + qp[1]) * Qm > 12 * 288:  # beyond the reference's ack_ri_bits array (sch.h:70)
            continue
        data = rng.integers(0, 256, tbs // 8 + 8).astype(np.uint8)
        qb = ref.uci_encode(u, data)
        c = po.sequence(int(rng.integers(1, 2 ** 30)), u["nof_bits"])
        qs = uci_rx(rng, qb, c, sigma=float(rng.choice([5, 30])))
        if tbs:
            ref.sb_reset(0)
        r2, out2, g2, qp = orc_ulsch_uci(oracle, u, qs, c)
        r, out, g, _d, _noi, _crc = ref.uci_decode(0, u, qs, c)
        assert (out == out2).all() and (g == g2).all(), (n, u["O"], out, out2)
        checked += 1
    assert checked >= 12


def _gpu_run(s, torch, cases, rng_ok=True):
    """cases: [(u, q_scrambled, c)] -> per case (ret, noi, out[4 + O_cqi], g, data) from one call"""
    dl = s.Dlsch(max_cb=8, nof_softbuffers=len(cases))
    tbs_list, uci_list, qs, cs, offs, doff = [], [], [], [], 0, 0
    for i, (u, q, c) in enumerate(cases):
        tbs_list.append(dict(tbs=u["tbs"], rv=u["rv"], Qm=u["Qm"], nof_bits=u["nof_bits"], nof_symb=u["nof_symb"],
                             softbuffer=i, q_offset=offs, data_offset=doff))
        uci_list.append(dict(O=u["O"], I_off=u["I_off"], M_sc=u["M_sc"], M_sc_init=u["M_sc_init"], c_offset=offs))
        qs.append(q)
        cs.append(c)
        offs += (u["nof_bits"] + 63) // 64 * 64
        doff += s.dlsch_data_len(max(u["tbs"], 8)) + 2
    dl.reset_range(0, len(cases))
    d_q = torch.zeros(offs, dtype=torch.int16, device="cuda")
    d_c = torch.zeros(offs, dtype=torch.uint8, device="cuda")
    for t, q, c in zip(tbs_list, qs, cs):
        d_q[t["q_offset"]:t["q_offset"] + q.size] = torch.from_numpy(q)
        d_c[t["q_offset"]:t["q_offset"] + c.size] = torch.from_numpy(c)
    d_g = torch.full((offs,), 7777, dtype=torch.int16, device="cuda")
    d_data = torch.zeros(doff, dtype=torch.uint8, device="cuda")
    d_ret = torch.full((len(cases),), -9, dtype=torch.int32, device="cuda")
    d_noi = torch.zeros(len(cases), dtype=torch.int32, device="cuda")
    res = (s.srsgpu_uci_result_t * len(cases))()
    d_res = torch.zeros(len(cases) * ctypes_sizeof(s), dtype=torch.uint8, device="cuda")
    assert dl.ulsch_uci_decode_dev(tbs_list, uci_list, d_q.data_ptr(), d_c.data_ptr(), d_g.data_ptr(),
                                   d_data.data_ptr(), 8, d_ret.data_ptr(), d_noi.data_ptr(), d_res.data_ptr()) == 0
    torch.cuda.synchronize()
    raw = d_res.cpu().numpy().tobytes()
    import ctypes
    ctypes.memmove(res, raw, len(raw))
    g, data, ret, noi = d_g.cpu().numpy(), d_data.cpu().numpy(), d_ret.cpu().numpy(), d_noi.cpu().numpy()
    outs = []
    for i, (u, _q, _c) in enumerate(cases):
        r = res[i]
        out = np.array([r.ack[0], r.ack[1], r.ri, r.cqi_ack] + [r.cqi[k] for k in range(u["O"][2])], np.uint8)
        t = tbs_list[i]
        outs.append((int(ret[i]), int(noi[i]), out, g[t["q_offset"]:t["q_offset"] + u["nof_bits"]],
                     data[t["data_offset"]:t["data_offset"] + u["tbs"] // 8], (r.Q_ack, r.Q_ri, r.Q_cqi)))
    dl.close()
    return outs


def ctypes_sizeof(s):
    import ctypes
    return ctypes.sizeof(s.srsgpu_uci_result_t)


@pytest.mark.gpu
def test_gpu_vs_golden(ugold):
    """every golden case in one call: ACK / RI / cqi_ack / CQI, g bits, ret and data equal the reference's"""
    import torch
    import srsgpu_phy as s
    z, man = ugold
    got = _gpu_run(s, torch, [(u, z[u["key"] + "_q"], z[u["key"] + "_c"]) for u in man])
    for u, (ret, noi, out, g, data, qp) in zip(man, got):
        k = u["key"]
        assert (out == z[k + "_out"]).all(), (k, out, z[k + "_out"])
        # the reference's g beyond the CQI and data bits is untouched scratch (the Q'_ri Qm entries the RI
        # leaves out): compare the entries the deinterleaver writes
        n = u["nof_bits"] - qp[1] * u["Qm"]
        assert (g[:n] == z[k + "_g"][:n]).all(), (k, np.nonzero(g[:n] != z[k + "_g"][:n])[0][:8])
        assert ret == u["ret"], (k, ret, u["ret"])
        if u["tbs"]:
            assert noi == u["noi"], k
            if ret == 0:
                assert (data == z[k + "_rx"]).all(), k


@pytest.mark.gpu
def test_gpu_mixed_batch_vs_oracle(oracle):
    """random configurations of all UCI kinds (with and without data, 11 / 12 PUSCH symbols) in one call
    against the oracle's UCI and g bits"""
    import torch
    import srsgpu_phy as s
    po = PdschOracle(oracle)
    rng = np.random.default_rng(5)
    cases = []
    while len(cases) < 24:
        Qm = int(rng.choice([2, 4, 6]))
        prb = int(rng.choice([1, 3, 8, 20, 50]))
        O = (int(rng.integers(0, 3)), int(rng.integers(0, 3)), int(rng.choice([0, 2, 9, 11, 14, 33, 100])))
        tbs = int(rng.choice([0, 0, 256, 1544]))
        u = uci_case(tbs, Qm, prb, nof_symb=int(rng.choice([11, 12])), O=O,
                     I_off=(int(rng.integers(0, 15)), int(rng.integers(0, 13)), int(rng.integers(2, 16))))
        if (tbs and u["nof_bits"] < 3 * (tbs + 24)) or O == (0, 0, 0):
            continue
        c = po.sequence(int(rng.integers(1, 2 ** 30)), u["nof_bits"])
        q = rng.integers(-300, 300, u["nof_bits"]).astype(np.int16)
        r, out, g, qp = orc_ulsch_uci(oracle, u, q, c)
        if r:
            continue
        cases.append((u, q, c, out, g, qp))
    got = _gpu_run(s, torch, [(u, q, c) for u, q, c, *_ in cases])
    for (u, _q, _c, out, g, qp), (ret, _noi, gout, gg, _d, gqp) in zip(cases, got):
        assert tuple(gqp) == qp, (u["O"], gqp, qp)
        assert (gout == out).all(), (u["O"], gout, out)
        n = u["nof_bits"] - qp[1] * u["Qm"]  # g entries the deinterleaver writes
        assert (gg[:n] == g[:n]).all(), (u["O"], np.nonzero(gg[:n] != g[:n])[0][:8])
