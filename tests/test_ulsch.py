"""UL-SCH decode (srslte_ulsch_decode, sch.c:883-889 -> srslte_ulsch_uci_decode
:944-985 without UCI -> ulsch_deinterleave :860-881 + decode_tb :437-498).

CPU: the oracle restatement (oracle/dlsch_oracle.c orc_ulsch_*) against the golden HARQ sequences
recorded from the reference build (tests/golden/make_ulsch_golden.py) and, where the reference
build is present, against the live reference on fresh random transmissions.
GPU: srsgpu_ulsch_decode_dev (include/srsgpu/ulsch_batch.h) against the same golden sequences
(return code, TB bytes, nof_iterations, cb_crc — bit-exact), many TBs of mixed sizes in one call
against the oracle, and the error behaviour."""
import json
import os

import numpy as np
import pytest

from srsgpu_testlib import DlschOracle, Ref, have_ref

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def ugold():
    z = np.load(os.path.join(HERE, "golden", "ulsch_golden.npz"))
    return z, json.loads(bytes(z["manifest"]))


@pytest.fixture(scope="module")
def dl(oracle):
    return DlschOracle(oracle)


def test_deinterleave_definition(dl):
    """orc_ulsch_deinterleave is the transpose of the 36.212 5.2.2.8 matrix: q entry
    (i rows + j) Qm + k holds g entry (j cols + i) Qm + k"""
    for Qm, prb, ns in [(2, 6, 12), (4, 25, 11), (6, 3, 12)]:
        rows, cols = 12 * prb, ns
        q = np.arange(rows * cols * Qm, dtype=np.int16)
        g = dl.ulsch_deinterleave(q, Qm, ns)
        for j in (0, rows // 2, rows - 1):
            for i in (0, cols - 1):
                for k in range(Qm):
                    assert g[(j * cols + i) * Qm + k] == q[(i * rows + j) * Qm + k]
        assert sorted(g.tolist()) == q.tolist()


def test_oracle_vs_golden(dl, ugold):
    z, man = ugold
    for c in man:
        sb = dl.softbuffer(16)
        dl.reset(sb)
        for t, st in enumerate(c["steps"]):
            sk = "%s_t%d" % (c["key"], t)
            ret, data, noi, crc = dl.ulsch_decode(sb, c["tbs"], st["rv"], c["Qm"], c["nof_symb"],
                                                  z[sk + "_llr"], c["max_halfits"])
            assert ret == st["ret"] and noi == st["noi"], (sk, ret, noi, st)
            assert (data[:(c["tbs"] + 24) // 8] == z[sk + "_out"]).all(), sk
            assert (crc == z[sk + "_cbcrc"]).all(), sk
        dl.free(sb)
    assert {st["ret"] for c in man for st in c["steps"]} == {0, -1}


@pytest.mark.skipif(not have_ref(), reason="reference build (oracle/_ref) absent")
def test_oracle_vs_live_reference(dl):
    """fresh transmissions: the reference encoder's q bits through AWGN, decoded by the reference
    and by the oracle with HARQ combining"""
    r = Ref()
    rng = np.random.default_rng(5)
    for tbs, Qm, prb, ns, snrs in [(2216, 4, 6, 11, [0.0, 2.0]), (15264, 6, 25, 12, [3.0, 5.0])]:
        nb = 12 * prb * ns * Qm
        data = rng.integers(0, 256, tbs // 8).astype(np.uint8)
        r.sb_reset(1)
        sb = dl.softbuffer(16)
        dl.reset(sb)
        for rv, snr in zip((0, 2), snrs):
            q = r.ul_encode(tbs, rv, Qm, nb, ns, data)
            y = np.where(q == 1, 1.0, -1.0) + 10 ** (-snr / 20) * rng.standard_normal(q.size)
            llr = (100 * y.astype(np.float32)).astype(np.int16)
            a = r.ul_decode(1, tbs, rv, Qm, ns, llr, 8)
            b = dl.ulsch_decode(sb, tbs, rv, Qm, ns, llr, 8)
            assert a[0] == b[0] and a[2] == b[2], (tbs, rv, a[0], b[0], a[2], b[2])
            assert (a[1][:(tbs + 24) // 8] == b[1][:(tbs + 24) // 8]).all()
            assert (a[3] == b[3]).all()
        dl.free(sb)


# ------------------------------------------------------------------ GPU ----

def _dev_decode(s, torch, g, tbl, llrs, maxh=8):
    off, qo, do = 0, [], []
    for t, q in zip(tbl, llrs):
        qo.append(off)
        off += (q.size + 63) // 64 * 64
    dq = torch.zeros(max(off, 1), dtype=torch.int16)
    for o, q in zip(qo, llrs):
        dq[o:o + q.size] = torch.from_numpy(np.ascontiguousarray(q, np.int16))
    dq = dq.cuda()
    dg = torch.zeros_like(dq)
    doff = 0
    for t, o in zip(tbl, qo):
        t["q_offset"], t["data_offset"] = o, doff
        do.append(doff)
        doff += s.dlsch_data_len(t["tbs"]) + 2
    dd = torch.zeros(max(doff, 1), dtype=torch.uint8, device="cuda")
    ret = torch.zeros(len(tbl), dtype=torch.int32, device="cuda")
    noi = torch.zeros(len(tbl), dtype=torch.int32, device="cuda")
    r = g.ulsch_decode_dev(tbl, dq.data_ptr(), dg.data_ptr(), dd.data_ptr(), maxh, ret.data_ptr(),
                           noi.data_ptr())
    torch.cuda.synchronize()
    data = dd.cpu().numpy()
    return r, ret.cpu().numpy(), noi.cpu().numpy(), [data[o:] for o in do], dg.cpu().numpy(), qo


@pytest.mark.gpu
def test_gpu_golden_harq_sequences(ugold):
    import torch
    import srsgpu_phy as s
    z, man = ugold
    g = s.Dlsch(len(man), 16, 64, stream=torch.cuda.current_stream().cuda_stream)
    for slot, c in enumerate(man):
        g.reset(slot)
        for t, st in enumerate(c["steps"]):
            sk = "%s_t%d" % (c["key"], t)
            tb = dict(tbs=c["tbs"], rv=st["rv"], Qm=c["Qm"], nof_bits=c["nbits"], nof_symb=c["nof_symb"],
                      softbuffer=slot)
            r, ret, noi, data, _, _ = _dev_decode(s, torch, g, [tb], [z[sk + "_llr"]], c["max_halfits"])
            assert r == 0
            assert ret[0] == st["ret"] and noi[0] == st["noi"], (sk, ret, noi, st)
            assert (data[0][:(c["tbs"] + 24) // 8] == z[sk + "_out"]).all(), sk
            assert (g.read_cb_crc(slot)[:c["C"]] == z[sk + "_cbcrc"]).all(), sk
    g.close()


@pytest.mark.gpu
def test_gpu_mixed_batch_one_call_vs_oracle(dl):
    """many PUSCH TBs of mixed PRB / Qm / N_symb / SNR in ONE call: deinterleaved g bits, return
    codes, bytes and nof_iterations equal the oracle's"""
    import torch
    import srsgpu_phy as s
    table = json.load(open(os.path.join(HERE, "golden", "c5_traffic.json")))
    rng = np.random.default_rng(11)
    tbl, llrs, ref = [], [], []
    qm_of = {1: 2, 2: 4, 3: 6}
    while len(tbl) < 24:
        prb = int(rng.choice([6, 15, 25, 50, 75, 100]))
        mcs = int(rng.integers(0, 29))
        tbs, Qm = table["tbs_by_prb_mcs"][prb - 1][mcs], qm_of[table["mod_by_mcs"][mcs]]
        ns = int(rng.choice([11, 12]))
        nb = 12 * prb * ns * Qm
        if table["cbsegm_C_C1_K1_C2_K2_F"][str(tbs)][5] or tbs + 24 > 0.9 * nb:
            continue
        data = rng.integers(0, 256, tbs // 8).astype(np.uint8)
        e = dl.encode(tbs, 0, Qm, nb, data)  # DL-SCH coded bits stand in for g: same encode_tb
        rows = nb // Qm // ns
        q = np.empty_like(e)  # interleave g -> q (the transpose the deinterleaver undoes)
        gi = np.arange(nb)
        j, rem = gi // (ns * Qm), gi % (ns * Qm)
        q[((rem // Qm) * rows + j) * Qm + rem % Qm] = e
        snr = float(rng.uniform(0.0, 4.0))
        y = np.where(q == 1, 1.0, -1.0) + 10 ** (-snr / 20) * rng.standard_normal(q.size)
        llr = (100 * y.astype(np.float32)).astype(np.int16)
        sb = dl.softbuffer(16)
        dl.reset(sb)
        ref.append(dl.ulsch_decode(sb, tbs, 0, Qm, ns, llr, 8))
        dl.free(sb)
        tbl.append(dict(tbs=tbs, rv=0, Qm=Qm, nof_bits=nb, nof_symb=ns, softbuffer=len(tbl)))
        llrs.append(llr)
    g = s.Dlsch(len(tbl), 16, 512, stream=torch.cuda.current_stream().cuda_stream)
    g.reset_range(0, len(tbl))
    r, ret, noi, data, dg, qo = _dev_decode(s, torch, g, tbl, llrs)
    assert r == 0
    for i, (t, (rr, dref, nref, cref)) in enumerate(zip(tbl, ref)):
        gdev = dg[qo[i]:qo[i] + t["nof_bits"]]
        assert (gdev == dl.ulsch_deinterleave(llrs[i], t["Qm"], t["nof_symb"])).all(), i
        assert ret[i] == rr and noi[i] == nref, (i, ret[i], rr, noi[i], nref)
        assert (data[i][:(t["tbs"] + 24) // 8] == dref[:(t["tbs"] + 24) // 8]).all(), i
        assert (g.read_cb_crc(i)[:cref.size] == cref).all(), i
    assert len(set(ret.tolist())) > 1 and len(set(noi.tolist())) > 2
    g.close()


@pytest.mark.gpu
def test_gpu_error_behaviour():
    import torch
    import srsgpu_phy as s
    g = s.Dlsch(2, 16, 64, stream=torch.cuda.current_stream().cuda_stream)
    bad = [dict(tbs=600, rv=0, Qm=2, nof_bits=1730, nof_symb=12, softbuffer=0)]  # not rows x 12 x 2
    dq = torch.zeros(4096, dtype=torch.int16, device="cuda")
    out = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    ret = torch.zeros(2, dtype=torch.int32, device="cuda")
    for b in (bad, [dict(bad[0], nof_bits=1728, Qm=3)], [dict(bad[0], nof_bits=1728, nof_symb=0)]):
        b[0].update(q_offset=0, data_offset=0)
        assert g.ulsch_decode_dev(b, dq.data_ptr(), dq.data_ptr(), out.data_ptr(), 8, ret.data_ptr(),
                                  ret.data_ptr()) == -1
    assert g.ulsch_decode_dev([], dq.data_ptr(), dq.data_ptr(), out.data_ptr(), 8, ret.data_ptr(),
                              ret.data_ptr()) == 0
    g.close()
