"""Parity of the MI355X DL-SCH transport-block decoder (libsrsgpu_phy.so, srsgpu_dlsch_*) with
the golden HARQ sequences recorded from the srsLTE reference (sch.c decode_tb) and with the CPU
oracle: return codes, TB bytes, nof_iterations, softbuffer cb_crc flags and soft bits."""
import json
import os

import numpy as np
import pytest

from srsgpu_testlib import DlschOracle, SOFTBUFFER_SIZE

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def s():
    import srsgpu_phy
    return srsgpu_phy


@pytest.fixture(scope="module")
def dgold():
    z = np.load(os.path.join(HERE, "golden", "dlsch_golden.npz"))
    return z, json.loads(bytes(z["manifest"]))


@pytest.fixture(scope="module")
def dl(oracle):
    return DlschOracle(oracle)


def _tb(tbs, rv, Qm, nbits, slot):
    return dict(tbs=tbs, rv=rv, Qm=Qm, nof_e_bits=nbits, softbuffer=slot)


def test_golden_harq_sequences(s, dgold):
    """Each golden TB in its own softbuffer; every transmission matches the reference."""
    z, man = dgold
    tbc = [c for c in man if c["kind"] == "tb"]
    g = s.Dlsch(len(tbc), 16, 64)
    for slot, c in enumerate(tbc):
        g.reset(slot)
        for t, st in enumerate(c["steps"]):
            sk = "%s_t%d" % (c["key"], t)
            ret, data, noi = g.decode([_tb(c["tbs"], st["rv"], c["Qm"], c["nbits"], slot)],
                                      [z[sk + "_llr"]], c["max_halfits"])
            nbytes = (c["tbs"] + 24) // 8
            assert ret[0] == st["ret"] and noi[0] == st["noi"], (sk, ret, noi, st)
            assert (data[0][:nbytes] == z[sk + "_out"]).all(), sk
            _, crc = g.read_softbuffer(slot)
            assert (crc[:c["C"]] == z[sk + "_cbcrc"]).all(), sk
    g.close()


def test_golden_all_first_transmissions_one_call(s, dgold):
    """All golden TBs' first transmissions in ONE call (mixed K, C, CRC types)."""
    z, man = dgold
    tbc = [c for c in man if c["kind"] == "tb"]
    g = s.Dlsch(len(tbc), 16, 128)
    for slot in range(len(tbc)):
        g.reset(slot)
    tbl = [_tb(c["tbs"], c["steps"][0]["rv"], c["Qm"], c["nbits"], i) for i, c in enumerate(tbc)]
    ret, data, noi = g.decode(tbl, [z["%s_t0_llr" % c["key"]] for c in tbc], 8)
    for i, c in enumerate(tbc):
        st = c["steps"][0]
        assert ret[i] == st["ret"] and noi[i] == st["noi"], c["key"]
        assert (data[i][:(c["tbs"] + 24) // 8] == z["%s_t0_out" % c["key"]]).all(), c["key"]
    g.close()


def test_softbuffer_soft_bits_vs_oracle(s, dl, dgold):
    """After a failed first transmission the device softbuffer rows equal the oracle's."""
    z, man = dgold
    c = [c for c in man if c["kind"] == "tb" and c["C"] > 1 and c["steps"][0]["ret"] != 0][0]
    g = s.Dlsch(1, 16, 32)
    g.reset(0)
    llr = z["%s_t0_llr" % c["key"]]
    g.decode([_tb(c["tbs"], 0, c["Qm"], c["nbits"], 0)], [llr], 8)
    rows, crc = g.read_softbuffer(0)
    sb = dl.softbuffer(16)
    dl.reset(sb)
    dl.decode(sb, c["tbs"], 0, c["Qm"], llr, 8)
    orows = np.ctypeslib.as_array(sb.buffer, shape=(16 * SOFTBUFFER_SIZE,)).reshape(16, -1)
    assert (rows[:c["C"]] == orows[:c["C"]]).all()
    dl.free(sb)
    g.close()


def test_direct_derm_rows(s, dl, dgold):
    """Direct de-rate-matching: a failed TB leaves every row of its not-yet-decoded blocks as the
    oracle's srslte_rm_turbo_rx_lut (all C rows, also those whose CRC passed in this call); an
    acked TB's rows are not written (read back as a reset row); decoded bytes, ret, noi and cb_crc
    equal the reference over the whole HARQ sequence in both modes."""
    z, man = dgold
    tbc = [c for c in man if c["kind"] == "tb" and c["C"] > 1]
    for c in tbc:
        outs = {}
        for direct in (True, False):
            g = s.Dlsch(1, 16, 32)
            g.set_direct_derm(direct)
            g.reset(0)
            sb = dl.softbuffer(16)
            dl.reset(sb)
            res = []
            for t, st in enumerate(c["steps"]):
                llr = z["%s_t%d_llr" % (c["key"], t)]
                ret, data, noi = g.decode([_tb(c["tbs"], st["rv"], c["Qm"], c["nbits"], 0)], [llr],
                                          c["max_halfits"])
                dl.decode(sb, c["tbs"], st["rv"], c["Qm"], llr, c["max_halfits"])
                rows, crc = g.read_softbuffer(0)
                orows = np.ctypeslib.as_array(sb.buffer, shape=(16 * SOFTBUFFER_SIZE,)).reshape(16, -1)
                if st["ret"] != 0 or not direct:
                    assert (rows[:c["C"]] == orows[:c["C"]]).all(), (c["key"], t, direct)
                res.append((ret[0], noi[0], data[0][:(c["tbs"] + 24) // 8].tobytes(), crc[:c["C"]].tobytes()))
                assert ret[0] == st["ret"] and noi[0] == st["noi"], (c["key"], t, direct)
            if direct and c["steps"][0]["ret"] == 0:
                rows, _ = g.read_softbuffer(0)
                assert not rows[:c["C"]].any()  # acked on the first transmission: rows never written
            outs[direct] = res
            dl.free(sb)
            g.close()
        assert outs[True] == outs[False], c["key"]


def test_rate_dematching_dev_golden(s, oracle, dgold):
    import torch
    z, man = dgold
    g = s.Dlsch(1, 1, 4)
    for c in man:
        if c["kind"] != "rm":
            continue
        K = c["K"]
        d_in = torch.from_numpy(np.ascontiguousarray(z[c["key"] + "_in"])).cuda()
        d_out = torch.zeros(3 * (K + 32) + 12, dtype=torch.int16, device="cuda")
        assert g.rm_rx_dev(d_in.data_ptr(), d_out.data_ptr(), d_in.numel(), K, c["rv"], c["sb"]) == 0
        torch.cuda.synchronize()
        assert (d_out.cpu().numpy() == z[c["key"] + "_out"]).all(), c["key"]
    g.close()


@pytest.mark.parametrize("direct", [True, False])
def test_random_harq_batches_vs_oracle(s, dl, oracle, direct):
    """Batches of random TBs (varied TBS/Qm/E/SNR/rv) across several HARQ rounds, one call per
    round, against the oracle with its own softbuffers; with the direct de-rate-matching
    (srsgpu_dlsch_set_direct_derm, the default: rows written after the decode for failed TBs only)
    and without it. E spans short blocks, E > 8192 (LLRs gathered from HBM) and E > 3K+12
    (repetition)."""
    rng = np.random.default_rng(77)
    good = [t for t in list(range(16, 6200, 24)) + list(range(6200, 80000, 312))
            if oracle.cbsegm(t)[5] == 0]
    n = 12
    g = s.Dlsch(n, 16, 256)
    g.set_direct_derm(direct)
    osb = [dl.softbuffer(16) for _ in range(n)]
    tbl, datas = [], []
    for i in range(n):
        tbs, Qm = int(rng.choice(good)), int(rng.choice([2, 4, 6]))
        C = oracle.cbsegm(tbs)[0]
        nb = int(3.1 * tbs * rng.uniform(0.4, 1.5))
        nb = max(nb - nb % Qm, Qm * C)
        tbl.append(_tb(tbs, 0, Qm, nb, i))
        datas.append(rng.integers(0, 256, tbs // 8).astype(np.uint8))
        g.reset(i)
        dl.reset(osb[i])
    snr = rng.uniform(-0.5, 3.0, n)
    for rnd, rv in enumerate((0, 2, 3, 1)):
        llrs = []
        for i, t in enumerate(tbl):
            t["rv"] = rv
            e = dl.encode(t["tbs"], rv, t["Qm"], t["nof_e_bits"], datas[i])
            y = np.where(e == 1, 1.0, -1.0) + 10 ** (-snr[i] / 20) * rng.standard_normal(e.size)
            llrs.append((100 * y).astype(np.float32).astype(np.int16))
        ret, data, noi = g.decode(tbl, llrs, 8)
        for i, t in enumerate(tbl):
            r, od, onoi, ocrc = dl.decode(osb[i], t["tbs"], rv, t["Qm"], llrs[i], 8)
            nbytes = (t["tbs"] + 24) // 8
            assert ret[i] == r and noi[i] == onoi, (rnd, i, ret[i], r, noi[i], onoi)
            assert (data[i][:nbytes] == od[:nbytes]).all(), (rnd, i)
            _, crc = g.read_softbuffer(i)
            assert (crc[:len(ocrc)] == ocrc).all(), (rnd, i)
    for b in osb:
        dl.free(b)
    g.close()


def test_full_subframe_batch_device(s, dl):
    """C3 shape: 64 x TBS 75376 (13 x K=5824, 64QAM, 90000 coded bits), noiseless LLRs, device
    pointers: every TB decodes with nof_iterations 1 (CRC after the first half-iteration)."""
    import torch
    n, tbs, nb = 64, 75376, 90000
    rng = np.random.default_rng(9)
    data = rng.integers(0, 256, (4, tbs // 8)).astype(np.uint8)
    e = np.stack([np.where(dl.encode(tbs, 0, 6, nb, d) == 1, 100, -100) for d in data]).astype(np.int16)
    e_all = e[np.arange(n) % 4]
    d_e = torch.from_numpy(np.ascontiguousarray(e_all)).cuda()
    dl_len = tbs // 8 + 6
    d_data = torch.zeros(n * dl_len, dtype=torch.uint8, device="cuda")
    d_ret = torch.full((n,), 7, dtype=torch.int32, device="cuda")
    d_noi = torch.zeros(n, dtype=torch.int32, device="cuda")
    g = s.Dlsch(n, 13, n * 13, stream=torch.cuda.current_stream().cuda_stream)
    for i in range(n):
        g.reset(i)
    tbl = [dict(tbs=tbs, rv=0, Qm=6, nof_e_bits=nb, softbuffer=i, e_offset=i * nb,
                data_offset=i * dl_len) for i in range(n)]
    assert g.decode_dev(tbl, d_e.data_ptr(), d_data.data_ptr(), 8, d_ret.data_ptr(),
                        d_noi.data_ptr()) == 0
    torch.cuda.synchronize()
    assert (d_ret.cpu().numpy() == 0).all()
    assert (d_noi.cpu().numpy() == 1).all()
    out = d_data.cpu().numpy().reshape(n, dl_len)
    assert (out[:, :tbs // 8] == data[np.arange(n) % 4]).all()
    g.close()


def test_invalid_and_empty_tbs(s):
    g = s.Dlsch(2, 13, 16)
    g.reset(0)
    g.reset(1)
    e = np.zeros(3000, np.int16)
    # 1001 bits: B' = 1025 is not a code block size -> filler bits -> SRSLTE_ERROR_INVALID_INPUTS
    ret, _, noi = g.decode([_tb(1001, 0, 2, 3000, 0), _tb(0, 0, 2, 3000, 1)], [e, e], 8)
    assert ret == [-2, 0] and list(noi) == [0, 0]
    with pytest.raises(RuntimeError):
        g.decode([_tb(1000, 0, 2, 3000, 5)], [e], 8)  # no such softbuffer
    g.close()


def test_encode_vs_oracle(s, dl):
    """srsgpu_dlsch_encode_dev (CRC24A, segmentation + CRC24B, turbo encoding, rate matching) is
    bit-exact with the oracle's encode_tb restatement (itself pinned to the reference encoder in
    test_dlsch_oracle.py) for single and multi-CB TBs (K1/K2 mixes), every rv and modulation."""
    import torch
    rng = np.random.default_rng(11)
    cases = []
    for tbs, nbits_per_qm in ((40, 120), (1000, 1500), (6120, 4000), (12216, 9000), (30576, 21000),
                              (51024, 30000), (75376, 15000), (97896, 40000)):
        for Qm in (2, 4, 6):
            cases.append((tbs, int(rng.integers(0, 4)), Qm, nbits_per_qm * Qm))
    g = s.Dlsch(8, 16, 16 * 64)
    tbl, datas, doff, eoff = [], [], 0, 0
    for tbs, rv, Qm, nbits in cases:
        data = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
        tbl.append(dict(tbs=tbs, rv=rv, Qm=Qm, nof_e_bits=nbits, softbuffer=0, data_offset=doff,
                        e_offset=eoff))
        datas.append(data)
        doff += tbs // 8 + 8
        eoff += nbits + 8
    d_data = torch.zeros(doff, dtype=torch.uint8, device="cuda")
    for t, d in zip(tbl, datas):
        d_data[t["data_offset"]:t["data_offset"] + d.size] = torch.from_numpy(d)
    d_e = torch.full((eoff,), 7, dtype=torch.uint8, device="cuda")
    assert g.encode_dev(tbl, d_data.data_ptr(), d_e.data_ptr()) == 0
    e = d_e.cpu().numpy()
    for (tbs, rv, Qm, nbits), t, d in zip(cases, tbl, datas):
        ref = dl.encode(tbs, rv, Qm, nbits, d)
        got = e[t["e_offset"]:t["e_offset"] + nbits]
        assert (got == ref).all(), (tbs, rv, Qm, np.nonzero(got != ref)[0][:5])
        assert e[t["e_offset"] + nbits] == 7  # nothing written past nof_e_bits
    # filler bits: refused like sch.c:203-206
    assert g.encode_dev([dict(tbs=1001, rv=0, Qm=2, nof_e_bits=3000, softbuffer=0)], d_data.data_ptr(),
                        d_e.data_ptr()) == -1
    g.close()


def test_encode_decode_roundtrip_full_size(s):
    """1024 x TBS 75376 (the C3 subframe load) encoded on the device, mapped to noiseless LLRs and
    decoded: every TB acks with its data after one half-iteration per CB."""
    import torch
    n, tbs, nbits = 256, 75376, 90000
    g = s.Dlsch(n, 13, n * 13)
    data = torch.randint(0, 256, (n, tbs // 8), dtype=torch.uint8, device="cuda")
    d_e = torch.zeros((n, nbits), dtype=torch.uint8, device="cuda")
    tbl = [dict(tbs=tbs, rv=0, Qm=6, nof_e_bits=nbits, softbuffer=i, data_offset=i * (tbs // 8),
                e_offset=i * nbits) for i in range(n)]
    assert g.encode_dev(tbl, data.data_ptr(), d_e.data_ptr()) == 0
    llr = (d_e.to(torch.int16) * 200 - 100).contiguous()
    dlen = tbs // 8 + 6
    out = torch.zeros((n, dlen), dtype=torch.uint8, device="cuda")
    ret = torch.zeros(n, dtype=torch.int32, device="cuda")
    noi = torch.zeros(n, dtype=torch.int32, device="cuda")
    tbl2 = [dict(tbs=tbs, rv=0, Qm=6, nof_e_bits=nbits, softbuffer=i, e_offset=i * nbits,
                 data_offset=i * dlen) for i in range(n)]
    assert g.decode_dev(tbl2, llr.data_ptr(), out.data_ptr(), 8, ret.data_ptr(), noi.data_ptr()) == 0
    torch.cuda.synchronize()
    assert (ret.cpu().numpy() == 0).all()
    assert (out[:, :tbs // 8].cpu().numpy() == data.cpu().numpy()).all()
    assert (noi.cpu().numpy() == 1).all()
    g.close()
