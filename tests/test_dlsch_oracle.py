"""CPU checks of the DL-SCH oracle (oracle/dlsch_oracle.c): de-rate-matching tables, the TB
encoder used for test traffic and transport-block decoding with HARQ softbuffers, against the
golden vectors recorded from the srsLTE reference and, where oracle/_ref exists, against the
reference itself on random cases."""
import json
import os

import numpy as np
import pytest

from srsgpu_testlib import DlschOracle, Oracle, Ref, have_ref

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def dl(oracle):
    return DlschOracle(oracle)


@pytest.fixture(scope="module")
def dgold():
    z = np.load(os.path.join(HERE, "golden", "dlsch_golden.npz"))
    return z, json.loads(bytes(z["manifest"]))


def test_golden_rate_dematching(dl, oracle, dgold):
    z, man = dgold
    n = 0
    for c in man:
        if c["kind"] != "rm":
            continue
        K = c["K"]
        nsb = oracle.lib.orc_autoimp_subblocks(K) if c["sb"] else 0
        out = np.zeros(3 * (K + 32) + 12, np.int16)
        dl.rm_rx(z[c["key"] + "_in"], out, K, c["rv"], nsb)
        assert (out == z[c["key"] + "_out"]).all(), c["key"]
        n += 1
    assert n >= 6


def test_golden_tb_harq_sequences(dl, oracle, dgold):
    """Every transmission of every HARQ sequence: return code, data, nof_iterations, cb_crc."""
    z, man = dgold
    sb = dl.softbuffer(16)
    try:
        for c in man:
            if c["kind"] != "tb":
                continue
            dl.reset(sb)
            tbs = c["tbs"]
            for t, st in enumerate(c["steps"]):
                sk = "%s_t%d" % (c["key"], t)
                r, data, noi, cb_crc = dl.decode(sb, tbs, st["rv"], c["Qm"], z[sk + "_llr"],
                                                 c["max_halfits"])
                assert r == st["ret"] and noi == st["noi"], (sk, r, noi, st)
                assert (cb_crc == z[sk + "_cbcrc"]).all(), sk
                assert (data[:(tbs + 24) // 8] == z[sk + "_out"]).all(), sk
            if c["steps"][-1]["ret"] == 0:
                assert (data[:tbs // 8] == z[c["key"] + "_data"]).all()
    finally:
        dl.free(sb)


def test_encoder_roundtrip_noiseless(dl, oracle):
    """Oracle encoder -> noiseless LLRs -> oracle decoder recovers the TB (every rv when the
    code rate leaves room; at rate 0.84 only rv 0 carries the systematic bits)."""
    rng = np.random.default_rng(3)
    sb = dl.softbuffer(16)
    for tbs, Qm, nb in [(75376, 6, 90000), (5736, 4, 12000), (376, 2, 1200), (31704, 2, 70000)]:
        data = rng.integers(0, 256, tbs // 8).astype(np.uint8)
        for rv in (range(4) if nb >= 3 * tbs else (0,)):
            e = dl.encode(tbs, rv, Qm, nb, data)
            dl.reset(sb)
            r, out, noi, _ = dl.decode(sb, tbs, rv, Qm, np.where(e == 1, 100, -100), 8)
            assert r == 0 and (out[:tbs // 8] == data).all(), (tbs, rv)
    dl.free(sb)


needs_ref = pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built (build container only)")


def _good_tbs(oracle):
    return [t for t in list(range(16, 6200, 8)) + list(range(6200, 80000, 56))
            if oracle.cbsegm(t)[5] == 0]


@needs_ref
def test_rm_tables_vs_reference(dl, oracle):
    r = Ref()
    for K in (40, 48, 400, 408, 512, 800, 816, 1056, 2048, 4032, 5824, 6144):
        nsb = oracle.lib.orc_autoimp_subblocks(K)
        for rv in range(4):
            for sb in (0, 1):
                e = (np.arange(3 * K + 12) + 1).astype(np.int16)
                a = np.zeros(3 * (K + 32) + 12, np.int16)
                b = a.copy()
                r.rm_rx(e, a, K, rv, sb)
                dl.rm_rx(e, b, K, rv, nsb if sb else 0)
                assert (a == b).all(), (K, rv, sb)


@needs_ref
def test_encoder_vs_reference(dl, oracle):
    r = Ref()
    good = _good_tbs(oracle)
    rng = np.random.default_rng(11)
    for _ in range(25):
        tbs, rv, Qm = int(rng.choice(good)), int(rng.integers(4)), int(rng.choice([2, 4, 6]))
        C = oracle.cbsegm(tbs)[0]
        nb = int(3.1 * tbs * rng.uniform(0.35, 1.6))
        nb = max(nb - nb % Qm, Qm * C)
        data = rng.integers(0, 256, tbs // 8).astype(np.uint8)
        assert (r.encode(tbs, rv, Qm, nb, data) == dl.encode(tbs, rv, Qm, nb, data)).all()


@needs_ref
def test_decode_harq_vs_reference(dl, oracle):
    r = Ref()
    good = _good_tbs(oracle)
    rng = np.random.default_rng(12)
    sb = dl.softbuffer(16)
    for _ in range(20):
        tbs, Qm = int(rng.choice(good)), int(rng.choice([2, 4, 6]))
        C = oracle.cbsegm(tbs)[0]
        nb = int(3.1 * tbs * rng.uniform(0.35, 1.6))
        nb = max(nb - nb % Qm, Qm * C)
        data = rng.integers(0, 256, tbs // 8).astype(np.uint8)
        snr = rng.uniform(-1, 4)
        r.sb_reset(0)
        dl.reset(sb)
        for rv in (0, 2, 3, 1):
            e = dl.encode(tbs, rv, Qm, nb, data)
            y = np.where(e == 1, 1.0, -1.0) + 10 ** (-snr / 20) * rng.standard_normal(e.size)
            llr = (100 * y).astype(np.float32).astype(np.int16)
            a = r.decode(0, tbs, rv, Qm, llr, 8)
            b = dl.decode(sb, tbs, rv, Qm, llr, 8)
            nbytes = (tbs + 24) // 8
            assert a[0] == b[0] and a[2] == b[2] and (a[3] == b[3]).all(), (tbs, rv)
            assert (a[1][:nbytes] == b[1][:nbytes]).all(), (tbs, rv)
            if a[0] == 0:
                break
    dl.free(sb)
