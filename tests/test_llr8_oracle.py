"""CPU checks of the 8-bit LLR chain oracle (oracle/pdsch_oracle.c orc_demod_b / orc_scramble_sb /
orc_csi_correction_b, oracle/dlsch_oracle.c orc_rm_turbo_rx_8bit / orc_dlsch_decode8) against
golden vectors recorded from the srsLTE reference (tests/golden/make_llr8_golden.py) and, where
oracle/_ref exists, against the reference on random cases (llr_is_8bit: pdsch.c:795-806,
sch.c:344-364)."""
import json
import os

import numpy as np
import pytest

from srsgpu_testlib import DlschOracle, Llr8, Ref, have_ref

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def l8(oracle):
    return Llr8(oracle)


@pytest.fixture(scope="module")
def gold():
    z = np.load(os.path.join(HERE, "golden", "llr8_golden.npz"))
    return z, json.loads(bytes(z["manifest"]))


def test_golden_demod_b(l8, gold):
    z, man = gold
    cases = [c for c in man if c["kind"] == "demod"]
    assert len(cases) == 72
    for c in cases:
        assert (l8.demod(c["mod"], z[c["key"] + "_sym"]) == z[c["key"] + "_llr"]).all(), c["key"]


def test_golden_scrambling_sb(l8, gold):
    z, man = gold
    for c in (c for c in man if c["kind"] == "scramble"):
        out = l8.scramble(c["rnti"], c["q"], c["nslot"], c["cell_id"], z[c["key"] + "_in"])
        assert (out == z[c["key"] + "_out"]).all(), c["key"]


def test_golden_rm_8bit(l8, gold):
    z, man = gold
    for c in (c for c in man if c["kind"] == "rm"):
        out = np.zeros(18600 * 2, np.int8)
        init = z[c["key"] + "_init"]
        out[:init.size] = init
        l8.rm_rx(z[c["key"] + "_e"], out, c["K"], c["rv"])
        assert (out[:init.size] == z[c["key"] + "_out"]).all(), c["key"]


def test_golden_dlsch_decode8(oracle, l8, gold):
    z, man = gold
    dl = DlschOracle(oracle)
    nack = nok = 0
    for c in (c for c in man if c["kind"] == "tb"):
        sb = dl.softbuffer(16)
        dl.reset(sb)
        for t in c["tx"]:
            ret, data, noi, crc = l8.decode(sb, c["tbs"], t["rv"], c["Qm"], z[t["key"] + "_llr"], 8)
            assert (ret, noi) == (t["ret"], t["noi"]), t["key"]
            assert (crc == z[t["key"] + "_cbcrc"]).all(), t["key"]
            if ret == 0:
                nok += 1
                assert (data[:c["tbs"] // 8] == z[c["key"] + "_tx"]).all(), t["key"]
            else:
                nack += 1
        dl.free(sb)
    assert nok >= 8 and nack >= 8  # both outcomes are covered


def test_refuses_undefined_8bit_sizes(oracle, l8):
    # 400 < K <= 800: the reference's 8-bit AUTO feeds a 16-bit window 3K+12 of 3(K+32)+12 values
    dl = DlschOracle(oracle)
    sb = dl.softbuffer(4)
    r, _, _, _ = l8.decode(sb, 456, 0, 2, np.ones(1200, np.int8), 8)
    dl.free(sb)
    assert r == -2


def test_csi_8bit_weights():
    # (int8_t)((float)e * (csi / csi_max)): truncation towards zero (pdsch.c:707-713)
    from srsgpu_testlib import Oracle
    l8 = Llr8(Oracle())
    e = np.array([100, -100, 127, -128, 7, -7], np.int8)
    out = l8.csi_correction(1, np.array([0.5, 1.0, 0.3], np.float32), e)
    assert out.tolist() == [50, -50, 127, -128, 2, -2]


@pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built")
def test_random_vs_reference(l8):
    r = Llr8(Ref(), ref=True)
    rng = np.random.default_rng(5)
    for mod in (1, 2, 3):
        for n in (3, 8, 17, 64, 333):
            for amp in (0.2, 1.5, 6.0):
                sym = ((rng.standard_normal(n) + 1j * rng.standard_normal(n)) * amp).astype(np.complex64)
                assert (l8.demod(mod, sym) == r.demod(mod, sym)).all()
    for K in (40, 408, 816, 1024, 2048, 2112, 6144):
        for rv in range(4):
            e = rng.integers(-128, 128, 2 * (3 * K + 12) + 5).astype(np.int8)
            a = l8.rm_rx(e, np.zeros(18600 * 2, np.int8), K, rv)
            b = r.rm_rx(e, np.zeros(18600 * 2, np.int8), K, rv)
            assert (a == b).all(), (K, rv)
