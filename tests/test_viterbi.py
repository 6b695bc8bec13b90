"""PDCCH Viterbi decoder (§8(f) rank 1's convolutional decoding: srslte_viterbi_decode_f on the
tail-biting K=7 r=1/3 decoder of pdcch.c:79,341): the oracle restatement of the reference's AVX2
16-bit path (oracle/pdsch_oracle.c orc_viterbi37_tb_decode_f) against golden vectors recorded
from the reference (tests/golden/make_viterbi_golden.py) and, with oracle/_ref, random cases
(CPU); the batched GPU decoder (include/srsgpu/viterbi_batch.h) against both (GPU)."""
import json
import os

import numpy as np
import pytest

from srsgpu_testlib import Ref, have_ref, viterbi_tb_decode_f

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def gold():
    z = np.load(os.path.join(HERE, "golden", "viterbi_golden.npz"))
    return z, json.loads(bytes(z["manifest"]))


def test_golden_oracle(oracle, gold):
    z, man = gold
    assert len(man) == 40
    for c in man:
        out = viterbi_tb_decode_f(oracle, z[c["key"] + "_sym"], c["F"])
        assert (out == z[c["key"] + "_out"]).all(), c["key"]


@pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built")
def test_random_vs_reference(oracle):
    ref = Ref()
    rng = np.random.default_rng(12)
    for F in (20, 45, 61, 96):
        for snr in (-4.0, 1.0, 8.0):
            x = (rng.standard_normal(3 * F) + 10 ** (snr / 20) * np.where(rng.random(3 * F) < 0.5, 1, -1)).astype(np.float32)
            assert (viterbi_tb_decode_f(oracle, x, F) == viterbi_tb_decode_f(ref, x, F, ref=True)).all()


@pytest.mark.gpu
def test_gpu_batch_vs_golden_and_oracle(oracle, gold):
    """all golden frames plus 600 random ones (DCI-like lengths, mixed SNR) in one launch"""
    import torch
    import srsgpu_phy as s
    z, man = gold
    rng = np.random.default_rng(99)
    frames = [z[c["key"] + "_sym"] for c in man]
    want = [z[c["key"] + "_out"] for c in man]
    for i in range(600):
        F = int(rng.choice([37, 41, 43, 47, 57, 58]))
        snr = float(rng.uniform(-4, 10))
        x = (rng.standard_normal(3 * F) + 10 ** (snr / 20) * np.where(rng.random(3 * F) < 0.5, 1, -1)).astype(np.float32)
        frames.append(x)
        want.append(viterbi_tb_decode_f(oracle, x, F))
    got = s.viterbi37_tb_decode_f_batch(torch, frames)
    for i, (g, w) in enumerate(zip(got, want)):
        assert (g == w).all(), i


@pytest.fixture(scope="module")
def dgold():
    z = np.load(os.path.join(HERE, "golden", "dci_golden.npz"))
    return z, json.loads(bytes(z["manifest"]))


def test_golden_dci_oracle(oracle, dgold):
    """srslte_pdcch_decode_msg's candidate decode (mean check, rm_conv_rx, Viterbi, CRC16)"""
    from srsgpu_testlib import dci_decode
    z, man = dgold
    assert len(man) == 84 and 0 < sum(c["decoded"] for c in man) < 84
    for c in man:
        r, d, crc = dci_decode(oracle, z[c["key"] + "_e"], c["nof_bits"])
        assert r == c["decoded"], c["key"]
        if r:
            assert (d == z[c["key"] + "_bits"]).all() and crc == c["crc_rem"], c["key"]


@pytest.mark.gpu
def test_gpu_dci_batch_vs_golden_and_oracle(oracle, dgold):
    """every golden candidate plus 500 random ones (all PDCCH formats, DCI sizes 19..57) in one
    launch: skip decision, bits and CRC remainder equal"""
    import torch
    import srsgpu_phy as s
    from srsgpu_testlib import dci_decode
    z, man = dgold
    cands = [(z[c["key"] + "_e"], c["nof_bits"]) for c in man]
    want = [(c["decoded"], z[c["key"] + "_bits"], c["crc_rem"]) for c in man]
    rng = np.random.default_rng(5)
    for i in range(500):
        E = int(rng.choice([72, 144, 288, 576]))
        nb = int(rng.choice([19, 21, 25, 27, 31, 43, 57]))
        amp = float(rng.uniform(0.2, 3))
        e = (amp * (rng.standard_normal(E) + np.where(rng.random(E) < 0.5, 1, -1))).astype(np.float32)
        cands.append((e, nb))
        want.append(dci_decode(oracle, e, nb))
    got = s.dci_decode_batch(torch, cands)
    for i, (g, w) in enumerate(zip(got, want)):
        assert g[0] == w[0], i
        if w[0]:
            assert (g[1] == w[1]).all() and g[2] == w[2], i
