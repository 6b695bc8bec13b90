"""8-bit turbo decoding path (srslte_tdec_iteration_8bit, turbodecoder.c:392-563, and the int8
window decoders of turbodecoder_win.h): the CPU oracle (oracle/tdec8_oracle.c) against the golden
vectors recorded from the reference (tests/golden/make_tdec8_golden.py) and, where the reference
build exists, against the reference itself; the GPU path against both (marked gpu)."""
import os

import numpy as np
import pytest

from srsgpu_testlib import (AUTO, AVX8_WINDOW, SSE8_WINDOW, Oracle, Ref, have_ref, make_cb8,
                            natural_to_sb)

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "tdec8_golden.npz")


def golden_cases():
    g = np.load(GOLDEN)
    cases = []
    for kind in ("c8", "c16"):
        i = 0
        while "%s_%d_meta" % (kind, i) in g:
            impl, sb, K = (int(v) for v in g["%s_%d_meta" % (kind, i)])
            cases.append((kind, impl, sb, K, g["%s_%d_in" % (kind, i)], g["%s_%d_dec" % (kind, i)]))
            i += 1
    return cases


def test_oracle_matches_golden():
    o = Oracle()
    cases = golden_cases()
    assert len(cases) == 14
    for kind, impl, sb, K, inp, dec in cases:
        nhalf = dec.shape[0]
        got = o.tdec8_run(impl, sb, inp, K, nhalf) if kind == "c8" else o.tdec8_run16(impl, inp, K, nhalf)
        assert got is not None
        np.testing.assert_array_equal(got, dec, err_msg="%s impl=%d sb=%d K=%d" % (kind, impl, sb, K))


def test_golden_decodes_at_5db():
    """the 8-bit decoders decode (they need a few dB more than the 16-bit ones)"""
    for kind, impl, sb, K, inp, dec in golden_cases():
        if kind == "c8" and impl == AUTO and K == 6144 and sb == 1:
            assert dec[-1].any()  # non-trivial output; the bit check is in the GPU test
    o = Oracle()
    bits, llr = make_cb8(6144, 5.0, 3, 16.0, o)
    d = o.tdec8_run(AUTO, 0, llr, 6144, 8)
    assert (np.unpackbits(d[-1]) == bits).all()


@pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built (build container only)")
def test_oracle_matches_reference_sweep():
    o, r = Oracle(), Ref()
    rng = np.random.default_rng(8)
    # every 8-bit window size regime: 16 sub-blocks (K % 32 == 0 and != 0), 32 sub-blocks
    Ks = [816, 848, 880, 1024, 1504, 2048, 2112, 2176, 3200, 5120, 6144]
    for K in Ks:
        nsb = o.lib.orc_autoimp_subblocks_8bit(K)
        for sb in (0, 1):
            ebno, scale = float(rng.choice([1.0, 4.0, 6.0])), float(rng.choice([8.0, 20.0, 64.0]))
            _, llr = make_cb8(K, ebno, K + sb, scale, o)
            inp = natural_to_sb(llr, K, nsb) if sb else llr
            np.testing.assert_array_equal(o.tdec8_run(AUTO, sb, inp, K, 8),
                                          r.tdec8_run(AUTO, sb, inp, K, 8), err_msg="K=%d sb=%d" % (K, sb))
    for impl, K in ((SSE8_WINDOW, 1504), (AVX8_WINDOW, 3200)):
        _, llr = make_cb8(K, 4.0, K, 20.0, o)
        w = llr.astype(np.int16) * 3  # values beyond int8: truncated by the reference
        np.testing.assert_array_equal(o.tdec8_run16(impl, w, K, 6), r.tdec8_run16(impl, w, K, 6))


# ------------------------------------------------------------------ GPU ----
@pytest.fixture(scope="module")
def s():
    import torch  # noqa: F401  (one HIP runtime per process: torch's)
    import srsgpu_phy
    return srsgpu_phy


def _padded8(inp):
    buf = np.zeros(3 * (6144 + 32) + 64, inp.dtype)
    buf[:inp.size] = inp
    return buf


@pytest.mark.gpu
def test_golden_dropin_per_halfiteration(s):
    """srslte_tdec_iteration_8bit / srslte_tdec_iteration (manual int8 types) on the GPU, decision
    bytes after every half-iteration equal to the reference's"""
    for kind, impl, sb, K, inp, dec in golden_cases():
        d = s.Tdec(6144, impl)
        if kind == "c16" or not sb:
            d.force_not_sb()
        assert d.new_cb(K) == 0
        buf = _padded8(inp)
        out = np.zeros(K // 8, np.uint8)
        for n in range(dec.shape[0]):
            if kind == "c8":
                d.iteration_8bit(buf, out)
            else:
                d.iteration(buf, out)
            np.testing.assert_array_equal(out, dec[n], err_msg="%s impl=%d sb=%d K=%d n=%d" % (kind, impl, sb, K, n))
        assert d.get_nof_iterations() == dec.shape[0]
        out2 = np.zeros(K // 8, np.uint8)
        if kind == "c8":
            assert d.run_all_8bit(buf, out2, dec.shape[0], K) == 0
            np.testing.assert_array_equal(out2, dec[-1])
        d.free()


@pytest.mark.gpu
@pytest.mark.parametrize("K,sb", [(848, 1), (1024, 0), (2112, 1), (6144, 1), (6144, 0), (512, 0), (40, 1)])
def test_batch_auto8_vs_oracle(s, K, sb):
    """many code blocks per launch (pair-interleaved lanes, odd count) vs the oracle"""
    o = Oracle()
    b = s.TdecBatch(33, 6144)
    nsb = o.lib.orc_autoimp_subblocks_8bit(K)
    rng = np.random.default_rng(K + sb)
    ins, refs = [], []
    for i in range(33):
        ebno, scale = float(rng.choice([2.0, 5.0])), float(rng.choice([8.0, 20.0, 64.0]))
        _, llr = make_cb8(K, ebno, 1000 * K + i, scale, o)
        inp = natural_to_sb(llr, K, nsb) if (sb and nsb >= 16) else llr
        ins.append(inp.astype(np.int16))
        refs.append(o.tdec8_run(AUTO, sb, inp, K, 6)[-1])
    got = b.run(s.SRSGPU_TDEC_AUTO_8BIT, sb, ins, K, 6)
    np.testing.assert_array_equal(got, np.stack(refs))
    b.close()


@pytest.mark.gpu
def test_batch_auto8_early_stop(s):
    """CRC early stop on the int8 decoders: nof_iterations = first half-iteration whose decision
    passes the CRC (sch.c:361-391), from the oracle's per-half-iteration decisions"""
    o = Oracle()
    K, n, maxh = 6144, 24, 8
    b = s.TdecBatch(n, 6144)
    rng = np.random.default_rng(5)
    ins, exp_noi, exp_ok, exp_bytes = [], [], [], []
    for i in range(n):
        data = rng.integers(0, 2, K - 24, dtype=np.uint8)
        crc = o.crc(s.CRC24B, np.packbits(data), K - 24)
        bits = np.concatenate([data, np.array([(crc >> (23 - j)) & 1 for j in range(24)], np.uint8)])
        from srsgpu_testlib import awgn_llr8
        llr = awgn_llr8(o.tcod_encode(bits), float(rng.choice([3.0, 5.0, 8.0])), rng, 16.0)
        inp = natural_to_sb(llr, K, 32)
        ins.append(inp.astype(np.int16))
        dec = o.tdec8_run(AUTO, 1, inp, K, maxh)
        stop = next((h for h in range(maxh) if o.crc(s.CRC24B, dec[h], K) == 0), None)
        exp_noi.append(maxh if stop is None else stop + 1)
        exp_ok.append(0 if stop is None else 1)
        exp_bytes.append(dec[maxh - 1 if stop is None else stop])
    out, ok, noi = b.decode(s.SRSGPU_TDEC_AUTO_8BIT, 1, ins, K, maxh, s.CRC24B, K)
    np.testing.assert_array_equal(noi, exp_noi)
    np.testing.assert_array_equal(ok, exp_ok)
    np.testing.assert_array_equal(out, np.stack(exp_bytes))
    assert 0 < sum(exp_ok) < n or sum(exp_ok) == n
    b.close()


@pytest.mark.gpu
def test_int8_undefined_cases_fail_loudly(s):
    """where the reference has no defined result the GPU path returns an error instead of guessing"""
    b = s.TdecBatch(2, 6144)
    x = np.zeros(3 * (512 + 32) + 12, np.int16)
    with pytest.raises(RuntimeError):
        b.run(s.SRSGPU_TDEC_AUTO_8BIT, 1, [x], 512, 2)  # 8-bit SB input at 400 < K <= 800
    b.close()
    d = s.Tdec(6144, s.SRSLTE_TDEC_AVX8_WINDOW)  # int8 type, 16-bit SB input
    assert d.new_cb(6144) == 0
    assert d.run_all(np.zeros(3 * (6144 + 32) + 12, np.int16), np.zeros(768, np.uint8), 2, 6144) == -1
    d.free()
