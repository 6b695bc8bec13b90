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
