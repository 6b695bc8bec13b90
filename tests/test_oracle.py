"""CPU checks of the test oracle (oracle/liboracle.so): golden vectors recorded from the
reference, and — where oracle/_ref exists (build container) — the reference itself."""
import numpy as np
import pytest

from srsgpu_testlib import (AUTO, AVX_WINDOW, CRC24A, CRC24B, GENERIC, SSE, SSE_WINDOW, Ref,
                            cb_sizes, have_ref, make_cb, natural_to_sb, pack_bits)


def test_golden_run_cases(oracle, golden):
    z, manifest = golden
    n = 0
    for c in manifest:
        if c["kind"] != "run":
            continue
        k = c["key"]
        dec, app1, ext1 = oracle.tdec_run(c["impl"], c["sb"], z[k + "_in"], c["K"], c["halfits"])
        assert (dec == z[k + "_dec"]).all(), k
        assert (app1 == z[k + "_app1"]).all(), k
        assert (ext1 == z[k + "_ext1"]).all(), k
        n += 1
    assert n >= 30


def test_golden_early_stop_cases(oracle, golden):
    z, manifest = golden
    seen_noi = set()
    for c in manifest:
        if c["kind"] != "early_stop":
            continue
        k = c["key"]
        ok, out, noi = oracle.decode_cb(c["impl"], c["sb"], z[k + "_in"], c["K"], c["max_halfits"],
                                        c["poly"], c["K"])
        assert ok == c["crc_ok"] and noi == c["noi"], k
        assert (out == z[k + "_out"]).all(), k
        seen_noi.add(noi)
    assert len(seen_noi) >= 4  # fixtures exercise several stopping points


def test_golden_high_snr_decodes(golden):
    z, manifest = golden
    for c in manifest:
        if c["kind"] == "early_stop" and c["crc_ok"]:
            assert (z[c["key"] + "_out"] == pack_bits(z[c["key"] + "_bits"])).all()


def test_interleaver_is_permutation_and_contention_free(oracle):
    for K in (40, 408, 816, 2048, 5824, 6144):
        f, r = oracle.interl(K, 1)
        assert sorted(f) == list(range(K))
        assert (r[f] == np.arange(K)).all()
        # QPP: pi(x + t*W) = pi(x) mod W for every window length W dividing K
        for W in (8, 16):
            if K % W == 0:
                L = K // W
                x = np.arange(K)
                assert ((f[x] % L) == (f[x % L] % L)).all()
        for nsb in (8, 16):
            if K % nsb == 0:
                fs, rs = oracle.interl(K, nsb)
                assert (rs[fs] == np.arange(K)).all()


def test_crc_known_answers(oracle):
    # CRC of a message with its own CRC appended is zero (TS 36.212 5.1.1)
    rng = np.random.default_rng(3)
    for poly in (CRC24A, CRC24B):
        for nbytes in (1, 3, 64, 765):
            d = rng.integers(0, 256, nbytes, dtype=np.uint8)
            c = oracle.crc(poly, d, 8 * nbytes)
            full = np.concatenate([d, np.array([c >> 16, (c >> 8) & 255, c & 255], np.uint8)])
            assert oracle.crc(poly, full, 8 * nbytes + 24) == 0
    assert oracle.crc(CRC24A, np.zeros(4, np.uint8), 32) == 0


def test_cbsegm_20mhz_mcs28(oracle):
    # C3: TBS 75376 -> 13 code blocks of K=5824
    assert oracle.cbsegm(75376) == (13, 13, 5824, 0, 5760, 0)
    assert oracle.cbsegm(1000)[0] == 1


ref_only = pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built (build container only)")


@ref_only
def test_oracle_matches_reference_random():
    from srsgpu_testlib import Oracle
    o, r = Oracle(), Ref()
    rng = np.random.default_rng(11)
    Ks = cb_sizes()
    for t in range(60):
        K = int(Ks[rng.integers(len(Ks))])
        impl = int(rng.choice([AUTO, AUTO, GENERIC, SSE, SSE_WINDOW, AVX_WINDOW]))
        if impl == SSE_WINDOW and (K % 8 or K // 8 <= 40):
            impl = AUTO
        if impl == AVX_WINDOW and (K % 16 or K // 16 <= 40):
            impl = AUTO
        sb = int(rng.integers(2)) if impl == AUTO else 0
        bits, llr = make_cb(K, float(rng.uniform(0, 6)), 100 + t, o)
        nsb = o.lib.orc_autoimp_subblocks(K)
        inp = natural_to_sb(llr, K, nsb) if (sb and nsb) else llr
        a = o.tdec_run(impl, sb, inp, K, 9)
        b = r.tdec_run(impl, sb, inp, K, 9)
        assert all((x == y).all() for x, y in zip(a, b)), (K, impl, sb)


@ref_only
def test_oracle_matches_reference_saturation():
    from srsgpu_testlib import Oracle
    o, r = Oracle(), Ref()
    rng = np.random.default_rng(12)
    for K in (40, 400, 408, 816, 6144):
        for impl in (AUTO, GENERIC, SSE):
            inp = rng.integers(-32768, 32768, 3 * K + 12).astype(np.int16)
            a = o.tdec_run(impl, 0, inp, K, 8)
            b = r.tdec_run(impl, 0, inp, K, 8)
            assert all((x == y).all() for x, y in zip(a, b)), (K, impl)


@ref_only
def test_oracle_helpers_match_reference():
    from srsgpu_testlib import Oracle
    o, r = Oracle(), Ref()
    for K in (40, 512, 1024, 6144):
        for nsb in (1, 8, 16):
            if K % nsb == 0:
                a, b = o.interl(K, nsb), r.interl(K, nsb)
                assert (a[0] == b[0]).all() and (a[1] == b[1]).all()
        bits = np.random.default_rng(K).integers(0, 2, K, dtype=np.uint8)
        assert (o.tcod_encode(bits) == r.tcod_encode(bits)).all()
    for tbs in (0, 16, 6120, 6200, 75376, 149776):
        assert o.cbsegm(tbs) == r.cbsegm(tbs)
