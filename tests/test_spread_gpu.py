"""k_win_spread, the latency form of one windowed half-iteration for a few pairs (DESIGN §5 "Drop-in
latency"), against k_win_bidir / k_win_bidir_run on the same job: decisions after every
half-iteration count and the decoder state (app1 / ext1, reference index space) bit for bit, for
every windowed kind and 1..16 pairs. SRSGPU_SPREAD=0 (knob snapshot reloaded) selects the
k_win_bidir launches for the same job. Both forms are pinned to the oracle and the reference's
golden vectors elsewhere (test_tdec_gpu.py, test_tdec8.py: their single-block and small-batch
cases now run through k_win_spread)."""
import os

import numpy as np
import pytest

from srsgpu_testlib import AUTO, AVX_WINDOW, SSE_WINDOW, make_cb, make_cb8, natural_to_sb

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def s():
    import srsgpu_phy
    return srsgpu_phy


def _run(s, impl, sb, ins, K, nh, spread):
    os.environ["SRSGPU_SPREAD"] = "1" if spread else "0"
    s.knobs_reload()
    b = s.TdecBatch(len(ins), 6144)
    try:
        s.prof_reset()
        s.prof_enable(True)
        out = b.run(impl, sb, ins, K, nh)
        s.prof_enable(False)
        used = s.prof_get("k_win_spread")[1]
        st = None if impl == s.SRSGPU_TDEC_AUTO_8BIT else [b.read_state(i, K) for i in range(len(ins))]
    finally:
        b.close()
        os.environ.pop("SRSGPU_SPREAD", None)
        s.knobs_reload()
    return out, st, used


@pytest.mark.parametrize("impl,K,sb,n", [
    (AUTO, 6144, 0, 1), (AUTO, 6144, 1, 3), (AUTO, 6144, 0, 32), (AUTO, 4096, 1, 2),
    (AVX_WINDOW, 1024, 0, 5), (AVX_WINDOW, 768, 0, 1), (SSE_WINDOW, 6144, 0, 2), (SSE_WINDOW, 512, 0, 7),
    (16, 6144, 1, 3), (16, 6144, 0, 1), (16, 2048, 0, 4)])
def test_spread_equals_bidir(s, oracle, impl, K, sb, n):
    rng = np.random.default_rng(K * 7 + n + sb)
    ins = []
    for i in range(n):
        if impl == s.SRSGPU_TDEC_AUTO_8BIT:
            _, llr = make_cb8(K, float(rng.choice([1.0, 3.0])), 77 * K + i, float(rng.choice([8.0, 64.0])), oracle)
            nsb = oracle.lib.orc_autoimp_subblocks_8bit(K)
            x = natural_to_sb(llr, K, nsb) if (sb and nsb >= 16) else llr
        else:
            _, llr = make_cb(K, float(rng.uniform(0.5, 3.0)), int(rng.integers(1 << 30)), oracle)
            nsb = oracle.lib.orc_autoimp_subblocks(K)
            x = natural_to_sb(llr, K, nsb) if (sb and impl == AUTO and nsb) else llr
        ins.append(x.astype(np.int16))
    if impl == AUTO and n == 1:  # full-range inputs: every saturating corner
        x = rng.integers(-32768, 32768, ins[0].size).astype(np.int16)
        ins = [x]
    for nh in (1, 2, 3, 5):
        got, st, used = _run(s, impl, sb, ins, K, nh, True)
        ref, rst, used0 = _run(s, impl, sb, ins, K, nh, False)
        assert used == nh and used0 == 0, (used, used0)
        np.testing.assert_array_equal(got, ref, err_msg="impl=%d K=%d nh=%d" % (impl, K, nh))
        if st is not None:
            for i in range(n):
                assert (st[i][0] == rst[i][0]).all() and (st[i][1] == rst[i][1]).all(), (impl, K, nh, i)


@pytest.mark.parametrize("spread,poll", [("1", "1"), ("1", "0"), ("0", "1")])
def test_spread_dropin_matches(s, oracle, spread, poll):
    """the drop-in protocol (one srslte_tdec_iteration per half-iteration: one k_win_spread launch
    that also writes the decision bytes, its two workgroups per pair meeting on an arrival counter,
    and the host polling the launch's completion word) against the oracle's decisions after every
    half-iteration, several code blocks in a row on one handle; SRSGPU_SPREAD_POLL=0 synchronises the
    stream instead, SRSGPU_SPREAD=0 takes k_win_bidir + k_decide"""
    os.environ["SRSGPU_SPREAD"], os.environ["SRSGPU_SPREAD_POLL"] = spread, poll
    s.knobs_reload()
    try:
        d = s.Tdec(6144)
        d.force_not_sb()
        for i, K in enumerate((6144, 4096, 6144, 1024)):
            _, llr = make_cb(K, 1.0 + 0.3 * i, 4242 + i, oracle)
            ref = oracle.tdec_run(AUTO, 0, llr, K, 8)[0]
            assert d.new_cb(K) == 0
            out = np.zeros(K // 8, np.uint8)
            for h in range(8):
                d.iteration(llr, out)
                assert (out == ref[h]).all(), (spread, poll, K, h)
        d.free()
    finally:
        os.environ.pop("SRSGPU_SPREAD", None)
        os.environ.pop("SRSGPU_SPREAD_POLL", None)
        s.knobs_reload()
