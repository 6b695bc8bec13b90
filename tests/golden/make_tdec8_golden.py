"""Golden vectors of the 8-bit turbo decoding path (srslte_tdec_iteration_8bit, and the manual
8-bit window types through srslte_tdec_iteration) recorded from the srsLTE reference compiled from
its own sources (oracle/_ref/libsrsref.so, target `make -C oracle ref`).

    python tests/golden/make_tdec8_golden.py   -> tests/golden/tdec8_golden.npz

Each case: impl, sb_layout, K, the int8 (or int16) input and the decision bytes after each of 8
half-iterations. Inputs: random bits, turbo encoded, BPSK over AWGN, quantised to int8
(tests/srsgpu_testlib.py awgn_llr8).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from srsgpu_testlib import (AUTO, AVX8_WINDOW, GENERIC, SSE, SSE8_WINDOW, Oracle, Ref,  # noqa: E402
                            make_cb, make_cb8, natural_to_sb)

# (impl, sb_layout, K, Eb/N0, scale): AUTO over every 8-bit regime (16 / 32 sub-blocks, K % 32
# != 0 tail, the int16 fallbacks) plus manual types through both entry points
CASES8 = [(AUTO, 1, 6144, 5.0, 16.0), (AUTO, 0, 6144, 2.0, 40.0), (AUTO, 1, 2112, 5.0, 16.0),
          (AUTO, 1, 848, 5.0, 16.0), (AUTO, 0, 848, 3.0, 60.0), (AUTO, 1, 1024, 5.0, 8.0),
          (AUTO, 1, 40, 3.0, 20.0), (AUTO, 0, 512, 3.0, 20.0), (AUTO, 1, 400, 3.0, 20.0),
          (GENERIC, 1, 1024, 5.0, 16.0), (SSE, 0, 512, 5.0, 16.0)]
CASES16 = [(SSE8_WINDOW, 848), (AVX8_WINDOW, 2112), (AVX8_WINDOW, 6144)]
NHALF = 8


def main():
    o, r = Oracle(), Ref()
    out = {}
    for i, (impl, sb, K, ebno, scale) in enumerate(CASES8):
        _, llr = make_cb8(K, ebno, 100 + i, scale, o)
        nsb = o.lib.orc_autoimp_subblocks_8bit(K)
        inp = natural_to_sb(llr, K, nsb) if (sb and impl == AUTO and nsb >= 16) else llr
        out["c8_%d_meta" % i] = np.array([impl, sb, K], np.int32)
        out["c8_%d_in" % i] = inp
        out["c8_%d_dec" % i] = r.tdec8_run(impl, sb, inp, K, NHALF)
    for i, (impl, K) in enumerate(CASES16):
        _, llr = make_cb(K, 5.0, 200 + i, o)
        llr = (llr // 3).astype(np.int16)  # values beyond int8: the reference truncates
        out["c16_%d_meta" % i] = np.array([impl, 0, K], np.int32)
        out["c16_%d_in" % i] = llr
        out["c16_%d_dec" % i] = r.tdec8_run16(impl, llr, K, NHALF)
    np.savez_compressed(os.path.join(HERE, "tdec8_golden.npz"), **out)
    print("%d + %d cases" % (len(CASES8), len(CASES16)))


if __name__ == "__main__":
    main()
