"""Record golden turbo-decoder vectors from the srsLTE reference itself.

Runs in the build container only (needs oracle/_ref/libsrsref.so, built from the reference's
own sources by `make -C oracle ref`). For every case it stores the int16 input LLRs (synthetic:
random bits -> turbo encoder -> BPSK/AWGN -> int16, our own PRNG) and what the reference
produced: the hard decision after every half-iteration and the final app1/ext1 arrays
(decoder-internal, sub-block index space for windowed decoders), or for early-stop cases the
decoded bytes, CRC verdict and number of half-iterations (sch.c:356-391 loop).

    python tests/golden/make_golden.py        -> tests/golden/tdec_golden.npz
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from srsgpu_testlib import (AUTO, AVX_WINDOW, CRC24A, CRC24B, GENERIC, SSE, SSE_WINDOW, Oracle,  # noqa
                            Ref, make_cb, make_crc_cb, natural_to_sb)


def main():
    o, r = Oracle(), Ref()
    arrays, manifest = {}, []
    # (impl, K, sb_layout, ebno, halfits): AUTO covers all three reference decoders and both
    # input layouts; manual types pin each decoder on its own, incl. GENERIC (config 1).
    cases = []
    for K in (40, 128, 400, 408, 512, 800, 816, 1056, 2048, 5824, 6144):
        # Eb/N0 in the reference's convention (turbodecoder_test.c:209-217: noise std
        # sqrt(1/(Es/N0)), 3 dB below the textbook one); the waterfall sits near 4 dB.
        for eb in (1.0, 4.0):
            cases.append((AUTO, K, 0, eb, 8))
        if o.lib.orc_autoimp_subblocks(K):
            cases.append((AUTO, K, 1, 4.0, 8))
    cases += [(GENERIC, 6144, 0, 4.0, 8), (GENERIC, 104, 0, 3.0, 10), (SSE, 6144, 0, 4.0, 8),
              (SSE_WINDOW, 6144, 0, 4.0, 8), (SSE_WINDOW, 1024, 0, 2.0, 9),
              (AVX_WINDOW, 6144, 0, 4.5, 8), (AVX_WINDOW, 5824, 0, 3.0, 10)]
    for i, (impl, K, sb, eb, nh) in enumerate(cases):
        bits, llr = make_cb(K, eb, 1000 + i, o)
        nsb = o.lib.orc_autoimp_subblocks(K)
        inp = natural_to_sb(llr, K, nsb) if (sb and impl == AUTO and nsb) else llr
        dec, app1, ext1 = r.tdec_run(impl, sb, inp, K, nh)
        od = o.tdec_run(impl, sb, inp, K, nh)
        assert all((a == b).all() for a, b in zip(od, (dec, app1, ext1))), ("oracle drift", i)
        key = "run%03d" % i
        arrays[key + "_in"] = inp
        arrays[key + "_dec"] = dec
        arrays[key + "_app1"] = app1
        arrays[key + "_ext1"] = ext1
        arrays[key + "_bits"] = bits
        manifest.append(dict(key=key, kind="run", impl=impl, K=K, sb=sb, ebno=eb, halfits=nh))
    # early stop (CRC) cases
    es = [(AUTO, 6144, 0, CRC24B, 4.0, 8), (AUTO, 6144, 1, CRC24B, 4.5, 8),
          (AUTO, 5824, 1, CRC24B, 4.0, 10), (AUTO, 5824, 1, CRC24B, 3.0, 8),
          (AUTO, 1056, 0, CRC24A, 4.0, 10), (AUTO, 800, 1, CRC24B, 4.5, 8),
          (AUTO, 512, 1, CRC24A, 4.5, 8), (AUTO, 256, 0, CRC24A, 4.0, 8),
          (AUTO, 6144, 0, CRC24B, 6.0, 8), (AUTO, 40, 0, CRC24A, 3.5, 6),
          (GENERIC, 2048, 0, CRC24B, 4.5, 8), (SSE, 400, 0, CRC24A, 4.5, 8)]
    for i, (impl, K, sb, poly, eb, mh) in enumerate(es):
        bits, llr = make_crc_cb(K, eb, 5000 + i, poly, o)
        nsb = o.lib.orc_autoimp_subblocks(K)
        inp = natural_to_sb(llr, K, nsb) if (sb and nsb) else llr
        out = np.zeros(K // 8, np.uint8)
        import ctypes
        noi = ctypes.c_uint32(0)
        ok = r.lib.ref_tdec_decode_cb(impl, sb, inp.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)), K, mh,
                                      poly, K, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                      ctypes.byref(noi))
        ook, oout, onoi = o.decode_cb(impl, sb, inp, K, mh, poly, K)
        assert ok == ook and onoi == noi.value and (oout == out).all(), ("oracle drift es", i)
        key = "es%03d" % i
        arrays[key + "_in"] = inp
        arrays[key + "_out"] = out
        arrays[key + "_bits"] = bits
        manifest.append(dict(key=key, kind="early_stop", impl=impl, K=K, sb=sb, poly=poly, ebno=eb,
                             max_halfits=mh, crc_ok=int(ok), noi=int(noi.value)))
    arrays["manifest"] = np.frombuffer(json.dumps(manifest).encode(), np.uint8)
    path = os.path.join(HERE, "tdec_golden.npz")
    np.savez_compressed(path, **arrays)
    print("wrote", path, os.path.getsize(path), "bytes,", len(manifest), "cases")


if __name__ == "__main__":
    main()
