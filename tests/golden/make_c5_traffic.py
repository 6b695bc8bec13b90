"""Record the C5 (BASELINE configs[4], mixed-bandwidth multi-cell) traffic table from the srsLTE
reference itself: for every allocation size 1..100 PRB and every MCS 0..28, the TBS
(ra.c:697-731: srslte_ra_tbs_idx_from_mcs, then srslte_ra_tbs_from_idx) and per MCS the
modulation (srslte_ra_mod_from_mcs). Cells of {6, 25, 50, 100} PRB (1.4 / 5 / 10 / 20 MHz) with
allocations of 1..nof_prb PRB span K = 40 .. 6144. bench.py's C5 leg and tests/test_c5_gpu.py
draw their transport blocks from this table; the code block segmentation (cbsegm.c:58-140) of
every TBS is recorded too, and none has filler bits (F = 0), which the reference would refuse
(sch.c:455-458).

    python tests/golden/make_c5_traffic.py   -> tests/golden/c5_traffic.json
"""
import ctypes
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SO = os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle", "_ref", "libsrsref.so")


def main():
    lib = ctypes.CDLL(REF_SO)
    lib.ref_mcs_tbs.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    lib.ref_cbsegm.argtypes = [ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    tbs, segm, mods = [], {}, []
    for prb in range(1, 101):
        row = []
        for mcs in range(29):
            mod = ctypes.c_uint32()
            t = lib.ref_mcs_tbs(mcs, prb, ctypes.byref(mod))
            assert t > 0
            if prb == 1:
                mods.append(mod.value)
            row.append(t)
            if t not in segm:
                s = (ctypes.c_uint32 * 6)()
                assert lib.ref_cbsegm(t, s) == 0
                segm[t] = list(s)
        tbs.append(row)
    assert all(v[5] == 0 for v in segm.values()), "filler bits"
    with open(os.path.join(HERE, "c5_traffic.json"), "w") as f:
        json.dump({"source": "srsLTE ra.c / cbsegm.c via oracle/_ref/libsrsref.so",
                   "mod_by_mcs": mods, "tbs_by_prb_mcs": tbs,
                   "cbsegm_C_C1_K1_C2_K2_F": {str(k): v for k, v in sorted(segm.items())}}, f)
    ks = sorted(set(v[2] for v in segm.values()) | set(v[4] for v in segm.values() if v[3]))
    print("%d TBS values, %d code block sizes, K %d..%d" % (len(segm), len(ks), ks[0], ks[-1]))


if __name__ == "__main__":
    main()
