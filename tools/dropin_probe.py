"""Where a drop-in srslte_tdec_iteration call spends its time: 16 code blocks of K = 6144, one call
per half-iteration (decode_tb_cb's protocol, sch.c:356-391), against srslte_tdec_run_all (all
half-iterations in one call). Run under rocprofv3 --kernel-trace --memory-copy-trace --stats to split
device time from launch / copy / synchronisation cost. argv[1]: output JSON."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "empower-srslte_amd"))
import srsgpu_phy as s  # noqa: E402

K, NHALF, NCB = 6144, 8, 16
rng = np.random.default_rng(5)
bits = rng.integers(0, 2, (NCB, 3 * K + 12))
llr = np.ascontiguousarray(((2 * bits - 1) * 40 + rng.normal(0, 30, bits.shape)).clip(-2000, 2000).astype(np.int16))
out = np.zeros(K // 8, np.uint8)
d = s.Tdec(K)
d.force_not_sb()


def per_call(rows):
    t0 = time.perf_counter()
    for r in rows:
        d.new_cb(K)
        for _ in range(NHALF):
            d.iteration(r, out)
    return (time.perf_counter() - t0) / (len(rows) * NHALF) * 1e6


def run_all(rows):
    t0 = time.perf_counter()
    for r in rows:
        d.run_all(r, out, NHALF, K)
    return (time.perf_counter() - t0) / len(rows) * 1e6


per_call(llr[:2])
run_all(llr[:2])
res = {"K": K, "half_iterations": NHALF, "code_blocks": NCB,
       "us_per_iteration_call": round(per_call(llr), 2),
       "us_per_run_all_call": round(run_all(llr), 2)}
res["us_per_halfit_in_run_all"] = round(res["us_per_run_all_call"] / NHALF, 2)
d.free()
print(json.dumps(res))
if len(sys.argv) > 1:
    json.dump(res, open(sys.argv[1], "w"), indent=1)
