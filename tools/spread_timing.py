"""Phase stamps of k_win_spread (timing build: make -C empower-srslte_amd timing; shader clock) over
the drop-in protocol: per half-iteration mode, the cycles from kernel start to the end of the alpha
prepass, of phase A (alpha wave, beta wave), the barrier, phase B and the epilogue, averaged over
code blocks. argv[1]: output JSON."""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("SRSGPU_LIB", os.path.join(REPO, "empower-srslte_amd", "lib", "timing", "libsrsgpu_phy.so"))
sys.path.insert(0, os.path.join(REPO, "empower-srslte_amd"))
import srsgpu_phy as s  # noqa: E402

K = 6144
rng = np.random.default_rng(3)
buf = (ctypes.c_ulonglong * 16)()
names = ["prepass_a", "phaseA_alpha", "phaseA_beta", "barrier", "phaseB", "epilogue"]
acc = {m: {n: [] for n in names} for m in (2, 1, 0)}
d = s.Tdec(K)
d.force_not_sb()
out = np.zeros(K // 8, np.uint8)
for cb in range(12):
    llr = (rng.normal(0, 60, 3 * K + 12)).astype(np.int16)
    d.new_cb(K)
    for h in range(6):
        d.iteration(llr, out)
        s._lib.srsgpu_debug_td_times(buf, 16)
        t = list(buf)
        for b in (0, 1):  # the pair's two workgroups
            v = t[8 * b:8 * b + 8]
            mode = 2 if h == 0 else (1 if h & 1 else 0)
            if cb < 2:
                continue
            acc[mode]["prepass_a"].append(v[1] - v[0])
            acc[mode]["phaseA_alpha"].append(v[2] - v[0])
            acc[mode]["phaseA_beta"].append(v[3] - v[0])
            acc[mode]["barrier"].append(v[4] - v[0])
            acc[mode]["phaseB"].append(v[5] - v[0])
            acc[mode]["epilogue"].append(v[6] - v[0] if v[6] > v[0] else 0)
res = {"unit": "shader clock cycles from kernel start (wave 0 of each workgroup)",
       "modes": {str(m): {n: float(np.median(x)) for n, x in acc[m].items() if x} for m in acc}}
d.free()
print(json.dumps(res))
json.dump(res, open(sys.argv[1], "w"), indent=1)
