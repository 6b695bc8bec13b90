"""Where do windowed-decoder decisions differ from the golden reference? (GPU box debugging aid)
Prints, for a few golden cases, the bit errors after half-iteration 1 by sub-block (chain) and by
step range (first / second half of the chain)."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "empower-srslte_amd"))
import srsgpu_phy as s  # noqa

z = np.load(os.path.join(REPO, "tests", "golden", "tdec_golden.npz"))
man = json.loads(bytes(z["manifest"]).decode())
b = s.TdecBatch(64, 6144)
for c in man:
    if c["kind"] != "run" or c["impl"] != 0 or c["K"] <= 400 or c.get("ebno") != 1.0:
        continue
    K = c["K"]
    nb = s.autoimp_get_subblocks(K)
    L = K // nb
    for h in (1, 2):
        out = b.run(c["impl"], c["sb"], [z[c["key"] + "_in"]], K, h)
        ref = z[c["key"] + "_dec"][h - 1]
        err = np.nonzero(np.unpackbits(out[0]) != np.unpackbits(ref))[0]
        chains = np.bincount(err // L, minlength=nb)
        half = np.bincount((err % L) >= (L // 32) * 16, minlength=2)
        print(c["key"], "K", K, "sb", c["sb"], "halfit", h, "errors", err.size, "by chain",
              chains.tolist(), "first/second half", half.tolist(), "first pos", err[:6].tolist(),
              flush=True)
