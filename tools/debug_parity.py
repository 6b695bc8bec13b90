"""List golden cases whose GPU decode differs (GPU box debugging aid)."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "empower-srslte_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import srsgpu_phy as s  # noqa

z = np.load(os.path.join(REPO, "tests", "golden", "tdec_golden.npz"))
man = json.loads(bytes(z["manifest"]).decode())
b = s.TdecBatch(64, 6144)
for c in man:
    if c["kind"] != "run":
        continue
    bad = []
    for h in range(1, c["halfits"] + 1):
        out = b.run(c["impl"], c["sb"], [z[c["key"] + "_in"]], c["K"], h)
        ref = z[c["key"] + "_dec"][h - 1]
        if not (out[0] == ref).all():
            bad.append((h, int(np.unpackbits(out[0] ^ ref).sum())))
    print(c["key"], "impl", c["impl"], "K", c["K"], "sb", c["sb"], "bad(halfit,bits)", bad[:4], flush=True)
