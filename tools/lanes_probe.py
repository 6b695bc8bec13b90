"""Pipeline and traffic legs at 1 / 2 / 4 streams (GPU box diagnostic for bench's lanes)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "empower-srslte_amd"))
import torch  # noqa: E402
import srsgpu_phy as s  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda", 0)
for kind in ("c3_coded", "c5"):
    for lanes in (1, 2, 4):
        r = bench.run_traffic(s, torch, dev, 40, 2, kind, lanes=lanes)
        print(kind, lanes, r["subframes_per_s"], r["ms_per_batch"], r["acked_tbs"], r["tbs"], flush=True)
