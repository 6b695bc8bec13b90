"""Host time per API call of the C5 receive step (GPU box diagnostic): how long each call takes
to return (no synchronisation), against the GPU time of the whole step."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "empower-srslte_amd"))
import torch  # noqa: E402
import srsgpu_traffic as tr  # noqa: E402

table = json.load(open(os.path.join(REPO, "tests", "golden", "c5_traffic.json")))
dev = torch.device("cuda", 0)
for kind in ("c5", "coded"):
    if kind == "c5":
        m = tr.MixedCells(table, 1024, torch, dev, seed=21, snr_db=20.0)
    else:
        m = tr.MixedCells(table, 1024, torch, dev, prbs=(100,), seed=22, snr_db=30.0, mcs=28, full_band=True)
    for _ in range(2):
        m.step()
    torch.cuda.synchronize()
    acc = {}
    t0 = time.perf_counter()
    for _ in range(5):
        for c in m.cells:
            n, gsz, N = c["n"], c["gsz"], c["N"]
            for name, f in (("ofdm", lambda: c["ofdm"].rx_dev(n, c["x"].data_ptr(), 15 * N, c["grid"].data_ptr(), gsz)),
                            ("chest", lambda: c["chest"].estimate_dev(c["sf_idx"], c["grid"].data_ptr(), gsz, c["ce"].data_ptr(), c["noise"].data_ptr())),
                            ("llr", lambda: c["pd"].llr_dev(c["sfs"], c["grid"].data_ptr(), c["ce"].data_ptr(), gsz, m.d_e.data_ptr(), c["e_offs"]))):
                a = time.perf_counter()
                f()
                acc[name] = acc.get(name, 0) + time.perf_counter() - a
        a = time.perf_counter()
        m.decode()
        acc["decode"] = acc.get("decode", 0) + time.perf_counter() - a
    host = time.perf_counter() - t0
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    print(kind, "per step: host %.3f ms, wall %.3f ms;" % (host / 5e-3, wall / 5e-3),
          {k: round(v / 5e-3, 3) for k, v in acc.items()}, flush=True)
    m.close()
