"""Host (enqueue) cost of each call of the headline step, per lane: the OFDM, estimator, PDSCH LLR,
softbuffer reset and DL-SCH calls of srsgpu_traffic.MixedCells, timed one by one around the ctypes
call over many steps with the GPU running asynchronously (as in bench.py's headline: 2 lanes, four
descriptor sets in turn). Prints microseconds per call and per step; JSON to argv[1] if given."""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "empower-srslte_amd"))
import srsgpu_traffic as tr  # noqa: E402

dev = torch.device("cuda:0")
table = json.load(open(os.path.join(REPO, "tests", "golden", "c5_traffic.json")))
lanes, rotate, steps = 2, int(os.environ.get("ROTATE", "4")), 60
ms = []
for li in range(lanes):
    st = torch.cuda.Stream(dev)
    ms.append(tr.MixedCells(table, 1024, torch, dev, seed=22, stream=st.cuda_stream, snr_db=20.0,
                            keep=list(range(li, 1024, lanes)), prbs=(100,), mcs=28, full_band=True, rotate=rotate))
torch.cuda.synchronize()
acc = {}


def timed(name, f):
    t = time.perf_counter()
    r = f()
    acc[name] = acc.get(name, 0.0) + time.perf_counter() - t
    assert r == 0 or r is None, (name, r)


def step(m):
    m.cur = (m.cur + 1) % m.rotate
    for c in m.cells:
        n, gsz, N = c["n"], c["gsz"], c["N"]
        timed("ofdm_rx", lambda: c["ofdm"].rx_dev(n, c["x"].data_ptr(), 15 * N, c["grid"].data_ptr(), gsz))
        timed("chest", lambda: c["chest"].estimate_dev(c["sf_idx"], c["grid"].data_ptr(), gsz, c["ce"].data_ptr(),
                                                       c["noise"].data_ptr()))
        timed("pdsch_llr", lambda: c["pd"].llr_dev(c["sfs_rot"][m.cur], c["grid"].data_ptr(), c["ce"].data_ptr(),
                                                   gsz, m.d_e.data_ptr(), c["e_offs"]))
    timed("sb_reset", lambda: m.dlsch.reset_range(m.cur * m.ntb, m.ntb))
    timed("dlsch", lambda: m.dlsch.decode_dev(m.tb_rot[m.cur], m.d_e.data_ptr(), m.d_data.data_ptr(), m.max_halfits,
                                              m.d_ret.data_ptr(), m.d_noi.data_ptr()))


for _ in range(8):
    for m in ms:
        step(m)
torch.cuda.synchronize()
acc.clear()
t0 = time.perf_counter()
for _ in range(steps):
    for m in ms:
        step(m)
host = time.perf_counter() - t0
torch.cuda.synchronize()
wall = time.perf_counter() - t0
out = {"rotate": rotate, "lanes": lanes, "steps": steps,
       "us_per_call": {k: round(v / steps / lanes * 1e6, 1) for k, v in acc.items()},
       "host_us_per_step": round(host / steps * 1e6, 1), "wall_us_per_step": round(wall / steps * 1e6, 1)}
print(json.dumps(out))
if len(sys.argv) > 1:
    json.dump(out, open(sys.argv[1], "w"), indent=1)
for m in ms:
    m.close()
