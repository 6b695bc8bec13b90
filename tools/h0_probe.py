"""Device time per 1024-subframe batch of the headline's DL-SCH kernels (one stream, one engine, no
tail stream), from the library's HIP-event scopes: an A/B harness for experimental library builds
(SRSGPU_LIB=.../lib/xp/NAME/libsrsgpu_phy.so). Prints one JSON line; argv[1]: output file."""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "empower-srslte_amd"))
import srsgpu_phy as s  # noqa: E402
import srsgpu_traffic as tr  # noqa: E402

dev = torch.device("cuda:0")
table = json.load(open(os.path.join(REPO, "tests", "golden", "c5_traffic.json")))
m = tr.MixedCells(table, 1024, torch, dev, seed=22, snr_db=20.0, prbs=(100,), mcs=28, full_band=True)
for _ in range(5):
    m.step()
torch.cuda.synchronize()
s.prof_reset()
s.prof_enable(True)
n = 10
for _ in range(n):
    m.step()
torch.cuda.synchronize()
s.prof_enable(False)
out = {"lib": s.LIB_PATH}
for k in ("k_ofdm_rx", "k_chest", "k_pdsch_llr", "k_ldderm", "k_win_bidir_h0", "k_decide", "k_win_bidir_es", "k_tb_finish"):
    ms, cnt = s.prof_get(k)
    out[k] = round(ms / n, 4)
print(json.dumps(out))
if len(sys.argv) > 1:
    json.dump(out, open(sys.argv[1], "w"))
m.close()
