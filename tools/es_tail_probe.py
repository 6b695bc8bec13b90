"""Early-stop tail of the headline batch: how many code blocks still run after each half-iteration.

The headline workload (bench.py run_traffic "c3": 1024 C3 subframes, 20 MHz 64QAM MCS 28, 20 dB,
seed 22) decoded with a budget of m = 1..8 half-iterations; for each m the code blocks whose CRC
passed (softbuffer cb_crc) and the DL-SCH call's time. Passed(m) - Passed(m-1) code blocks stop
after exactly m half-iterations, so the histogram says how long the early-stop launch's
stragglers run. Writes one JSON object to argv[1] (default stdout)."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "empower-srslte_amd"))


def main():
    import torch
    import srsgpu_traffic as tr
    dev = torch.device("cuda:0")
    table = json.load(open(os.path.join(REPO, "tests", "golden", "c5_traffic.json")))
    snr = float(os.environ.get("SNR_DB", "20"))
    m = tr.MixedCells(table, 1024, torch, dev, seed=22, snr_db=snr, prbs=(100,), mcs=28, full_band=True)
    torch.cuda.synchronize()
    ncb = m.ncb
    out = {"workload": "headline c3 1024 sf, %g dB" % snr, "code_blocks": ncb, "per_budget": {}}
    prev = 0
    for h in range(1, 9):
        m.max_halfits = h
        m.front_end()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            m.decode()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 5
        passed = sum(int(m.dlsch.read_cb_crc(m.softbuffer_of(t)).sum()) for t in m.tb_list)
        acked = int((m.d_ret.cpu().numpy() == 0).sum())
        out["per_budget"][str(h)] = {"cbs_passed": passed, "stop_here": passed - prev,
                                     "still_running": ncb - passed, "acked_tbs": acked,
                                     "dlsch_ms": round(dt * 1e3, 4)}
        prev = passed
    m.close()
    s = json.dumps(out, indent=1)
    if len(sys.argv) > 1:
        open(sys.argv[1], "w").write(s)
    print(s)


if __name__ == "__main__":
    main()
