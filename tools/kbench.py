"""Isolated kernel timings of the coded C3 pipeline (BASELINE configs[2] subframes): one stream,
one 512-subframe batch at a time, a device synchronisation after every stage, so every kernel runs
alone on the GPU (the bench's two-stream legs overlap kernels, which inflates each one's duration).
Per stage: milliseconds per batch from the library's HIP events (srsgpu_prof_*), and the HBM
fraction of the kernels with algorithmic bytes (bench.py ALG_BYTES_PER_SF, compact estimate rows).

  python tools/kbench.py [--sf 512] [--reps 20] [--snr 20] [--schedule auto|hybrid|per_halfit|fused8]

Run it under rocprofv3 --kernel-trace --stats for the per-kernel durations of the same launches.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "empower-srslte_amd"))

ALG = {"k_ofdm_rx": 14 * 2048 * 8 + 14 * 1200 * 8, "k_chest": 800 * 8 + 4 * 1200 * 8 + 4,
       "k_pdsch_llr": 15000 * 8 + 4 * 1200 * 8 + 90000 * 2, "k_ldderm": 90000 * 2 + 6 * 13 * 5824}
SCHED = {"auto": dict(es_fused=2, es_chunk=8), "hybrid": dict(es_fused=3, es_chunk=8),
         "per_halfit": dict(es_fused=0), "fused8": dict(es_fused=1, es_chunk=8)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=int, default=512)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--snr", type=float, default=20.0)
    ap.add_argument("--schedule", default="auto")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    import srsgpu_phy as s
    import srsgpu_traffic as tr
    torch.cuda.set_device(0)
    s.set_schedule(**SCHED[a.schedule])
    table = json.load(open(os.path.join(REPO, "tests", "golden", "c5_traffic.json")))
    m = tr.MixedCells(table, a.sf, torch, torch.device("cuda", 0), seed=22, snr_db=a.snr, prbs=(100,), mcs=28,
                      full_band=True)
    c = m.cells[0]
    n, gsz, N = c["n"], c["gsz"], c["N"]
    stages = {
        "ofdm": lambda: c["ofdm"].rx_dev(n, c["x"].data_ptr(), 15 * N, c["grid"].data_ptr(), gsz),
        "chest": lambda: c["chest"].estimate_dev(c["sf_idx"], c["grid"].data_ptr(), gsz, c["ce"].data_ptr(),
                                                 c["noise"].data_ptr()),
        "pdsch": lambda: c["pd"].llr_dev(c["sfs"], c["grid"].data_ptr(), c["ce"].data_ptr(), gsz,
                                         m.d_e.data_ptr(), c["e_offs"]),
        "dlsch": lambda: (m.decode(), 0)[1],
    }
    for _ in range(3):  # warm up (and bring the clocks up)
        for f in stages.values():
            assert f() == 0
    torch.cuda.synchronize()
    res = {}
    for name, f in stages.items():
        s.prof_reset()
        s.prof_enable(True)
        t0 = time.perf_counter()
        host = 0.0
        for _ in range(a.reps):
            h0 = time.perf_counter()
            assert f() == 0
            host += time.perf_counter() - h0
            torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / a.reps * 1e3
        s.prof_enable(False)
        ks = {}
        for k in ("k_ofdm_rx", "k_chest", "k_gold", "k_pdsch_llr", "k_ldderm", "k_derm", "k_load", "k_win_bidir",
                  "k_decide", "k_es_bytes", "k_tb_finish", "k_rows_late"):
            ms, cnt = s.prof_get(k)
            if cnt:
                e = {"ms": round(ms / a.reps, 4), "launches": round(cnt / a.reps, 2)}
                if k in ALG:
                    e["hbm_frac"] = round(ALG[k] * n / (ms / a.reps / 1e3) / 8e12, 3)
                ks[k] = e
        res[name] = {"wall_ms": round(wall, 4), "host_ms": round(host / a.reps * 1e3, 4), "kernels": ks}
    acks, good, noi = m.check()
    out = {"subframes": n, "snr_db": a.snr, "schedule": a.schedule, "acked": acks, "good": good,
           "nof_iterations_mean": noi, "stages": res,
           "serial_ms_per_batch": round(sum(v["wall_ms"] for v in res.values()), 4)}
    m.close()
    js = json.dumps(out, indent=1)
    print(js)
    if a.out:
        open(a.out, "w").write(js)


if __name__ == "__main__":
    main()
