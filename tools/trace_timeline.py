"""Overlap analysis of a rocprofv3 kernel trace (kt_kernel_trace.csv) of the headline bench.

Takes the last `--kernels` dispatches whose name matches the pipeline's kernels (the timed steps
come last in the trace), and reports per kernel: launches, summed duration, the time it ran
alone on the GPU (no other kernel in flight), and the time the GPU was busy at all, with the
concurrency histogram (how much wall time 0, 1, 2, 3+ kernels were in flight) over the window.
Usage: trace_timeline.py TRACE.csv [--steps N] [--per-step K] [out.json]"""
import argparse
import csv
import json
import re
from collections import defaultdict


def short(name):
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r"<.*", "", n)
    n = n.replace("void ", "").replace("srsgpu::", "")
    return n.strip()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=10, help="timed steps to analyse (the last ones)")
    ap.add_argument("--marker", default="k_tb_finish", help="kernel that ends a lane's step")
    ap.add_argument("--lanes", type=int, default=2)
    ap.add_argument("out", nargs="?")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         int(r["Queue_Id"])))
    rows.sort()
    # window: from the start of the kernel after the (steps*lanes+1)-th last marker to the last marker end
    marks = [i for i, r in enumerate(rows) if r[2] == a.marker]
    need = a.steps * a.lanes
    if len(marks) <= need:
        raise SystemExit("not enough steps in the trace")
    first = marks[-need - 1] + 1
    last = marks[-1]
    win = rows[first:last + 1]
    t0 = min(r[0] for r in win)
    t1 = max(r[1] for r in win)
    ev = []
    for s, e, n, q in win:
        ev.append((s, 1, n))
        ev.append((e, -1, n))
    ev.sort(key=lambda x: (x[0], x[1]))
    active = defaultdict(int)
    hist = defaultdict(float)
    alone = defaultdict(float)
    share = defaultdict(float)  # wall time weighted by 1/concurrency
    prev = t0
    for t, d, n in ev:
        dt = t - prev
        if dt > 0:
            c = sum(active.values())
            hist[min(c, 3)] += dt
            if c == 1:
                only = [k for k, v in active.items() if v][0]
                alone[only] += dt
            for k, v in active.items():
                if v:
                    share[k] += dt * v / c
        active[n] += d
        prev = t
    per = defaultdict(lambda: [0, 0.0])
    for s, e, n, q in win:
        per[n][0] += 1
        per[n][1] += e - s
    wall = t1 - t0
    steps = a.steps
    out = {"window_us": round(wall / 1e3, 1), "steps": steps, "us_per_step": round(wall / 1e3 / steps, 1),
           "concurrency_us_per_step": {str(k): round(v / 1e3 / steps, 1) for k, v in sorted(hist.items())},
           "kernels": {}}
    for n, (cnt, dur) in sorted(per.items(), key=lambda x: -x[1][1]):
        out["kernels"][n] = {"launches_per_step": round(cnt / steps, 2), "us_per_step": round(dur / 1e3 / steps, 1),
                             "avg_us": round(dur / 1e3 / cnt, 1), "alone_us_per_step": round(alone[n] / 1e3 / steps, 1),
                             "wall_share_us_per_step": round(share[n] / 1e3 / steps, 1)}
    s = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(s)
    print(s)


if __name__ == "__main__":
    main()
