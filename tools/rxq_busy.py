"""Copy engine and compute busy time of the queue's saturated runs, from a rocprofv3 kernel +
memory-copy trace of tools/rxq_probe.py (csv output):
    python tools/rxq_busy.py TRACE_DIR [--gap-ms 30]
The timeline is cut into runs at idle gaps longer than --gap-ms (queue setup between modes); per run:
wall, kernel busy (union of kernel intervals), H2D copy busy, both at once, and the copy engine's
idle gaps between consecutive copies (median / p90 / sum)."""
import argparse
import csv
import glob
import os

import numpy as np


def intervals(path, want=None):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if want and not want(r):
                continue
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return sorted(out)


def union(iv):
    res = []
    for a, b in iv:
        if res and a <= res[-1][1]:
            res[-1][1] = max(res[-1][1], b)
        else:
            res.append([a, b])
    return res


def overlap(u, v):
    i = j = 0
    tot = 0
    while i < len(u) and j < len(v):
        a, b = max(u[i][0], v[j][0]), min(u[i][1], v[j][1])
        if a < b:
            tot += b - a
        if u[i][1] < v[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap-ms", type=float, default=30.0)
    a = ap.parse_args()
    kf = glob.glob(os.path.join(a.trace, "**", "*kernel_trace.csv"), recursive=True)
    cf = glob.glob(os.path.join(a.trace, "**", "*memory_copy_trace.csv"), recursive=True)
    ker = sum((intervals(p) for p in kf), [])
    cop = sum((intervals(p, lambda r: "HOST_TO_DEVICE" in r.get("Direction", "")) for p in cf), [])
    allv = union(sorted(ker + cop))
    runs, cur = [], [allv[0]]
    for iv in allv[1:]:
        if iv[0] - cur[-1][1] > a.gap_ms * 1e6:
            runs.append((cur[0][0], cur[-1][1]))
            cur = []
        cur.append(iv)
    runs.append((cur[0][0], cur[-1][1]))
    for r0, r1 in runs:
        k = union([iv for iv in ker if r0 <= iv[0] < r1])
        c = union([iv for iv in cop if r0 <= iv[0] < r1])
        wall = (r1 - r0) / 1e6
        if wall < 5:
            continue
        kb = sum(b - x for x, b in k) / 1e6
        cb = sum(b - x for x, b in c) / 1e6
        both = overlap(k, c) / 1e6
        gaps = np.array([c[i + 1][0] - c[i][1] for i in range(len(c) - 1)]) / 1e6 if len(c) > 1 else np.zeros(1)
        print("run %.1f ms: kernels busy %.1f ms (%.0f%%), H2D busy %.1f ms (%.0f%%), both %.1f ms; "
              "%d copy spans, gaps median %.3f p90 %.3f sum %.1f ms" %
              (wall, kb, 100 * kb / wall, cb, 100 * cb / wall, both, len(c), np.median(gaps),
               np.percentile(gaps, 90), gaps.sum()))


if __name__ == "__main__":
    main()
