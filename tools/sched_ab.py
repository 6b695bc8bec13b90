"""In-process A/B of the decoder launch schedules (srsgpu_tdec_set_schedule) on the subframe legs:
the same inputs, the schedules timed in turn for several rounds (bench.schedule_ab). Prints one
JSON object: per leg, ms per batch per schedule (each round) and the median.

  python tools/sched_ab.py [--legs c3,coded30,coded16,c5,tm3] [--steps N]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

SCHEDULES = {
    "auto": dict(es_fused=2, es_chunk=8, sse_bidir=1),
    "es_fused8": dict(es_fused=1, es_chunk=8, sse_bidir=1),
    "es_fused1": dict(es_fused=1, es_chunk=1, sse_bidir=1),
    "per_halfit": dict(es_fused=0, es_chunk=8, sse_bidir=1),
    "per_halfit_sse1": dict(es_fused=0, es_chunk=8, sse_bidir=0),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--legs", default="c3,coded30,coded16,c5")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--lanes", type=int, default=2, help="HIP streams the batch is split over")
    ap.add_argument("--schedules", default=None, help="comma-separated subset of the schedules")
    args = ap.parse_args()
    import torch
    import bench
    import srsgpu_phy as s
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    bench.schedule_ab.__defaults__ = (args.reps,)
    sch = SCHEDULES if not args.schedules else {k: SCHEDULES[k] for k in args.schedules.split(",")}
    out = {}
    for leg in args.legs.split(","):
        if leg in ("c3", "tm3"):
            r = bench.run_pipeline(s, torch, dev, args.steps, 2, tm=3 if leg == "tm3" else 1, lanes=args.lanes,
                                   schedules=sch)
        elif leg.startswith("coded"):
            r = bench.run_traffic(s, torch, dev, 2 * args.steps, 2, "c3_coded", snr_db=float(leg[5:]),
                                  lanes=args.lanes, schedules=sch)
        else:
            r = bench.run_traffic(s, torch, dev, 2 * args.steps, 2, "c5", lanes=args.lanes, schedules=sch)
        out[leg] = {"ms_per_batch": r["ms_per_batch"], "nof_iterations_mean": r["nof_iterations_mean"],
                    "schedule_ab": r["schedule_ab"]}
        print(leg, {k: v["median"] for k, v in r["schedule_ab"].items()}, file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
