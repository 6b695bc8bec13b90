"""Per-launch HBM traffic of the decoder kernel from two rocprofv3 PMC passes (FETCH_SIZE and
WRITE_SIZE, collected separately as MI355X_MICROARCH.md's HBM section prescribes) of
`bench.py --no-pipeline`. Writes the profiles/*pmc_traffic*.json that bench.py reads into
roofline.traffic.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch. The guide's x2 correction applies to 16-B/lane
streaming reads only; the decoder reads 8-B (short4) and 4-B lanes, which the guide lists as
uncalibrated, so the raw counter is reported and the correction is recorded as not applied.

usage: python3 tools/pmc_traffic.py <fetch_csv> <write_csv> <out_json>
"""
import csv
import json
import sys

KERNEL = "k_win_bidir"


def per_launch(path, counter):
    """counter summed over its instance rows per dispatch, averaged over the kernel's dispatches"""
    per = {}
    for r in csv.DictReader(open(path)):
        if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
            per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return sum(per.values()) / len(per), len(per)


fetch_kib, nf = per_launch(sys.argv[1], "FETCH_SIZE")
write_kib, nw = per_launch(sys.argv[2], "WRITE_SIZE")
alg = 6 * 4096 * 6144
out = {
    "workload": "batched_turbo_decode_4096xK6144_8halfits",
    "kernel": KERNEL,
    "launches": [nf, nw],
    "fetch_bytes_per_launch": round(fetch_kib * 1024),
    "write_bytes_per_launch": round(write_kib * 1024),
    "hbm_bytes_per_launch": round((fetch_kib + write_kib) * 1024),
    "alg_bytes_per_launch": alg,
    "traffic_over_alg": round((fetch_kib + write_kib) * 1024 / alg, 3),
    "fetch_x2_correction": "not applied (8-B and 4-B lane accesses are uncalibrated on gfx950)",
}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out))
