"""Per-launch HBM traffic of the decoder kernel from two rocprofv3 PMC passes (FETCH_SIZE and
WRITE_SIZE, collected separately as MI355X_MICROARCH.md's HBM section prescribes) of
`bench.py --no-pipeline`. Writes the profiles/*pmc_traffic*.json that bench.py reads into
roofline.traffic.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch. The guide's x2 FETCH_SIZE correction (16-B/lane
streaming reads) is applied: the decoder's dominant reads (SP0 / P1 in T4 layout) are 16 B per
lane; the raw counter is recorded beside it.

usage: python3 tools/pmc_traffic.py <fetch_csv> <write_csv> <out_json>
"""
import csv
import json
import sys

# the fused fixed-iteration decoder (all 8 half-iterations per launch) when the run has it,
# otherwise the per-half-iteration kernel; names matched up to the template argument list
KERNELS = (("k_win_bidir_run", 8), ("k_win_bidir", 1))


def kernel_of(path):
    names = {r["Kernel_Name"] for r in csv.DictReader(open(path))}
    for k, h in KERNELS:
        if any(k + "<" in n or n.endswith(k) for n in names):
            return k, h
    raise SystemExit("no decoder kernel in " + path)


KERNEL, HALFITS = kernel_of(sys.argv[1])


def per_launch(path, counter):
    """counter summed over its instance rows per dispatch, averaged over the kernel's dispatches"""
    per = {}
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        if (KERNEL + "<" in n or n.endswith(KERNEL)) and r["Counter_Name"] == counter:
            per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return sum(per.values()) / len(per), len(per)


fetch_kib, nf = per_launch(sys.argv[1], "FETCH_SIZE")
write_kib, nw = per_launch(sys.argv[2], "WRITE_SIZE")
# SURVEY 8(d) compulsory bytes per launch: (3(K+32)+12)*2 + K/8 per CB per decode, / 8 half-its
alg = ((3 * (6144 + 32) + 12) * 2 + 6144 // 8) * 4096 / 8 * HALFITS
fetch = fetch_kib * 1024 * 2  # gfx950: FETCH_SIZE counts half the bytes of 16-B/lane reads
write = write_kib * 1024
out = {
    "workload": "batched_turbo_decode_4096xK6144_8halfits",
    "kernel": KERNEL,
    "halfits_per_launch": HALFITS,
    "launches": [nf, nw],
    "fetch_size_raw_bytes_per_launch": round(fetch_kib * 1024),
    "fetch_bytes_per_launch": round(fetch),
    "write_bytes_per_launch": round(write),
    "hbm_bytes_per_launch": round(fetch + write),
    "alg_bytes_per_launch": round(alg),
    "traffic_over_alg": round((fetch + write) / alg, 3),
    "fetch_x2_correction": "applied (MI355X_MICROARCH.md HBM: FETCH_SIZE reports half the bytes of "
                           "16-B/lane reads; the decoder's SP0/P1 reads are 16 B/lane, its X2/A reads "
                           "4 B/lane, uncalibrated)",
    "source": sys.argv[3].split("/")[-1],
}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out))
