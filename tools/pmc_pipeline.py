"""Per-kernel HBM traffic of a pipeline leg from two rocprofv3 PMC passes (FETCH_SIZE and
WRITE_SIZE, separate runs as MI355X_MICROARCH.md's HBM section prescribes), against bench.py's
algorithmic bytes (ALG_BYTES_PER_SF) per stream batch of the C3 leg (512 subframes with two lanes,
1024 with one: the optional fourth argument).

FETCH_SIZE / WRITE_SIZE are KiB per dispatch. gfx950 reports half the bytes of wide coalesced
streaming reads in FETCH_SIZE (the guide's x2 correction): both the raw and the doubled value are
listed. Only kernels launched once per stream batch are tabulated (k_decide / per-half-iteration
decoders vary per launch).

usage: python3 tools/pmc_pipeline.py <fetch_csv> <write_csv> <out_json> [subframes_per_launch]
"""
import csv
import json
import sys
from collections import defaultdict

SF = 512  # subframes per stream batch of the C3 legs (default: 2 streams x 512 = 1024 per step)
NLLR, NRE = 90000, 15000
KS = [5824] * 13
ALG = {  # bytes per subframe, as bench.py ALG_BYTES_PER_SF (N = 2048, compact estimate rows)
    "k_ofdm_rx": 14 * 2048 * 8 + 14 * 1200 * 8,
    "k_chest": 800 * 8 + 4 * 1200 * 8 + 4,
    "k_pdsch_llr": NRE * 8 + 4 * 1200 * 8 + NLLR * 2,
    "k_load_derm": NLLR * 2 + 6 * sum(KS),
    "k_tb_finish": sum(k // 8 for k in KS) + 75376 // 8,
}


def per_kernel(path, counter):
    per = defaultdict(dict)  # kernel -> dispatch -> value
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("srsgpu::", "")
        d = per[n]
        d[r["Dispatch_Id"]] = d.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return {k: (sum(v.values()) / len(v), len(v)) for k, v in per.items()}


def main():
    sf = int(sys.argv[4]) if len(sys.argv) > 4 else SF
    fetch, write = per_kernel(sys.argv[1], "FETCH_SIZE"), per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f, nf = fetch.get(k, (0.0, 0))
        w, nw = write.get(k, (0.0, 0))
        base = next((a for a in ALG if k.startswith(a)), None)
        row = {"fetch_kib_raw": round(f, 1), "fetch_bytes_x2": int(2 * f * 1024), "write_bytes": int(w * 1024),
               "dispatches": [nf, nw]}
        if base:
            alg = ALG[base] * sf
            row["alg_bytes"] = alg
            row["subframes_per_launch"] = sf
            row["traffic_over_alg"] = round((2 * f + w) * 1024 / alg, 2)
        out[k] = row
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    for k, r in out.items():
        print("%-45s fetch x2 %8.1f MB  write %8.1f MB  %s" % (k[:45], r["fetch_bytes_x2"] / 1e6, r["write_bytes"] / 1e6,
                                                          ("traffic/alg %.2f" % r["traffic_over_alg"]) if "alg_bytes" in r else ""))


if __name__ == "__main__":
    main()
