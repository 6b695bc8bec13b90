"""Per-kernel durations of a pipeline leg from a rocprofv3 kernel trace, per 512-subframe stream
batch, with the HBM fraction of the kernel's algorithmic bytes.

  python tools/kstats.py gpurun_out/<tag>/kt_coded30/kt_kernel_trace.csv [--c3]

The bench runs the decoder headline and the traffic synthesis first: only kernels from the leg's
first receive FFT on are counted. A leg's kernels run once per stream batch: the count of
k_tb_finish launches is the number of stream batches.
"""
import argparse
import csv
from collections import defaultdict

HBM = 8000.0  # GB/s

# algorithmic bytes per launch of one 512-subframe C3 stream batch (20 MHz SISO, 64QAM, TBS 75376)
SF = 512
C3_BYTES = {
    "k_ofdm_rx_c": SF * (229376 + 134400),     # samples in (CPs skipped) + grid out
    "k_chest": SF * (6400 + 134400),           # pilots in + estimates out
    "k_pdsch_llr": SF * (120000 + 120000 + 180000),
    "k_derm": SF * (180000 + 482000),
    "k_load_sb": SF * 13 * 5824 * 12,         # 6 B in + 6 B out per info bit
    "k_tb_finish": SF * 2 * 9422,             # TB bytes out + the decisions they come from
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--c3", action="store_true", help="HBM fractions with the C3 stream batch's bytes")
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    # the leg starts at its first receive FFT (the headline and the traffic synthesis run before)
    t0 = min(int(r["Start_Timestamp"]) for r in rows if "k_ofdm_rx" in r["Kernel_Name"])
    by = defaultdict(list)
    for r in rows:
        if int(r["Start_Timestamp"]) < t0:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("srsgpu::", "")
        by[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    nb = max(1, len(by.get("k_tb_finish", [])))
    print(f"stream batches (k_tb_finish launches): {nb}")
    tot = 0.0
    for name, d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        if name.startswith("__amd") or "at::native" in name or name.startswith("k_win_bidir_run"):
            continue
        per_batch = sum(d) / nb
        tot += per_batch
        key = next((k for k in C3_BYTES if name.startswith(k)), None) if args.c3 else None
        frac = ""
        if key:
            avg = sum(d) / len(d)
            frac = f"  {C3_BYTES[key] / (avg * 1e-6) / 1e9:7.0f} GB/s = {C3_BYTES[key] / (avg * 1e-6) / 1e9 / HBM:.2f} of HBM"
        print(f"{name:40s} launches {len(d):6d}  avg {sum(d) / len(d):8.1f} us  per batch {per_batch:8.1f} us{frac}")
    print(f"sum per stream batch (serial): {tot:.1f} us")


if __name__ == "__main__":
    main()
