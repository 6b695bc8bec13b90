"""One saturated configuration of bench.py's rx_queue leg, for tracing the queue's pipeline
(rocprofv3 --kernel-trace --memory-copy-trace -- python3 tools/rxq_probe.py OUT.json [BATCH [PACED,...]]):
SC16 samples in registered memory, DMA ingest, 4096 subframes through one queue at max_batch BATCH
(default 1024), no paced runs. Writes the leg's record to OUT.json."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "empower-srslte_amd"))


def main():
    import torch
    import srsgpu_phy as s
    import bench
    os.environ["BENCH_RXQ_VARIANTS"] = "dma"
    b = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    paced = tuple(int(x) for x in sys.argv[3].split(",")) if len(sys.argv) > 3 else ()
    dev = torch.device("cuda:0")
    out = bench.rx_queue_leg(s, torch, dev, batches=(b,), paced_streams=paced)
    json.dump(out, open(sys.argv[1], "w"), indent=1)
    for k, v in out["saturated"].items():
        print(k, v["subframes_per_s"], v["mean_batch"], v["ingest_GBps"], v["dispatcher_us_per_sf"])
    for k, v in out["paced"].items():
        print("paced", k, v["latency_ms_p99"], v["mean_batch"], v["producer_late_ms_max"])


if __name__ == "__main__":
    main()
