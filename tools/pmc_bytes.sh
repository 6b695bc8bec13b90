#!/bin/bash
# HBM traffic per kernel: separate FETCH_SIZE and WRITE_SIZE passes (MI355X_MICROARCH.md §HBM)
set -e
TAG=${1:-bytes}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
for c in FETCH_SIZE WRITE_SIZE TCC_HIT_sum TCC_MISS_sum; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -T -d gpurun_out/$TAG/$c -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/$c.log 2>&1
  python3 tools/pmc_summary.py gpurun_out/$TAG/$c/pmc_counter_collection.csv
done
