#!/bin/bash
# kernel trace of the full bench (decoder + C3 pipeline) for per-kernel time shares
set -e
TAG=${1:-pipe}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -T -d gpurun_out/$TAG/trace -o kt -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/trace.log 2>&1
cat gpurun_out/$TAG/trace/kt_kernel_stats.csv
