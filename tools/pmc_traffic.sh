#!/bin/bash
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes over the decoder-only bench, summarised
# into profiles/<tag>_pmc_traffic.json (read by bench.py for roofline.traffic)
set -e
TAG=${1:-r01}
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_$TAG
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_$TAG/$c -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pipeline > gpurun_out/pmc_$TAG/$c.log 2>&1
done
python3 tools/pmc_traffic.py gpurun_out/pmc_$TAG/FETCH_SIZE/pmc_counter_collection.csv gpurun_out/pmc_$TAG/WRITE_SIZE/pmc_counter_collection.csv gpurun_out/pmc_$TAG/${TAG}_pmc_traffic.json
