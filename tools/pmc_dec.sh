#!/bin/bash
# SQ counters of the decoder kernels on the headline workload (per dispatch, tools/pmc_summary.py)
set -e
TAG=${1:-pmcdec}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
C="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU"
timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -T -d gpurun_out/$TAG/sq -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pipeline > gpurun_out/$TAG/sq.log 2>&1
python3 tools/pmc_summary.py gpurun_out/$TAG/sq/pmc_counter_collection.csv | grep -E "k_win"
