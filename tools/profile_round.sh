#!/bin/bash
# GPU-box profiling recipe (run from the repo root via gpurun):
#   1. kernel trace + stats (per-kernel durations)
#   2. separate --pmc passes for HBM traffic (FETCH_SIZE, WRITE_SIZE) and SQ issue/stall counters
# Output goes to gpurun_out/$TAG; tools/summarise_profile.py condenses it into profiles/.
set -e
TAG=${1:-prof}
STEPS=${STEPS:-5}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
BENCH="python3 bench.py --steps $STEPS --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -T -d $OUT/trace -o kt -- $BENCH > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -T -d $OUT/pmc_fetch -o pmc -- $BENCH > $OUT/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -T -d $OUT/pmc_write -o pmc -- $BENCH > $OUT/pmc_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -T -d $OUT/pmc_sq -o pmc -- $BENCH > $OUT/pmc_sq.log 2>&1
echo done
