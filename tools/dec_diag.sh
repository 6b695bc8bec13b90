#!/bin/bash
# decoder diagnosis: phase timing (debug build) + SQ counters of the headline decoder
set -e
TAG=${1:-diag}
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 120 python3 tools/td_timing.py > $O/phase.txt 2>&1
cat $O/phase.txt
C="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU"
timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -T -d $O/sq -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pipeline > $O/sq.log 2>&1
python3 tools/pmc_summary.py $O/sq/pmc_counter_collection.csv | grep -E "k_win"
C2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM"
timeout -k 10 120 rocprofv3 --pmc $C2 --kernel-trace --output-format csv -T -d $O/sq2 -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pipeline > $O/sq2.log 2>&1
python3 tools/pmc_summary.py $O/sq2/pmc_counter_collection.csv | grep -E "k_win"
