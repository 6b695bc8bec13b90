#!/bin/bash
# quick GPU iteration: parity tests, bench, kernel trace + SQ counters for the decoder kernel
set -e
TAG=${1:-quick}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
cat gpurun_out/$TAG/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -T -d gpurun_out/$TAG/trace -o kt -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/trace.log 2>&1
cat gpurun_out/$TAG/trace/kt_kernel_stats.csv
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -T -d gpurun_out/$TAG/pmc_sq -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/pmc_sq.log 2>&1
python3 tools/pmc_summary.py gpurun_out/$TAG/pmc_sq/pmc_counter_collection.csv
