#!/bin/bash
# decoder iteration: decoder + DL-SCH + pipeline parity tests, then headline timing and a kernel trace
set -e
TAG=${1:-dec}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_tdec_gpu.py tests/test_dlsch_gpu.py tests/test_c5_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pipeline > gpurun_out/$TAG/bench.json
python3 -c "import json;d=json.load(open('gpurun_out/$TAG/bench.json'));print(d['value'], d['roofline']['avg_launch_ms'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -T -d gpurun_out/$TAG/trace -o kt -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pipeline > gpurun_out/$TAG/trace.log 2>&1
grep -E "k_win|k_decide|k_load" gpurun_out/$TAG/trace/kt_kernel_stats.csv | cut -c1-200
