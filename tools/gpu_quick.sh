#!/bin/bash
# decoder parity tests + headline bench (decoder only) + a kernel trace of the headline
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-quick}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_tdec_gpu.py tests/test_tdec8.py tests/test_dlsch_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python bench.py --no-cpu-baseline --no-pipeline > $O/bench.json 2> $O/bench.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o kt -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-pipeline > $O/trace.log 2>&1
head -8 $O/trace/kt_kernel_stats.csv | cut -d, -f1-4
