#!/bin/bash
# C5 / coded-traffic iteration: the new tests, then the bench
set -e
TAG=${1:-c5}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_c5_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -5 gpurun_out/$TAG/pytest.log
timeout -k 10 400 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -30 gpurun_out/$TAG/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/$TAG/bench.json'));print(json.dumps({k:d.get(k) for k in ('value','pipeline_coded','pipeline_c5')},indent=1))"
