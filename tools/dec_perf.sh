#!/bin/bash
# decoder iteration loop: decoder parity tests, then the decoder-only bench twice (value spread)
set -e
TAG=${1:-dec}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -m pytest tests/test_tdec_gpu.py tests/test_dlsch_gpu.py -m gpu -x -q -p no:cacheprovider > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pipeline > gpurun_out/$TAG/bench$i.json 2> gpurun_out/$TAG/bench$i.err
  python3 -c "import json;d=json.load(open('gpurun_out/$TAG/bench$i.json'));print(d['value'], d['roofline']['avg_launch_ms'])"
done
