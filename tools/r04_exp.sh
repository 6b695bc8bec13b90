#!/bin/bash
# r04 experiments: GPU tests of the DL-SCH path, then the headline leg alone under schedule A/B and
# 2 / 3 / 4 lanes, and a kernel trace of the headline. Each GPU step under its own time limit.
set -e
export TMPDIR=/tmp
TAG=${1:-r04x}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_dlsch_gpu.py tests/test_llr8_gpu.py tests/test_pipeline_gpu.py tests/test_ulsch.py tests/test_c5_gpu.py tests/test_tdec_gpu.py tests/test_chest.py tests/test_ofdm.py tests/test_capi.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for L in 2 3 4; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --legs none --ab-headline --lanes $L --steps 20 > $O/head_l$L.json 2> $O/head_l$L.err || { tail -20 $O/head_l$L.err; exit 1; }
  echo lanes $L done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_headline -o kt -- python3 bench.py --no-cpu-baseline --legs none --steps 20 > $O/trace_headline.log 2>&1 || { tail -20 $O/trace_headline.log; exit 1; }
echo all done
