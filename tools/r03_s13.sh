#!/bin/bash
# decoder-side GPU tests, the schedule A/B (auto vs per half-iteration) and kernel traces of the
# coded 30 dB and C5 legs; every GPU step under its own limit, stops at the first failure
set -e
export TMPDIR=/tmp
TAG=${1:-r03_s13}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_tdec_gpu.py tests/test_dlsch_gpu.py tests/test_c5_gpu.py tests/test_ulsch.py tests/test_pipeline_gpu.py tests/test_rx_queue_gpu.py tests/test_ue_dl_gpu.py tests/test_pdsch_gpu.py tests/test_chest.py tests/test_ofdm.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python tools/sched_ab.py --legs c3,coded30,c5 --schedules auto,per_halfit > $O/sched_ab.json 2> $O/sched_ab.err || { tail -20 $O/sched_ab.err; exit 1; }
grep -v amdgpu.ids $O/sched_ab.err
cd /tmp
for n in coded30 c5; do
  if [ $n = c5 ]; then L="--legs c5"; else L="--legs coded --coded-snr 30"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$n -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 --no-cpu-baseline $L > $O/kt_$n.log 2>&1
  echo "$n traced"
done
echo all done
