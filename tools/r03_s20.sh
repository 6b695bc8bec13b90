#!/bin/bash
# OFDM twiddle preload: OFDM / chest / pipeline parity, coded 30 dB trace and the leg timings
set -e
export TMPDIR=/tmp
TAG=${1:-r03_s20}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_ofdm.py tests/test_chest.py tests/test_pipeline_gpu.py tests/test_rx_queue_gpu.py tests/test_ue_dl_gpu.py tests/test_c5_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_coded30 -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 --no-cpu-baseline --legs coded --coded-snr 30 > $O/kt_coded30.log 2>&1
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python tools/sched_ab.py --legs coded30,c3,c5 --schedules auto > $O/sched_ab.json 2> $O/sched_ab.err || { tail -20 $O/sched_ab.err; exit 1; }
grep -v amdgpu.ids $O/sched_ab.err
echo all done
