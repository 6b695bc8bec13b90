#!/bin/bash
# the whole GPU suite after the chest block-sum change, then the TM3 / C3 legs and a TM3 trace
set -e
export TMPDIR=/tmp
TAG=${1:-r03_s19}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python tools/sched_ab.py --legs tm3,c3,coded30 --schedules auto > $O/sched_ab.json 2> $O/sched_ab.err || { tail -20 $O/sched_ab.err; exit 1; }
grep -v amdgpu.ids $O/sched_ab.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_tm3 -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 --no-cpu-baseline --legs tm3 > $O/kt_tm3.log 2>&1
echo "all done"
