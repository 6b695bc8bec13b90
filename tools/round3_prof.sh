#!/bin/bash
# r03 profiles: kernel-trace stats of the pipeline legs (coded C3 at 30 and 16 dB, C3 fixed-8, C5,
# TM3; separate runs, each under its own limit) and the 2-rank gloo rehearsal
set -e
export TMPDIR=/tmp
TAG=${1:-r03}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp
prof() { # name, bench args...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$n -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 --no-cpu-baseline "$@" > $O/kt_$n.log 2>&1
  echo "$n done"
}
prof coded30 --legs coded --coded-snr 30
prof coded16 --legs coded --coded-snr 16
prof c3 --legs c3
prof c5 --legs c5
prof tm3 --legs tm3
cd $GRAFT_REPO_ROOT
bash tools/dist_rehearsal.sh $TAG
echo all done
