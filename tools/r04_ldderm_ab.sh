#!/bin/bash
# headline A/B of the de-rate-matching loader (SRSGPU_LDERM=tile vs the T4 default), alternating,
# each run under its own limit
set -e
export TMPDIR=/tmp
TAG=${1:-r04lab}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --legs none > $O/t4_$r.json 2> $O/t4_$r.err || { tail -20 $O/t4_$r.err; exit 1; }
  SRSGPU_LDERM=tile timeout -k 10 240 python bench.py --no-cpu-baseline --legs none > $O/tile_$r.json 2> $O/tile_$r.err || { tail -20 $O/tile_$r.err; exit 1; }
done
echo all done
