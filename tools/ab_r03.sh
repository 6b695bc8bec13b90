#!/bin/bash
# A/B of the round-3 decoder schedules on the pipeline legs: default (early stop fused into one
# launch per half-iteration, two-wave SSE decoder), SRSGPU_ES_CHUNK=2 / 8 (half-iterations per
# early-stop launch), SRSGPU_TDEC_FUSED=0 (per-half-iteration launches + k_decide) and
# SRSGPU_SSE_BIDIR=0 (one-wave SSE decoder). Optionally the decoder GPU tests first (TESTS=1).
# Each run under its own limit; stops at the first failure.
set -e
TAG=${1:-ab}
O=gpurun_out/$TAG
mkdir -p $O
LEGS=${LEGS:-c3,coded,c5}
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
run() { # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --legs $LEGS > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 tools/leg_summary.py $O/$n.json
}
for v in ${VARIANTS:-default chunk2 chunk8 nofused seqsse}; do
  case $v in
    default*) run $v SRSGPU_AB=1 ;;
    chunk2) run $v SRSGPU_ES_CHUNK=2 ;;
    chunk8) run $v SRSGPU_ES_CHUNK=8 ;;
    nofused) run $v SRSGPU_TDEC_FUSED=0 ;;
    seqsse) run $v SRSGPU_SSE_BIDIR=0 ;;
  esac
done
echo all done
