#!/bin/bash
# r03 GPU record: the whole -m gpu suite, the default bench, the decoder scaling probe and
# kernel-trace stats of the coded C3 leg at 16 and 30 dB and of the TM3 leg. Every GPU step under its
# own time limit; stops at the first failure.
set -e
export TMPDIR=/tmp
TAG=${1:-r03}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo bench done
echo all done
