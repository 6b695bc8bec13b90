#!/bin/bash
# GPU record of selected test files only (fast iteration); stops at the first failure
set -e
export TMPDIR=/tmp
TAG=${1:-subset}
shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest "$@" -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
