#!/bin/bash
# GPU parity run of the given test files (default: the whole -m gpu suite), one pytest process.
set -e
export TMPDIR=/tmp
TAG=${1:-check}
shift || true
TESTS=${@:-tests}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest $TESTS -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
