#!/bin/bash
# GPU record: the given test files (default: the whole -m gpu suite), then the full bench.
# Every GPU step under its own time limit; stops at the first failure.
set -e
export TMPDIR=/tmp
TAG=${1:-check}
shift || true
TESTS=${@:-tests}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest $TESTS -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo bench done
