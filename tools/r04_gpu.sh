#!/bin/bash
# r04 GPU record: the whole -m gpu suite, smoke, the default bench, and a kernel trace (--stats) of
# the headline leg (BASELINE configs[2]). Every GPU step under its own time limit; stops at the first
# failure.  Usage: tools/r04_gpu.sh TAG [bench|nobench] [trace]
set -e
export TMPDIR=/tmp
TAG=${1:-r04}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
if [ "${2:-bench}" = bench ]; then
  timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  echo bench done
fi
if [ "${3:-}" = trace ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_headline -o kt -- python3 bench.py --no-cpu-baseline --no-pipeline --steps 20 > $O/trace_headline.log 2>&1 || { tail -20 $O/trace_headline.log; exit 1; }
  echo headline trace done
fi
if [ "${4:-}" = pmc ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_$c -o pmc -- python3 bench.py --no-cpu-baseline --legs none --steps 3 --warmup 1 > $O/pmc_$c.log 2>&1 || { tail -5 $O/pmc_$c.log; exit 1; }
  done
  python3 tools/pmc_pipeline.py $O/pmc_FETCH_SIZE/pmc_counter_collection.csv $O/pmc_WRITE_SIZE/pmc_counter_collection.csv $O/pmc_pipeline.json
fi
echo all done
