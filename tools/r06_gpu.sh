#!/bin/bash
# r06 GPU record: the -m gpu suite (or the given test files), smoke, the default bench (compact line +
# detail file), optionally a kernel trace (--stats) of the headline leg with its overlap timeline, the
# pipeline FETCH/WRITE PMC passes, and the FETCH/WRITE passes of the configs[1] decoder (decoder_c2).
# Every GPU step under its own time limit; stops at the first failure.
# Usage: tools/r06_gpu.sh TAG [bench|nobench] [trace|notrace] [pmc|nopmc] [c2pmc|noc2pmc] [TESTS...]
set -e
export TMPDIR=/tmp
TAG=${1:-r06}
MODE=${2:-bench}
TRACE=${3:-notrace}
PMC=${4:-nopmc}
C2PMC=${5:-noc2pmc}
shift 5 || shift $#
TESTS=${@:-tests}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ "$TESTS" != none ]; then
  timeout -k 10 700 python -u -m pytest $TESTS -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if [ "$MODE" = bench ]; then
  timeout -k 10 700 python bench.py --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  echo bench done; wc -c $O/bench.json
fi
if [ "$TRACE" = trace ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_headline -o kt -- python3 bench.py --no-cpu-baseline --legs none --steps 20 --detail $O/trace_detail.json > $O/trace_headline.log 2>&1 || { tail -20 $O/trace_headline.log; exit 1; }
  python3 tools/trace_timeline.py $(find $O/trace_headline -name 'kt_kernel_trace.csv' | head -1) $O/headline_overlap.json --steps 10 > $O/headline_overlap.txt 2>&1 || true
  echo headline trace done
fi
if [ "$PMC" = pmc ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_$c -o pmc -- python3 bench.py --no-cpu-baseline --legs none --steps 3 --warmup 1 --detail $O/pmc_detail.json > $O/pmc_$c.log 2>&1 || { tail -5 $O/pmc_$c.log; exit 1; }
  done
  python3 tools/pmc_pipeline.py $(find $O/pmc_FETCH_SIZE -name 'pmc_counter_collection.csv' | head -1) $(find $O/pmc_WRITE_SIZE -name 'pmc_counter_collection.csv' | head -1) $O/pmc_pipeline.json ${PMC_SF:-1024}
fi
if [ "$C2PMC" = c2pmc ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/c2pmc_$c -o pmc -- python3 bench.py --no-cpu-baseline --no-pipeline --steps 3 --warmup 1 --detail $O/c2pmc_detail.json > $O/c2pmc_$c.log 2>&1 || { tail -5 $O/c2pmc_$c.log; exit 1; }
  done
  python3 tools/pmc_traffic.py $(find $O/c2pmc_FETCH_SIZE -name 'pmc_counter_collection.csv' | head -1) $(find $O/c2pmc_WRITE_SIZE -name 'pmc_counter_collection.csv' | head -1) $O/c2_pmc_traffic.json
fi
echo all done
