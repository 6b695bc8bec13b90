#!/bin/bash
# End-of-milestone GPU record: full parity suite, full bench (with the CPU baseline), kernel trace
# stats of the full bench, decoder HBM traffic (FETCH_SIZE / WRITE_SIZE passes) and SQ counters.
set -e
TAG=${1:-round}
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo bench done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -T -d $O/trace -o kt -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1
echo trace done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -T -d $O/trace_headline -o kt -- python3 bench.py --no-cpu-baseline --no-pipeline > $O/trace_headline.log 2>&1
echo headline trace done
bash tools/pmc_traffic.sh $TAG > $O/traffic.log 2>&1
echo traffic done
bash tools/pmc_dec.sh ${TAG}_sq > $O/sq.log 2>&1
echo sq done
