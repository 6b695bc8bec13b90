#!/bin/bash
# Round GPU record: full parity suite, full bench (CPU baseline included), kernel-trace stats of
# the headline bench, decoder HBM traffic (FETCH_SIZE / WRITE_SIZE passes) and SQ counters.
# Every GPU step under its own time limit; the script stops at the first failure.
set -e
TAG=${1:-round}
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo bench done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -T -d $O/trace_headline -o kt -- python3 bench.py --no-cpu-baseline --no-pipeline > $O/trace_headline.log 2>&1
echo headline trace done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_$c -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pipeline > $O/pmc_$c.log 2>&1
done
python3 tools/pmc_traffic.py $O/pmc_FETCH_SIZE/pmc_counter_collection.csv $O/pmc_WRITE_SIZE/pmc_counter_collection.csv $O/${TAG}_pmc_traffic.json
C="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -T -d $O/sq -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pipeline > $O/sq.log 2>&1
python3 tools/pmc_summary.py $O/sq/pmc_counter_collection.csv > $O/${TAG}_pmc_sq.txt
cat $O/${TAG}_pmc_sq.txt | grep k_win
echo all done
