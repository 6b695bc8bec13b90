#!/bin/bash
# r03 headline decoder profile: kernel stats + FETCH/WRITE + SQ passes (separate runs)
set -e
TAG=r03_s3
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp
B="$R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pipeline"
timeout -k 10 300 python3 $B > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $B > $OUT/kt.log 2>&1
B2="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pipeline"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/$c -o pmc -- python3 $B2 > $OUT/$c.log 2>&1
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU --kernel-trace --output-format csv -d $OUT/sq -o pmc -- python3 $B2 > $OUT/sq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $OUT/tcc -o pmc -- python3 $B2 > $OUT/tcc.log 2>&1
cd $R
python3 tools/pmc_traffic.py $OUT/FETCH_SIZE/pmc_counter_collection.csv $OUT/WRITE_SIZE/pmc_counter_collection.csv $OUT/${TAG}_pmc_traffic.json
python3 tools/pmc_summary.py $OUT/sq/pmc_counter_collection.csv > $OUT/sq.txt
python3 tools/pmc_summary.py $OUT/tcc/pmc_counter_collection.csv > $OUT/tcc.txt
echo done
