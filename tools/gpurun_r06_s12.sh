set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_s12; mkdir -p $O
timeout -k 10 300 python -u bench.py --legs laneab --steps 20 --warmup 5 --no-cpu-baseline --detail $O/laneab.json > $O/laneab.log 2> $O/laneab.err &&
BENCH_AB_ENV=SRSGPU_ES_PRIO=0 timeout -k 10 300 python -u bench.py --legs envab --steps 20 --warmup 5 --no-cpu-baseline --detail $O/ab_esprio.json > $O/ab_esprio.log 2> $O/ab_esprio.err &&
BENCH_AB_ENV=SRSGPU_TAIL_PRIO=0 timeout -k 10 300 python -u bench.py --legs envab --steps 20 --warmup 5 --no-cpu-baseline --detail $O/ab_tailprio.json > $O/ab_tailprio.log 2> $O/ab_tailprio.err
