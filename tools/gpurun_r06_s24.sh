set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_s24; mkdir -p $O
BENCH_AB_ENV=SRSGPU_ES_PRIO=0 timeout -k 10 300 python -u bench.py --legs envab --steps 20 --warmup 5 --no-cpu-baseline --detail $O/ab_esprio.json > $O/ab_esprio.log 2> $O/ab_esprio.err &&
BENCH_AB_ENV=SRSGPU_TAIL_PRIO=0 timeout -k 10 300 python -u bench.py --legs envab --steps 20 --warmup 5 --no-cpu-baseline --detail $O/ab_tailprio.json > $O/ab_tailprio.log 2> $O/ab_tailprio.err &&
BENCH_AB_ENV=SRSGPU_H0_PRIO=1 timeout -k 10 300 python -u bench.py --legs envab --steps 20 --warmup 5 --no-cpu-baseline --detail $O/ab_h0prio.json > $O/ab_h0prio.log 2> $O/ab_h0prio.err
