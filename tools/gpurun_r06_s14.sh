set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_s14; mkdir -p $O
BENCH_AB_ENV=SRSGPU_SPLIT_EARLY=1 timeout -k 10 300 python -u bench.py --legs envab --steps 20 --warmup 5 --no-cpu-baseline --detail $O/ab_split.json > $O/ab_split.log 2> $O/ab_split.err &&
BENCH_AB_ENV=SRSGPU_SPLIT_EARLY=1 timeout -k 10 300 python -u bench.py --legs envab --lanes 2 --steps 20 --warmup 5 --no-cpu-baseline --detail $O/ab_split_2lanes.json > $O/ab_split_2lanes.log 2> $O/ab_split_2lanes.err
