set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_s13; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 &&
BENCH_AB_ENV=SRSGPU_LDERM_PP=0 timeout -k 10 300 python -u bench.py --legs envab --steps 20 --warmup 5 --no-cpu-baseline --detail $O/ab_pp.json > $O/ab_pp.log 2> $O/ab_pp.err &&
BENCH_AB_ENV=SRSGPU_SPLIT_EARLY=1 timeout -k 10 300 python -u bench.py --legs envab --steps 20 --warmup 5 --no-cpu-baseline --detail $O/ab_split.json > $O/ab_split.log 2> $O/ab_split.err
