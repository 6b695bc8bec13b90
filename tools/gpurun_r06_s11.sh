set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_s11; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 &&
BENCH_AB_ENV=SRSGPU_LDERM_FAST=0 timeout -k 10 300 python -u bench.py --legs envab --steps 20 --warmup 5 --no-cpu-baseline --detail $O/ab_ldf.json > $O/ab_ldf.log 2> $O/ab_ldf.err &&
BENCH_AB_ENV=SRSGPU_LDERM_FAST=0 timeout -k 10 300 python -u bench.py --legs envab --lanes 1 --steps 20 --warmup 5 --no-cpu-baseline --detail $O/ab_ldf_1lane.json > $O/ab_ldf_1lane.log 2> $O/ab_ldf_1lane.err &&
BENCH_AB_ENV=SRSGPU_DECIDE_WORDS=0 timeout -k 10 300 python -u bench.py --legs envab --lanes 1 --steps 20 --warmup 5 --no-cpu-baseline --detail $O/ab_dw_1lane.json > $O/ab_dw_1lane.log 2> $O/ab_dw_1lane.err
