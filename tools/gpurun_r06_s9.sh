set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_s9; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 &&
BENCH_AB_ENV=SRSGPU_H0_DECIDE=0 timeout -k 10 300 python -u bench.py --legs envab --steps 20 --warmup 5 --no-cpu-baseline --detail $O/ab_h0.json > $O/ab_h0.log 2> $O/ab_h0.err &&
BENCH_AB_ENV=SRSGPU_H0_DECIDE=0 timeout -k 10 300 python -u bench.py --legs c2,envab --lanes 1 --steps 20 --warmup 5 --no-cpu-baseline --detail $O/ab_h0_1lane.json > $O/ab_h0_1lane.log 2> $O/ab_h0_1lane.err
