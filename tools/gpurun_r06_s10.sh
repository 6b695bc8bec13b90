set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_s10; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 &&
BENCH_AB_ENV=SRSGPU_H0_DECIDE=0 timeout -k 10 300 python -u bench.py --legs envab --steps 20 --warmup 5 --no-cpu-baseline --detail $O/ab_h0.json > $O/ab_h0.log 2> $O/ab_h0.err &&
BENCH_AB_ENV=SRSGPU_H0_DECIDE=0 timeout -k 10 300 python -u bench.py --legs envab --lanes 1 --steps 20 --warmup 5 --no-cpu-baseline --detail $O/ab_h0_1lane.json > $O/ab_h0_1lane.log 2> $O/ab_h0_1lane.err &&
SRSGPU_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --legs c2,c3,tm3,c5 --detail $O/rehearsal_2rank_gloo.json > $O/rehearsal.log 2> $O/rehearsal.err
