set -o pipefail
O=gpurun_out/r06_s2; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -u bench.py --legs rxq --steps 20 --warmup 5 --no-cpu-baseline --detail $O/bench_detail.json > $O/bench.log 2> $O/bench.err &&
BENCH_AB_ENV=SRSGPU_EPILOGUE=split timeout -k 10 300 python -u bench.py --legs envab --steps 20 --warmup 5 --no-cpu-baseline --detail $O/envab_detail.json > $O/envab.log 2> $O/envab.err
