set -o pipefail
O=gpurun_out/r06_s3; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1 &&
BENCH_AB_ENV=SRSGPU_ES_COMPACT=0 timeout -k 10 300 python -u bench.py --legs envab,cached --steps 20 --warmup 5 --no-cpu-baseline --detail $O/ab_compact.json > $O/ab_compact.log 2> $O/ab_compact.err &&
BENCH_AB_ENV=SRSGPU_EPILOGUE=split timeout -k 10 300 python -u bench.py --legs envab --steps 20 --warmup 5 --no-cpu-baseline --detail $O/ab_epilogue.json > $O/ab_epilogue.log 2> $O/ab_epilogue.err
