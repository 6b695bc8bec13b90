set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_s18; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_es_lds_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_esl.log 2>&1 &&
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 &&
BENCH_AB_ENV=SRSGPU_ES_LDS=0 timeout -k 10 300 python -u bench.py --legs envab --steps 20 --warmup 5 --no-cpu-baseline --detail $O/ab_esl.json > $O/ab_esl.log 2> $O/ab_esl.err
