set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_s7; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
BENCH_AB_ROTATE=4 timeout -k 10 300 python -u bench.py --legs tailab --steps 20 --warmup 5 --no-cpu-baseline --detail $O/tailab.json > $O/tailab.log 2> $O/tailab.err &&
timeout -k 10 600 python -u bench.py --legs rxq --steps 10 --warmup 3 --no-cpu-baseline --detail $O/rxq_kcopy.json > $O/rxq_kcopy.log 2> $O/rxq_kcopy.err &&
SRSGPU_RXQ_COPY=dma timeout -k 10 600 python -u bench.py --legs rxq --steps 10 --warmup 3 --no-cpu-baseline --detail $O/rxq_dma.json > $O/rxq_dma.log 2> $O/rxq_dma.err
