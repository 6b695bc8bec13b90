set -o pipefail
O=gpurun_out/r06_s6; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 &&
BENCH_AB_ROTATE=4 BENCH_AB_ENV=SRSGPU_H2D=dma timeout -k 10 300 python -u bench.py --legs envab --steps 20 --warmup 5 --no-cpu-baseline --detail $O/ab_h2d.json > $O/ab_h2d.log 2> $O/ab_h2d.err &&
BENCH_AB_ENV=SRSGPU_DEFER_P1=0 timeout -k 10 300 python -u bench.py --legs envab --steps 20 --warmup 5 --no-cpu-baseline --detail $O/ab_p1.json > $O/ab_p1.log 2> $O/ab_p1.err &&
BENCH_TAIL_PRIO=1 timeout -k 10 300 python -u bench.py --legs tailab --steps 20 --warmup 5 --no-cpu-baseline --detail $O/tailab_prio.json > $O/tailab_prio.log 2> $O/tailab_prio.err &&
timeout -k 10 300 python -u bench.py --legs cached --lanes 3 --steps 20 --warmup 5 --no-cpu-baseline --detail $O/lanes3.json > $O/lanes3.log 2> $O/lanes3.err
