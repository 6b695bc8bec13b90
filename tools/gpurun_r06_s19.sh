set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_s19; mkdir -p $O
BENCH_AB_ENV=SRSGPU_ES_LDS=0 timeout -k 10 300 python -u bench.py --legs envab --lanes 2 --steps 20 --warmup 5 --no-cpu-baseline --detail $O/ab_esl_2lanes.json > $O/ab_esl_2lanes.log 2> $O/ab_esl_2lanes.err
