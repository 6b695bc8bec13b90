set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_s16; mkdir -p $O
timeout -k 10 300 python -u bench.py --legs feab --steps 20 --warmup 5 --no-cpu-baseline --detail $O/feab.json > $O/feab.log 2> $O/feab.err
