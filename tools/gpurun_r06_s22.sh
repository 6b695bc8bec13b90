set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_s22; mkdir -p $O
SRSGPU_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --legs c2,c3,tm3,c5 --detail $O/rehearsal_2rank_gloo.json > $O/rehearsal.log 2> $O/rehearsal.err
