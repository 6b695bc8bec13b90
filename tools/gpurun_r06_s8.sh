set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_s8; mkdir -p $O
timeout -k 10 200 python -u tools/host_cost.py $O/host_cost_rot4.json > $O/host_cost.log 2>&1 &&
ROTATE=1 timeout -k 10 200 python -u tools/host_cost.py $O/host_cost_rot1.json >> $O/host_cost.log 2>&1 &&
bash tools/r06_gpu.sh r06_s8 bench trace pmc noc2pmc
