set -o pipefail
bash tools/r06_gpu.sh r06_s15 bench trace pmc noc2pmc
