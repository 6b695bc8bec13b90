set -o pipefail
bash tools/r06_gpu.sh r06_s21 bench trace pmc noc2pmc
