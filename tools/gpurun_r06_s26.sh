set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_s26; mkdir -p $O
timeout -k 10 120 python -u tools/dropin_probe.py $O/dropin.json > $O/dropin.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/prof -o run -- python3 -u tools/dropin_probe.py $O/dropin_prof.json > $O/prof.log 2>&1
