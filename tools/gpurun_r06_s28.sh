set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_s28; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_spread_gpu.py tests/test_tdec_gpu.py tests/test_tdec8.py > $O/pytest.log 2>&1 &&
timeout -k 10 120 python -u tools/dropin_probe.py $O/dropin.json > $O/dropin.log 2>&1 &&
SRSGPU_SPREAD=0 timeout -k 10 120 python -u tools/dropin_probe.py $O/dropin_nospread.json > $O/dropin_nospread.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/prof -o run -- python3 -u tools/dropin_probe.py $O/dropin_prof.json > $O/prof.log 2>&1
