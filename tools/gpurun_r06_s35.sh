set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_s35; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_spread_gpu.py tests/test_tdec_gpu.py tests/test_tdec8.py > $O/pytest.log 2>&1 || exit 1
for i in 1 2 3; do timeout -k 10 120 python -u tools/dropin_probe.py $O/dropin_$i.json > $O/dropin_$i.log 2>&1 || exit 1; done
