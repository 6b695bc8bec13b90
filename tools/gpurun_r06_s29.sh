set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_s29; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_spread_gpu.py tests/test_tdec_gpu.py tests/test_tdec8.py > $O/pytest.log 2>&1 || exit 1
for v in main aonly l2 aonly_l2; do
  if [ $v = main ]; then L=$PWD/empower-srslte_amd/lib/libsrsgpu_phy.so; else L=$PWD/empower-srslte_amd/lib/xp/$v/libsrsgpu_phy.so; fi
  SRSGPU_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 -u tools/dropin_probe.py $O/dropin_$v.json > $O/prof_$v.log 2>&1 || exit 1
done
