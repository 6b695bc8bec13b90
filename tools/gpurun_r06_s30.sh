set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_s30; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_spread_gpu.py tests/test_tdec_gpu.py tests/test_tdec8.py > $O/pytest.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/dropin_probe.py $O/dropin.json > $O/dropin.log 2>&1 || exit 1
SRSGPU_SPREAD_POLL=0 timeout -k 10 120 python -u tools/dropin_probe.py $O/dropin_nopoll.json > $O/dropin_nopoll.log 2>&1 || exit 1
SRSGPU_LIB=$PWD/empower-srslte_amd/lib/xp/split1/libsrsgpu_phy.so timeout -k 10 120 python -u tools/dropin_probe.py $O/dropin_split1.json > $O/dropin_split1.log 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u tools/dropin_probe.py $O/dropin_prof.json > $O/prof.log 2>&1
