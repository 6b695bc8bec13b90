#!/bin/bash
# decoder iteration: parity tests, headline timing, kernel trace, phase timing (debug build)
set -e
TAG=${1:-dec}
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_tdec_gpu.py tests/test_tdec8.py tests/test_dlsch_gpu.py tests/test_c5_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pipeline > $O/bench.json
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['roofline']['avg_launch_ms'], d.get('decoder_8bit',{}).get('mbps'))"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -T -d $O/trace -o kt -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pipeline > $O/trace.log 2>&1
grep -E "k_win|k_decide|k_load" $O/trace/kt_kernel_stats.csv | cut -c1-120
if [ -f empower-srslte_amd/lib/timing/libsrsgpu_phy.so ]; then timeout -k 10 120 python3 tools/td_timing.py > $O/phase.txt 2>&1; cat $O/phase.txt; fi
