#!/bin/bash
# isolated kernel timings (tools/kbench.py) under schedule / OFDM variants, plus a kernel trace of
# the default one. Each GPU step under its own time limit.
set -e
export TMPDIR=/tmp
TAG=${1:-r04kb}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 540 python -u -m pytest tests/test_dlsch_gpu.py tests/test_llr8_gpu.py tests/test_c5_gpu.py tests/test_ce_rows_gpu.py tests/test_chest.py tests/test_ofdm.py tests/test_pipeline_gpu.py tests/test_ulsch.py tests/test_txdiv.py tests/test_tx_mimo_gpu.py tests/test_uci.py tests/test_pdcch.py tests/test_pcfich.py tests/test_extcp.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python tools/kbench.py --schedule auto --out $O/kb_auto.json > $O/kb_auto.log 2>&1 || { tail -20 $O/kb_auto.log; exit 1; }
SRSGPU_OFDM_TW=table timeout -k 10 200 python tools/kbench.py --schedule auto --out $O/kb_twtable.json > $O/kb_twtable.log 2>&1 || { tail -20 $O/kb_twtable.log; exit 1; }
SRSGPU_OFDM_TW=table timeout -k 10 200 python -u -m pytest tests/test_ofdm.py tests/test_extcp.py -m gpu -q -k ofdm --timeout 100 --timeout-method thread -p no:cacheprovider > $O/pytest_twtable.log 2>&1 || { tail -20 $O/pytest_twtable.log; exit 1; }
tail -1 $O/pytest_twtable.log
SRSGPU_LDERM=tile timeout -k 10 200 python tools/kbench.py --schedule auto --out $O/kb_ldtile.json > $O/kb_ldtile.log 2>&1 || { tail -20 $O/kb_ldtile.log; exit 1; }
timeout -k 10 200 python tools/kbench.py --schedule per_halfit --out $O/kb_perhalfit.json > $O/kb_perhalfit.log 2>&1 || { tail -20 $O/kb_perhalfit.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_kb -o kt -- python3 tools/kbench.py --schedule auto > $O/trace_kb.log 2>&1 || { tail -20 $O/trace_kb.log; exit 1; }
echo all done
