#!/bin/bash
# k_chest workgroups-per-grid A/B (SRSGPU_CHEST_PARTS) with tools/kbench.py, each under its own limit
set -e
export TMPDIR=/tmp
TAG=${1:-r04cab}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_chest.py tests/test_extcp.py -m gpu -q --timeout 100 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for p in 1 2 4 8; do
  SRSGPU_CHEST_PARTS=$p timeout -k 10 200 python tools/kbench.py --schedule auto --out $O/kb_parts$p.json > $O/kb_parts$p.log 2>&1 || { tail -20 $O/kb_parts$p.log; exit 1; }
done
SRSGPU_CHEST_PARTS=8 timeout -k 10 200 python -u -m pytest tests/test_chest.py -m gpu -q --timeout 100 --timeout-method thread -p no:cacheprovider > $O/pytest8.log 2>&1 || { tail -20 $O/pytest8.log; exit 1; }
tail -1 $O/pytest8.log
echo all done
