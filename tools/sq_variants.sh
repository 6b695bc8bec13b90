#!/bin/bash
# SQ counters of the decoder kernel for each library variant under empower-srslte_amd/lib/xp/ and
# the product library (diagnostic only)
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-sq}
mkdir -p $O
C="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU"
C2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS"
for v in $(ls empower-srslte_amd/lib/xp) prod; do
  L=empower-srslte_amd/lib/xp/$v/libsrsgpu_phy.so
  [ $v = prod ] && L=empower-srslte_amd/lib/libsrsgpu_phy.so
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/$v -o a -- python3 tools/dec_time.py $L > $O/$v.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc $C2 --kernel-trace --output-format csv -d $O/$v -o b -- python3 tools/dec_time.py $L >> $O/$v.log 2>&1
  echo "== $v"; python3 tools/pmc_summary.py $O/$v/a_counter_collection.csv | grep k_win || true
  python3 tools/pmc_summary.py $O/$v/b_counter_collection.csv | grep k_win || true
done
