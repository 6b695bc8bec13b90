#!/bin/bash
# decoder experiments: time each library variant under empower-srslte_amd/lib/xp/ (timing only)
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-xp}
mkdir -p $O
for v in $(ls empower-srslte_amd/lib/xp); do
  timeout -k 10 120 python3 tools/dec_time.py empower-srslte_amd/lib/xp/$v/libsrsgpu_phy.so 2>&1 | tee -a $O/times.txt
done
timeout -k 10 120 python3 tools/dec_time.py empower-srslte_amd/lib/libsrsgpu_phy.so 2>&1 | tee -a $O/times.txt
