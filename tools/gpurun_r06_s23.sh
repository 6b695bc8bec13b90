set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_s23; mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python -u tools/h0_probe.py $O/base_$i.json > $O/base_$i.log 2>&1 || exit 1
  SRSGPU_LIB=$PWD/empower-srslte_amd/lib/xp/nox2/libsrsgpu_phy.so timeout -k 10 200 python -u tools/h0_probe.py $O/nox2_$i.json > $O/nox2_$i.log 2>&1 || exit 1
  SRSGPU_LIB=$PWD/empower-srslte_amd/lib/xp/l2/libsrsgpu_phy.so timeout -k 10 200 python -u tools/h0_probe.py $O/l2_$i.json > $O/l2_$i.log 2>&1 || exit 1
done
