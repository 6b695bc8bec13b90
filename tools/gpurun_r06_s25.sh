set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_s25; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --legs none --steps 30 --warmup 5 --no-cpu-baseline --detail $O/base_$i.json > $O/base_$i.log 2> $O/base_$i.err || exit 1
  SRSGPU_LIB=$PWD/empower-srslte_amd/lib/xp/ntl/libsrsgpu_phy.so timeout -k 10 200 python -u bench.py --legs none --steps 30 --warmup 5 --no-cpu-baseline --detail $O/ntl_$i.json > $O/ntl_$i.log 2> $O/ntl_$i.err || exit 1
done
timeout -k 10 200 python -u tools/h0_probe.py $O/probe_base.json > $O/probe_base.log 2>&1 &&
SRSGPU_LIB=$PWD/empower-srslte_amd/lib/xp/ntl/libsrsgpu_phy.so timeout -k 10 200 python -u tools/h0_probe.py $O/probe_ntl.json > $O/probe_ntl.log 2>&1
