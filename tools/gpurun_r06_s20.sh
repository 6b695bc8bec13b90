set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_s20; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --legs none --steps 30 --warmup 5 --no-cpu-baseline --detail $O/base_$i.json > $O/base_$i.log 2> $O/base_$i.err || exit 1
  SRSGPU_LIB=$PWD/empower-srslte_amd/lib/xp/h0w2/libsrsgpu_phy.so timeout -k 10 200 python -u bench.py --legs none --steps 30 --warmup 5 --no-cpu-baseline --detail $O/h0w2_$i.json > $O/h0w2_$i.log 2> $O/h0w2_$i.err || exit 1
done
