#!/bin/bash
# r03 profiles: decoder scaling probe, kernel-trace stats of the coded C3 leg at 16 and 30 dB and of
# the TM3 and C5 legs (separate runs, each under its own limit), C5 with either SSE decoder, and
# the 2-rank gloo rehearsal
set -e
export TMPDIR=/tmp
TAG=${1:-r03}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/dec_scale.py > $O/dec_scale.txt 2>&1 || { tail -5 $O/dec_scale.txt; exit 1; }
cat $O/dec_scale.txt
cd /tmp
for snr in 16 30; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_coded$snr -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 --no-cpu-baseline --legs coded --coded-snr $snr > $O/kt_coded$snr.log 2>&1
  echo coded $snr done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_tm3 -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 --no-cpu-baseline --legs tm3 > $O/kt_tm3.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c5 -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 --no-cpu-baseline --legs c5 > $O/kt_c5.log 2>&1
cd $GRAFT_REPO_ROOT
# C5 with the bidirectional SSE decoder (default) and the one-wave one
timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --legs c5 > $O/c5_bidir.json 2> $O/c5_bidir.err
SRSGPU_SSE_BIDIR=0 timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --legs c5 > $O/c5_seq.json 2> $O/c5_seq.err
bash tools/dist_rehearsal.sh $TAG
echo all done
