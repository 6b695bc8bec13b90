#!/bin/bash
# lanes (HIP streams per rank) of the pipeline legs: 2 (the bench's), 3 and 4, default schedule
set -e
TAG=${1:-r03_s17}
O=gpurun_out/$TAG
mkdir -p $O
for L in 2 3 4; do
  timeout -k 10 400 python tools/sched_ab.py --legs c3,coded30,c5,tm3 --schedules auto --lanes $L --reps 2 > $O/lanes$L.json 2> $O/lanes$L.err || { tail -20 $O/lanes$L.err; exit 1; }
  echo "lanes $L"; grep -v amdgpu.ids $O/lanes$L.err
done
echo all done
