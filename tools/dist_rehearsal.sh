#!/bin/bash
# Multi-rank rehearsal on the one-GPU box: 2 ranks share the card over gloo (bench.py picks
# device LOCAL_RANK mod device count), every leg sharded and gathered as on an 8-GPU node
set -e
O=gpurun_out/${1:-dist}
mkdir -p $O
export SRSGPU_DIST_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 1 --no-cpu-baseline --legs c3,tm3,coded,c5 > $O/bench2.json 2> $O/bench2.err || { tail -20 $O/bench2.err; exit 1; }
python3 -c "import json;d=json.loads([l for l in open('$O/bench2.json') if l.startswith('{')][-1]);print(d['value'], d['n_gpus'], d.get('gather'));print({k:(d[k].get('partition'),d[k].get('gather_ms'),d[k].get('gathered_subframes'),d[k].get('subframes_per_s')) for k in ('pipeline','pipeline_tm3','pipeline_c5','pipeline_coded') if k in d})"
