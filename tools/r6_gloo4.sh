#!/bin/bash
# Round 6: bench.py's N = 4 path rehearsed on the one-GPU box -- four ranks on the same card over gloo
# (DSY_DIST_BACKEND=gloo), the legs with a multi-rank exchange: the headline and config 3's gossip simulator (4 chunks)
# (config 4 at 4 ranks on one card needs 4 x 82 GB of keys: only the driver's 8 cards hold it)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6g4
DSY_DIST_BACKEND=gloo timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 4 --steps 5 --warmup 2 --extra 3 --cpu-claims 0 > gpurun_out/r6g4/bench_g4.json 2> gpurun_out/r6g4/bench_g4.err || { grep -v "^\s*$" gpurun_out/r6g4/bench_g4.err | tail -20; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r6g4/bench_g4.json').read().strip().splitlines()[-1])
print(d['n_gpus'], d['value'], d['ms_per_step'], d.get('gossip_store_checksum'), d.get('gossip_ms_per_round'), d.get('gpu_matches_oracle'), (d.get('gossip_sim') or {}).get('chunks'))"
echo g4 done
