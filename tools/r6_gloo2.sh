#!/bin/bash
# Round 6: bench.py's N = 2 path rehearsed on the one-GPU box -- two ranks on the same card, torch.distributed over
# gloo (DSY_DIST_BACKEND=gloo; the driver's multi-GPU runs use RCCL), every leg, the gossip simulator in 4 chunks
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6g
DSY_DIST_BACKEND=gloo timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/r6g/bench_g2.json 2> gpurun_out/r6g/bench_g2.err || { tail -30 gpurun_out/r6g/bench_g2.err; exit 1; }
cut -c1-1200 gpurun_out/r6g/bench_g2.json
