#!/bin/bash
# RCCL on the one-GPU box: one rank (calls and dtypes), then two ranks sharing cuda:0 (accepted or refused by this
# RCCL build).  Each step under its own limit; the 2-rank step may fail without ending the call's first result.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29531 tools/rccl_probe.py > gpurun_out/rccl_probe_1.log 2>&1 || exit 1
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29532 tools/rccl_probe.py > gpurun_out/rccl_probe_2.log 2>&1
echo "two-rank rc=$?" >> gpurun_out/rccl_probe_2.log
