#!/bin/bash
# Round 6: k_fill reads the window's start cursor once per workgroup (the late-wave race the audit found) -- responder
# parity tests, twelve concurrent pairs of config 5 on rank 1's claims (where it tripped), then the 2-rank gloo
# rehearsal of the whole bench.py on the one card.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6x
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_sync_golden.py tests/test_respond_order_gpu.py tests/test_pipeline_gpu.py tests/test_heavy_tail_gpu.py tests/test_respond_scale_gpu.py tests/test_padded_lines_gpu.py > gpurun_out/r6x/tests.txt 2>&1 || { tail -30 gpurun_out/r6x/tests.txt; exit 1; }
tail -1 gpurun_out/r6x/tests.txt
bash tools/r6_cfg5_audit.sh || exit 1
DSY_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/r6x/bench_g2.json 2> gpurun_out/r6x/bench_g2.err
rc=$?
echo "gloo2 rc=$rc $(grep -o 'bounds check[^"]*' gpurun_out/r6x/bench_g2.err | head -1 | cut -c1-600)"
cut -c1-400 gpurun_out/r6x/bench_g2.json
echo fix done
