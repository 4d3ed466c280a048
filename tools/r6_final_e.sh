#!/bin/bash
# Round-6 final tree (k_fill cursor fix + its skew regression test): every GPU test in one process, smoke(), the
# default bench.py, then the 2-rank gloo rehearsal of the whole bench on the one card
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6e
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 > gpurun_out/r6e/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r6e/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r6e/gpu_tests.log
timeout -k 10 100 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6e/smoke.log 2>&1 || { tail -20 gpurun_out/r6e/smoke.log; exit 1; }
tail -1 gpurun_out/r6e/smoke.log
timeout -k 10 500 python bench.py > gpurun_out/r6e/bench.json 2> gpurun_out/r6e/bench.err || { tail -20 gpurun_out/r6e/bench.err; exit 1; }
cut -c1-250 gpurun_out/r6e/bench.json
DSY_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29520 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/r6e/bench_g2.json 2> gpurun_out/r6e/bench_g2.err || { tail -20 gpurun_out/r6e/bench_g2.err; exit 1; }
cut -c1-250 gpurun_out/r6e/bench_g2.json
echo final_e done
