#!/bin/bash
# One gpurun call: k_fill phase profile (DSY_FILL_PROFILE) of the headline and SHA-1 legs, a kernel trace of the
# headline, the responder parity tests, then the 2-rank gloo rehearsal of bench.py on one GPU (the simulator leg).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
DSY_FILL_PROFILE=1 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --extra sha1 --cpu-claims 0 --sim-peers 0 --pipeline 1 > gpurun_out/fillprof.json 2> gpurun_out/fillprof.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_head -o bench --output-format csv -- python bench.py --steps 20 --extra none --cpu-claims 0 --sim-peers 0 > gpurun_out/prof_head.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_heavy_tail_gpu.py tests/test_respond_scale_gpu.py tests/test_sync_golden.py} > gpurun_out/t.log 2>&1 || { tail -20 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
if [ -n "$GLOO" ]; then
  DSY_DIST_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 2 --steps 5 --extra 3 --cpu-claims 0 > gpurun_out/gloo2.json 2> gpurun_out/gloo2.err || { tail -20 gpurun_out/gloo2.err; exit 1; }
  tail -c 300 gpurun_out/gloo2.json
fi
