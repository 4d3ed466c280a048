#!/bin/bash
# Round-6 final tree, call C: the two regrouped oracle test modules (worlds shared across modes / windows), then the
# default bench.py again (config 1's traffic now read from profiles/pmc_traffic_cfg1.json)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6f
timeout -k 10 600 python -u -m pytest tests/test_pool_gpu.py tests/test_respond_scale_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread --durations=20 > gpurun_out/r6f/regroup_tests.log 2>&1 || { tail -40 gpurun_out/r6f/regroup_tests.log; exit 1; }
tail -25 gpurun_out/r6f/regroup_tests.log
timeout -k 10 600 python bench.py > gpurun_out/r6f/bench2.json 2> gpurun_out/r6f/bench2.err || { tail -20 gpurun_out/r6f/bench2.err; exit 1; }
cut -c1-400 gpurun_out/r6f/bench2.json
