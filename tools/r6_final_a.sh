#!/bin/bash
# Round-6 final tree, call A: every GPU test in one process (durations listed), then smoke()
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6f
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=40 > gpurun_out/r6f/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r6f/gpu_tests.log; exit 1; }
tail -50 gpurun_out/r6f/gpu_tests.log
timeout -k 10 100 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6f/smoke.log 2>&1 || { tail -20 gpurun_out/r6f/smoke.log; exit 1; }
cat gpurun_out/r6f/smoke.log
