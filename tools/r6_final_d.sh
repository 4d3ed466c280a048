#!/bin/bash
# Round-6 final tree (after the k_fill cursor fix): every GPU test in one process (durations), smoke(), the default
# bench.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6z
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=25 > gpurun_out/r6z/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r6z/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r6z/gpu_tests.log
timeout -k 10 100 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6z/smoke.log 2>&1 || { tail -20 gpurun_out/r6z/smoke.log; exit 1; }
tail -1 gpurun_out/r6z/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r6z/bench.json 2> gpurun_out/r6z/bench.err || { tail -20 gpurun_out/r6z/bench.err; exit 1; }
cut -c1-300 gpurun_out/r6z/bench.json
