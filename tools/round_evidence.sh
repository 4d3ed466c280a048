#!/bin/bash
# Round-end evidence on the GPU box: GPU parity suite, smoke, the default bench line, then tools/profile_round.sh
# (kernel stats + PMC passes).  Every step has its own time limit; the steps are chained with &&.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
bash tools/profile_round.sh
