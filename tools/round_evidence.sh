#!/bin/bash
# Round-end evidence on the GPU box: the default bench line, then tools/profile_round.sh (kernel stats + PMC passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out || exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
bash tools/profile_round.sh
