#!/bin/bash
# Round 6: the simulator's HIP engine against the oracle engine at the bench's gossip shape, 20 000 peers
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6sc
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_sim_gpu.py --durations=5 > gpurun_out/r6sc/tests.txt 2>&1 || { tail -30 gpurun_out/r6sc/tests.txt; exit 1; }
tail -8 gpurun_out/r6sc/tests.txt
