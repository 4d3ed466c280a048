#!/bin/bash
# Config 5 alone under rocprofv3: kernel stats, then FETCH_SIZE and WRITE_SIZE passes (one each).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cfg5p/trace -o t --output-format csv -- python tools/leg_run.py 5 --steps 4 > gpurun_out/cfg5p_trace.txt 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/cfg5p/fetch -o p --output-format csv -- python tools/leg_run.py 5 --steps 4 > gpurun_out/cfg5p_fetch.txt 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/cfg5p/write -o p --output-format csv -- python tools/leg_run.py 5 --steps 4 > gpurun_out/cfg5p_write.txt 2>&1
