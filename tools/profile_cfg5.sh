#!/bin/bash
# Config 5 (heavy-tailed packets) alone (tools/leg_run.py 5): kernel trace + stats, then separate PMC passes
# (FETCH_SIZE, WRITE_SIZE, SQ) as MI355X_MICROARCH.md prescribes.  Run through gpurun from the repo root.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-cfg5}
A="--steps 8"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace -o p --output-format csv -- python tools/leg_run.py 5 $A > gpurun_out/${TAG}_trace.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_fetch -o p --output-format csv -- python tools/leg_run.py 5 $A > gpurun_out/${TAG}_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_write -o p --output-format csv -- python tools/leg_run.py 5 $A > gpurun_out/${TAG}_write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS -d gpurun_out/${TAG}_sq -o p --output-format csv -- python tools/leg_run.py 5 $A > gpurun_out/${TAG}_sq.log 2>&1
