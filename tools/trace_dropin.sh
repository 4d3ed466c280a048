#!/bin/bash
# Kernel and memory-copy trace of bench.py's drop-in leg (SyncCommunity.respond through dsy_sync_respond_refs):
# where the host-buffer call's time goes beside the device step.  CSVs under gpurun_out/dropin_trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/dropin_trace \
    -o dropin -- python3 bench.py --extra dropin --cpu-claims 0 --steps 5 > gpurun_out/dropin_trace.log 2>&1
