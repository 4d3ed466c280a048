#!/bin/bash
# The drop-in path's host phases: the bench's drop-in leg with DSY_HOST_PROFILE=1 (one stderr line per responder call
# from the library: claims validated + staged, windows enqueued, device wait, total, microseconds) and the store_messages
# profile (tools/profile_store_messages.py: per-call times and the cProfile split).  Summarised by the caller.
set -o pipefail
mkdir -p gpurun_out
DSY_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py --extra dropin --cpu-claims 0 --steps 10 \
    > gpurun_out/hp_dropin.json 2> gpurun_out/hp_dropin.err &&
timeout -k 10 300 python -u tools/profile_store_messages.py > gpurun_out/hp_store_messages.json 2> gpurun_out/hp_sm.err
