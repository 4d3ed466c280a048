#!/bin/bash
# Round 4: store_messages with one meta object per batch (meta ids through the meta) -- its GPU tests, the
# store_messages profile and the drop-in bench leg.  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ingest.py \
    tests/test_sequence.py tests/test_dedup.py tests/test_undo.py > gpurun_out/r4_c_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/profile_store_messages.py > gpurun_out/r4_store_messages_profile.json 2> gpurun_out/r4_sm.err &&
timeout -k 10 400 python -u bench.py --extra dropin --cpu-claims 0 --steps 20 > gpurun_out/r4_dropin_c.json 2> gpurun_out/r4_dropin_c.err
