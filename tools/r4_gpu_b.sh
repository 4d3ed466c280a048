#!/bin/bash
# Round 4: drop-in path (dsy_sync_respond_refs, column-wise store_messages, chunked host blob), double_signed_sync and
# the deferred index merge of appended rows -- their GPU tests, then the drop-in and ingest bench legs.  Each GPU step
# has its own limit; the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ingest_slack.py tests/test_respond_refs_gpu.py \
    tests/test_ingest.py tests/test_sequence.py tests/test_undo.py tests/test_delete.py tests/test_claim_largest.py \
    tests/test_claim_modulo.py tests/test_dedup.py tests/test_pipeline_gpu.py tests/test_sync_golden.py \
    tests/test_bitmod.py tests/test_bloom_gpu.py tests/test_respond_order_gpu.py \
    > gpurun_out/r4_dropin_tests.log 2>&1 &&
DSY_HOST_PROFILE=1 timeout -k 10 400 python -u bench.py --extra dropin,ingest --cpu-claims 0 --steps 20 > gpurun_out/r4_dropin.json 2> gpurun_out/r4_dropin.err
