#!/bin/bash
# Round 4: the drop-in host path's column reads in C (dsy_host.c: store_messages, respond) -- the GPU tests that go
# through SyncCommunity.respond / store_messages, then the drop-in bench leg.  The first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_respond_refs_gpu.py \
    tests/test_pipeline_gpu.py tests/test_sync_golden.py tests/test_ingest.py tests/test_sequence.py \
    tests/test_claim_largest.py tests/test_claim_modulo.py > gpurun_out/r4_d_tests.log 2>&1 &&
timeout -k 10 400 python -u bench.py --extra dropin --cpu-claims 0 --steps 20 > gpurun_out/r4_dropin_d.json 2> gpurun_out/r4_dropin_d.err
