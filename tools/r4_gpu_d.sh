#!/bin/bash
# Round 4: the drop-in host path's column reads in C (dsy_host.c: store_messages, respond) and the prefetching filter
# gather of dsy_sync_respond_refs -- the GPU tests that go through SyncCommunity.respond / store_messages, then the
# drop-in bench leg alternated with the baseline library (DSY_LIB_PATH, same box), 3 rounds.  The first failure ends
# the call.
set -o pipefail
mkdir -p gpurun_out/dab
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_respond_refs_gpu.py \
    tests/test_pipeline_gpu.py tests/test_sync_golden.py tests/test_ingest.py tests/test_sequence.py \
    tests/test_claim_largest.py tests/test_claim_modulo.py > gpurun_out/r4_d_tests.log 2>&1 || exit 1
for i in 1 2 3; do
  DSY_LIB_PATH=$PWD/dispersy_amd/libdsybloom_base.so timeout -k 10 300 python -u bench.py --extra dropin --cpu-claims 0 \
      --steps 20 > gpurun_out/dab/base$i.json 2> gpurun_out/dab/base$i.err &&
  timeout -k 10 300 python -u bench.py --extra dropin --cpu-claims 0 --steps 20 > gpurun_out/dab/new$i.json \
      2> gpurun_out/dab/new$i.err || exit 1
done
