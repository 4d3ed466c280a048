#!/bin/bash
# Round 4: dsy_sync_respond_refs' filter gather on two host threads -- the GPU tests that go through
# SyncCommunity.respond, then the drop-in bench leg with DSY_GATHER_THREADS=1 / 2 alternated (same library, same
# box), 3 rounds.  The first failure ends the call.
set -o pipefail
mkdir -p gpurun_out/gab
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_respond_refs_gpu.py \
    tests/test_pipeline_gpu.py tests/test_respond_order_gpu.py tests/test_sync_golden.py \
    > gpurun_out/r4_gather_tests.log 2>&1 || exit 1
for i in 1 2 3; do
  DSY_GATHER_THREADS=1 timeout -k 10 300 python -u bench.py --extra dropin --cpu-claims 0 --steps 20 \
      > gpurun_out/gab/one$i.json 2> gpurun_out/gab/one$i.err &&
  DSY_GATHER_THREADS=2 timeout -k 10 300 python -u bench.py --extra dropin --cpu-claims 0 --steps 20 \
      > gpurun_out/gab/two$i.json 2> gpurun_out/gab/two$i.err || exit 1
done
