#!/bin/bash
# Round 4: head / tail hashing passes (DSY_SPLIT_TAIL) -- the responder's parity tests (the full-size one checks every
# claim of the headline's 1024), then same-box A/B of the headline and SHA-1 leg with the passes on (1) and off (0).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_sync_golden.py \
    tests/test_respond_scale_gpu.py tests/test_respond_order_gpu.py tests/test_pipeline_gpu.py \
    tests/test_heavy_tail_gpu.py tests/test_ingest.py > gpurun_out/r4_split_tests.log 2>&1 &&
for rep in 1 2; do
  for p in 1 0; do
    DSY_SPLIT_TAIL=$p timeout -k 10 300 python -u bench.py --steps 30 --extra sha1 --cpu-claims 200 > gpurun_out/r4_split_${p}_${rep}.json 2> gpurun_out/r4_split_${p}_${rep}.err || exit 1
  done
done
