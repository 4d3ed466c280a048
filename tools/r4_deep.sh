#!/bin/bash
# Round 4: deep prefetch of heavy-tail keys in the line-staged hash (hash_key_dma_lines) -- responder parity tests,
# then same-box A/B (DSY_PAIR_DEEP=1 default / 0) of config 5 alone and the headline.  Each GPU step has its own
# limit; the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_heavy_tail_gpu.py \
    tests/test_sync_golden.py tests/test_respond_scale_gpu.py tests/test_respond_order_gpu.py tests/test_pipeline_gpu.py \
    > gpurun_out/r4_deep_tests.log 2>&1 &&
for rep in 1 2; do
  for p in 1 0; do
    DSY_PAIR_DEEP=$p timeout -k 10 300 python -u tools/leg_run.py 5 --steps 8 > gpurun_out/r4_deep_cfg5_${p}_${rep}.json 2> gpurun_out/r4_deep_cfg5_${p}_${rep}.err || exit 1
  done
done &&
for p in 1 0; do
  DSY_PAIR_DEEP=$p timeout -k 10 300 python -u bench.py --extra none --cpu-claims 0 > gpurun_out/r4_deep_head_${p}.json 2> gpurun_out/r4_deep_head_${p}.err || exit 1
done
