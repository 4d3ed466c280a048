#!/bin/bash
# Same-box A/B: each stage's line DMA issued at the top wave priority (s_setprio 3 around the issue, the task's own
# level restored after) -- responder parity tests on the new build, then tools/ab_lib.sh (headline + SHA-1 leg, 3
# rounds).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sync_golden.py \
    tests/test_respond_scale_gpu.py tests/test_heavy_tail_gpu.py tests/test_respond_order_gpu.py \
    > gpurun_out/r4_dmaprio_tests.log 2>&1 &&
ROUNDS=3 bash tools/ab_lib.sh
