#!/bin/bash
# Same-box A/B: hash_key_dma_lines specialised at compile time for the 1-byte prefix (no merged shifted / unshifted
# block copies) -- responder parity tests on the new build (every prefix length and the full-size claims), the
# register-only microbenchmarks, then tools/ab_lib.sh (headline + SHA-1 leg, 3 rounds) and one PMC pass of the
# headline's VALU count.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sync_golden.py \
    tests/test_respond_scale_gpu.py tests/test_heavy_tail_gpu.py tests/test_respond_order_gpu.py \
    tests/test_fullsize_gpu.py > gpurun_out/r4_r1_tests.log 2>&1 &&
timeout -k 10 120 tools/ilp_bench > gpurun_out/ilp_r4.txt 2>&1 &&
ROUNDS=3 bash tools/ab_lib.sh &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/r1_pmc -o p \
    --output-format csv -- python bench.py --steps 5 --warmup 1 --extra none --cpu-claims 0 > gpurun_out/r1_pmc.log 2>&1
