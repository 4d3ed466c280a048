#!/bin/bash
# Round 4: the gather drop-in's tests, the pipelined tests and the call-order test in ONE process (the order that
# faulted in round 3), then the default bench.  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_respond_gather_gpu.py \
    tests/test_pipeline_gpu.py tests/test_respond_order_gpu.py > gpurun_out/r4_order_tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r4_bench_a.json 2> gpurun_out/r4_bench_a.err
