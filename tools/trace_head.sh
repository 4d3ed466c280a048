#!/bin/bash
# The headline's k_pair_test wave-tasks (DSY_PAIR_TRACE), summarised on the box: launch span, SIMD last-end spread,
# tasks per SIMD, longest tasks.
set -o pipefail
mkdir -p gpurun_out
DSY_PAIR_TRACE=/tmp/head.trace timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --extra none --cpu-claims 0 --pipeline 1 > gpurun_out/head_trace_bench.json 2> gpurun_out/head_trace_bench.err &&
timeout -k 10 200 python tools/trace_summary.py /tmp/head.trace --windows 6 > gpurun_out/head_trace_summary.txt 2>&1
