#!/bin/bash
# Config 5 (heavy tail) with DSY_PAIR_TRACE: per window, the launch span against its longest wave-tasks (their serial
# digests), summarised on the box (the raw trace stays there).
set -o pipefail
mkdir -p gpurun_out
DSY_PAIR_TRACE=/tmp/cfg5.trace timeout -k 10 400 python -u tools/leg_run.py 5 --steps 1 --warmup 1 > gpurun_out/cfg5_trace_leg.json 2> gpurun_out/cfg5_trace_leg.err &&
timeout -k 10 200 python tools/trace_summary.py /tmp/cfg5.trace --windows 40 > gpurun_out/cfg5_trace_summary.txt 2>&1
