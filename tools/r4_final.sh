#!/bin/bash
# Round 4 end-of-round checks as the driver runs them: the whole -m gpu suite in one process, smoke(), then the
# default bench line.  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r4_bench_final.json 2> gpurun_out/r4_bench_final.err
