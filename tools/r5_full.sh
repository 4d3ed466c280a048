#!/bin/bash
# Round 5 full GPU check on one box: the whole -m gpu suite, smoke(), then the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5_full_tests.log 2>&1 || { tail -40 gpurun_out/r5_full_tests.log; exit 1; }
tail -2 gpurun_out/r5_full_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_smoke.log 2>&1 || { tail -20 gpurun_out/r5_smoke.log; exit 1; }
tail -2 gpurun_out/r5_smoke.log
