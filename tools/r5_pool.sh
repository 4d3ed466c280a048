#!/bin/bash
# Round 5 pooled families (DSY_POOL) with the padded line copy: pooled-correctness tests first, then bench legs
# (headline, SHA-1, config 5) per pool setting on one box.
set -o pipefail
mkdir -p gpurun_out
DSY_POOL=7 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_pool_gpu.py tests/test_sync_golden.py > gpurun_out/r5_pool_tests.txt 2>&1 || { tail -30 gpurun_out/r5_pool_tests.txt; exit 1; }
tail -1 gpurun_out/r5_pool_tests.txt
for p in 0 1 2 3 0; do
  DSY_POOL=$p timeout -k 10 300 python bench.py --steps 40 --extra sha1,5 --cpu-claims 0 > gpurun_out/r5_pool_$p.json 2> gpurun_out/r5_pool_$p.err || { tail -20 gpurun_out/r5_pool_$p.err; exit 1; }
  python tools/pool_summary.py "pool=$p" gpurun_out/r5_pool_$p.json || exit 1
done
