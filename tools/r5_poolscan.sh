#!/bin/bash
# Round 5: the per-(claim, bin) scan placement of pooled families (k_pool_scan, DSY_POOL_SCAN=1) against the
# scatter's atomics (DSY_POOL_SCAN=0) and the unpooled order (DSY_POOL=0), on one box.  Pooled-correctness tests
# first, then interleaved bench legs (headline + SHA-1 responder; DSY_POOL=3 pools MD5 and SHA-1), then the kernel
# stats of the pooled SHA-1 leg with the scan.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_pool_gpu.py -k "scan" > gpurun_out/r5_ps_tests.txt 2>&1 || { tail -30 gpurun_out/r5_ps_tests.txt; exit 1; }
tail -1 gpurun_out/r5_ps_tests.txt
DSY_POOL=3 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_heavy_tail_gpu.py tests/test_sync_golden.py > gpurun_out/r5_ps_tests2.txt 2>&1 || { tail -30 gpurun_out/r5_ps_tests2.txt; exit 1; }
tail -1 gpurun_out/r5_ps_tests2.txt
for cfg in "0 1" "3 1" "3 0" "0 1" "3 1" "3 0"; do
  set -- $cfg
  DSY_POOL=$1 DSY_POOL_SCAN=$2 timeout -k 10 300 python bench.py --steps 40 --extra sha1 --cpu-claims 0 > gpurun_out/r5_ps_$1_$2.json 2> gpurun_out/r5_ps_$1_$2.err || { tail -20 gpurun_out/r5_ps_$1_$2.err; exit 1; }
  python tools/pool_summary.py "pool=$1 scan=$2" gpurun_out/r5_ps_$1_$2.json | tee -a gpurun_out/r5_ps_summary.txt || exit 1
done
cd /tmp && export TMPDIR=/tmp
for sc in 1 0; do
  DSY_POOL=2 DSY_POOL_SCAN=$sc timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r5_ps_prof$sc -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --extra sha1 --cpu-claims 0 > $GRAFT_REPO_ROOT/gpurun_out/r5_ps_prof$sc.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r5_ps_prof$sc.log; exit 1; }
done
