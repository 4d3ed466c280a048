#!/bin/bash
# Round 6: the skewed-fill regression test (tests/test_fill_skew_gpu.py) on the fixed library, then on the pre-fix
# k_fill (dispersy_amd/libdsybloom_nofix.so: the cursor read per wave, with the same skew knob), where it must fail.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6k
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_fill_skew_gpu.py > gpurun_out/r6k/fixed.txt 2>&1 || { tail -30 gpurun_out/r6k/fixed.txt; exit 1; }
tail -2 gpurun_out/r6k/fixed.txt
DSY_LIB_PATH=$PWD/dispersy_amd/libdsybloom_nofix.so timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_fill_skew_gpu.py > gpurun_out/r6k/nofix.txt 2>&1
rc=$?
echo "pre-fix rc=$rc"
grep -h "Error\|assert\|bounds" gpurun_out/r6k/nofix.txt | head -5 | cut -c1-700
[ $rc -le 1 ] || exit 1
echo skew done
