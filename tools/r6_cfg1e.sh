#!/bin/bash
# Round 6: same-box A/B of config 1's line staging -- v1 (192-byte rows, per-lane dword window reads, (slots, lag)
# sort; dispersy_amd/libdsybloom_v1.so built from commit 103e43e) against v4 (208-byte rows, (slots, lag, e0) sort,
# dword-aligned ds_read_b128 windows with the carry read in the same LDS round trip) and the window staging (lines 0).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6c1e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_bloom_gpu.py > gpurun_out/r6c1e/tests.txt 2>&1 || { tail -40 gpurun_out/r6c1e/tests.txt; exit 1; }
tail -1 gpurun_out/r6c1e/tests.txt
for rep in 1 2; do
  for fam in md5 sha1; do
    DSY_LIB_PATH=$PWD/dispersy_amd/libdsybloom_v1.so timeout -k 10 300 python tools/cfg1_run.py --family $fam --lines 3 --check 0 > gpurun_out/r6c1e/v1_${fam}_$rep.json 2> gpurun_out/r6c1e/v1_${fam}_$rep.err || { tail -20 gpurun_out/r6c1e/v1_${fam}_$rep.err; exit 1; }
    timeout -k 10 300 python tools/cfg1_run.py --family $fam --lines 3,0 --check 0 > gpurun_out/r6c1e/v4_${fam}_$rep.json 2> gpurun_out/r6c1e/v4_${fam}_$rep.err || { tail -20 gpurun_out/r6c1e/v4_${fam}_$rep.err; exit 1; }
    python -c "
import json
for v in ('v1', 'v4'):
    d=json.load(open('gpurun_out/r6c1e/%s_${fam}_$rep.json' % v))
    print(v, '$fam', [(r['lines'], r['test_us'], r['add_us'], r['int32_frac']) for r in d['runs']])"
  done
done
echo done
