#!/bin/bash
# Round 6: line-staged config 1 after the slot/lag sort (A/B at 10 M keys) + FETCH pass, and the ingest leg with the
# flush phases profiled (DSY_FLUSH_PROFILE).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6c1b
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_bloom_gpu.py > gpurun_out/r6c1b/tests.txt 2>&1 || { tail -40 gpurun_out/r6c1b/tests.txt; exit 1; }
tail -1 gpurun_out/r6c1b/tests.txt
for fam in md5 sha1; do
  timeout -k 10 300 python tools/cfg1_run.py --family $fam --lines 3,0,3,0 > gpurun_out/r6c1b/ab_$fam.json 2> gpurun_out/r6c1b/ab_$fam.err || { tail -20 gpurun_out/r6c1b/ab_$fam.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/r6c1b/ab_$fam.json'))
print('$fam', [(r['lines'], r['test_us'], r['int32_frac'], r.get('gpu_vs_oracle',{}).get('membership_equal'), r['same_as_first']) for r in d['runs']])"
done
for fam in md5 sha1; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r6c1b/pmc_f_${fam}_3 -o p --output-format csv -- python tools/cfg1_run.py --family $fam --lines 3 --check 0 --reps 3 > gpurun_out/r6c1b/pmc_f_${fam}_3.log 2>&1 || { tail -20 gpurun_out/r6c1b/pmc_f_${fam}_3.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT -d gpurun_out/r6c1b/pmc_sq_${fam}_3 -o p --output-format csv -- python tools/cfg1_run.py --family $fam --lines 3 --check 0 --reps 3 > gpurun_out/r6c1b/pmc_sq_${fam}_3.log 2>&1 || { tail -20 gpurun_out/r6c1b/pmc_sq_${fam}_3.log; exit 1; }
done
DSY_FLUSH_PROFILE=1 timeout -k 10 400 python bench.py --steps 5 --warmup 1 --extra ingest --cpu-claims 0 --sim-peers 0 > gpurun_out/r6c1b/ingest.json 2> gpurun_out/r6c1b/ingest.err || { tail -20 gpurun_out/r6c1b/ingest.err; exit 1; }
grep flush_profile gpurun_out/r6c1b/ingest.err | head -40
echo done
