#!/bin/bash
# Round 6: line-staged config 1 with uniform windows (208-byte rows, (slots, lag, e0) sort) -- parity tests, A/B at
# 10 M keys, FETCH + SQ passes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6c1c
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_bloom_gpu.py tests/test_claim_largest.py tests/test_claim_modulo.py > gpurun_out/r6c1c/tests.txt 2>&1 || { tail -40 gpurun_out/r6c1c/tests.txt; exit 1; }
tail -1 gpurun_out/r6c1c/tests.txt
for fam in md5 sha1; do
  timeout -k 10 300 python tools/cfg1_run.py --family $fam --lines 3,0,3,0 > gpurun_out/r6c1c/ab_$fam.json 2> gpurun_out/r6c1c/ab_$fam.err || { tail -20 gpurun_out/r6c1c/ab_$fam.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/r6c1c/ab_$fam.json'))
print('$fam', [(r['lines'], r['test_us'], r['add_us'], r['int32_frac'], r.get('gpu_vs_oracle',{}).get('membership_equal'), r['same_as_first']) for r in d['runs']])"
done
for fam in md5 sha1; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r6c1c/pmc_f_${fam}_3 -o p --output-format csv -- python tools/cfg1_run.py --family $fam --lines 3 --check 0 --reps 3 > gpurun_out/r6c1c/pmc_f_${fam}_3.log 2>&1 || { tail -20 gpurun_out/r6c1c/pmc_f_${fam}_3.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r6c1c/pmc_w_${fam}_3 -o p --output-format csv -- python tools/cfg1_run.py --family $fam --lines 3 --check 0 --reps 3 > gpurun_out/r6c1c/pmc_w_${fam}_3.log 2>&1 || { tail -20 gpurun_out/r6c1c/pmc_w_${fam}_3.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT -d gpurun_out/r6c1c/pmc_sq_${fam}_3 -o p --output-format csv -- python tools/cfg1_run.py --family $fam --lines 3 --check 0 --reps 3 > gpurun_out/r6c1c/pmc_sq_${fam}_3.log 2>&1 || { tail -20 gpurun_out/r6c1c/pmc_sq_${fam}_3.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/r6c1c/pmc_clk_${fam}_3 -o p --output-format csv -- python tools/cfg1_run.py --family $fam --lines 3 --check 0 --reps 3 > gpurun_out/r6c1c/pmc_clk_${fam}_3.log 2>&1 || { tail -20 gpurun_out/r6c1c/pmc_clk_${fam}_3.log; exit 1; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r6c1c/trace -o t --output-format csv -- python tools/cfg1_run.py --family md5 --lines 3 --check 0 --reps 5 > gpurun_out/r6c1c/trace.log 2>&1 || { tail -20 gpurun_out/r6c1c/trace.log; exit 1; }
echo done
