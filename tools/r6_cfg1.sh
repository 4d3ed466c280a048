#!/bin/bash
# Round 6: config 1's line-aligned staging (hash_key_dma_packed) -- parity tests, then a same-box A/B at one size
# (10 M keys; DSY_BLOOM_LINES=3: MD5 + SHA-1 line-staged, 0: the round-5 windows), FETCH_SIZE and SQ passes per
# variant (tools/cfg1_run.py, one size: the per-dispatch averages are not a mix).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6c1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_bloom_gpu.py > gpurun_out/r6c1/tests.txt 2>&1 || { tail -40 gpurun_out/r6c1/tests.txt; exit 1; }
tail -1 gpurun_out/r6c1/tests.txt
for fam in md5 sha1; do
  timeout -k 10 300 python tools/cfg1_run.py --family $fam --lines 3,0,3,0 > gpurun_out/r6c1/ab_$fam.json 2> gpurun_out/r6c1/ab_$fam.err || { tail -20 gpurun_out/r6c1/ab_$fam.err; exit 1; }
  cat gpurun_out/r6c1/ab_$fam.json
done
for fam in md5 sha1; do
  for v in 3 0; do
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r6c1/pmc_f_${fam}_$v -o p --output-format csv -- python tools/cfg1_run.py --family $fam --lines $v --check 0 --reps 3 > gpurun_out/r6c1/pmc_f_${fam}_$v.log 2>&1 || { tail -20 gpurun_out/r6c1/pmc_f_${fam}_$v.log; exit 1; }
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT -d gpurun_out/r6c1/pmc_sq_${fam}_$v -o p --output-format csv -- python tools/cfg1_run.py --family $fam --lines $v --check 0 --reps 3 > gpurun_out/r6c1/pmc_sq_${fam}_$v.log 2>&1 || { tail -20 gpurun_out/r6c1/pmc_sq_${fam}_$v.log; exit 1; }
    timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/r6c1/pmc_clk_${fam}_$v -o p --output-format csv -- python tools/cfg1_run.py --family $fam --lines $v --check 0 --reps 3 > gpurun_out/r6c1/pmc_clk_${fam}_$v.log 2>&1 || { tail -20 gpurun_out/r6c1/pmc_clk_${fam}_$v.log; exit 1; }
  done
done
echo done
