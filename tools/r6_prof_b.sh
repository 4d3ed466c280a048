#!/bin/bash
# Round-6 final tree, profiling call B: kernel trace + stats of the whole default bench (every leg), then config 1's
# shader clock per family (kernel trace + GRBM_GUI_ACTIVE / GRBM_COUNT with the SQ instruction counts, separate runs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_full -o bench --output-format csv -- python bench.py --steps 20 --cpu-claims 0 > gpurun_out/prof_full.log 2>&1 || { tail -20 gpurun_out/prof_full.log; exit 1; }
for fam in md5 sha1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/clock_cfg1_$fam/trace_0 -o t --output-format csv -- python tools/cfg1_run.py --family $fam --lines 3 --check 0 --reps 5 > gpurun_out/clock_cfg1_${fam}_trace.log 2>&1 || { tail -20 gpurun_out/clock_cfg1_${fam}_trace.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU -d gpurun_out/clock_cfg1_$fam/pmc_0 -o p --output-format csv -- python tools/cfg1_run.py --family $fam --lines 3 --check 0 --reps 3 > gpurun_out/clock_cfg1_${fam}_pmc.log 2>&1 || { tail -20 gpurun_out/clock_cfg1_${fam}_pmc.log; exit 1; }
done
echo prof_b done
