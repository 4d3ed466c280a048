#!/bin/bash
# Profile bench.py on the GPU box (run through gpurun from the repo root; every step has its own time limit and the
# steps are chained with &&):
#   1. kernel trace + stats of the headline (config 2) alone -> the k_pair_test average to compare with bench.py's
#   2. kernel trace + stats of the full bench (every config)
#   3. separate PMC passes over the headline and config 1 (FETCH_SIZE, WRITE_SIZE, SQ), as the guide prescribes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
ARGS="--cpu-claims 0 ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_head -o bench --output-format csv -- python bench.py --steps 20 --extra none $ARGS > gpurun_out/prof_head.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_full -o bench --output-format csv -- python bench.py --steps 20 $ARGS > gpurun_out/prof_full.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o p --output-format csv -- python bench.py --steps 5 --warmup 1 --extra 1 $ARGS > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o p --output-format csv -- python bench.py --steps 5 --warmup 1 --extra 1 $ARGS > gpurun_out/pmc_write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS -d gpurun_out/pmc_sq -o p --output-format csv -- python bench.py --steps 5 --warmup 1 --extra 1 $ARGS > gpurun_out/pmc_sq.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/clock_head/trace_0 -o t --output-format csv -- python bench.py --steps 20 --extra none $ARGS > gpurun_out/clock_head_trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU -d gpurun_out/clock_head/pmc_0 -o p --output-format csv -- python bench.py --steps 5 --warmup 1 --extra none $ARGS > gpurun_out/clock_head_pmc.log 2>&1
