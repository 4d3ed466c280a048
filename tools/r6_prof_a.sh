#!/bin/bash
# Round-6 final tree, profiling call A (tools/profile_round.sh's headline steps): kernel trace + stats of the headline
# alone, separate FETCH_SIZE / WRITE_SIZE / SQ passes (headline + config 1 at the bench sizes), the headline clock pass
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
ARGS="--cpu-claims 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_head -o bench --output-format csv -- python bench.py --steps 20 --extra none $ARGS > gpurun_out/prof_head.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o p --output-format csv -- python bench.py --steps 5 --warmup 1 --extra none $ARGS > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o p --output-format csv -- python bench.py --steps 5 --warmup 1 --extra none $ARGS > gpurun_out/pmc_write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS -d gpurun_out/pmc_sq -o p --output-format csv -- python bench.py --steps 5 --warmup 1 --extra none $ARGS > gpurun_out/pmc_sq.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/clock_head/trace_0 -o t --output-format csv -- python bench.py --steps 20 --extra none $ARGS > gpurun_out/clock_head_trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU -d gpurun_out/clock_head/pmc_0 -o p --output-format csv -- python bench.py --steps 5 --warmup 1 --extra none $ARGS > gpurun_out/clock_head_pmc.log 2>&1 &&
tail -3 gpurun_out/prof_head.log && echo prof_a done
