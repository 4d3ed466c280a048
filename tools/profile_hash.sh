#!/bin/bash
# Profile the single-filter hashing kernels (tools/hash_sweep.py) on the GPU box: kernel trace + one PMC pass per
# counter group (the guide's rule: separate passes, <= 8 SQ counters each).  Run through gpurun from the repo root.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-hash}
mkdir -p $OUT
SW="python tools/hash_sweep.py --packets ${PACKETS:-4000000} --reps 3 --families ${FAMS:-md5,sha1} --ops test"
timeout -k 10 120 python tools/hash_sweep.py --packets ${PACKETS:-4000000} --reps 5 --families ${FAMS:-md5,sha1} --ops test > $OUT/sweep.json 2> $OUT/sweep.err &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/trace -o t --output-format csv -- $SW > $OUT/trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $OUT/pmc_a -o p --output-format csv -- $SW > $OUT/pmc_a.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA -d $OUT/pmc_b -o p --output-format csv -- $SW > $OUT/pmc_b.log 2>&1
echo done rc=$?
