#!/bin/bash
# Profile the single-filter hashing kernels (tools/hash_sweep.py) on the GPU box, for the product kernel and its
# compute-only build (DSY_BLOOM_DIAG=1): kernel trace, then one PMC pass each -- GRBM_GUI_ACTIVE over the kernel's
# duration is the shader clock it ran at, SQ_ACTIVE_INST_VALU / SQ_BUSY_CYCLES the VALU issue share (the guide's
# rule: separate passes, <= 8 SQ and <= 2 GRBM counters each).  Run through gpurun from the repo root.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-hash}
mkdir -p $OUT
SW="python tools/hash_sweep.py --packets ${PACKETS:-4000000} --reps 3 --families ${FAMS:-sha1} --ops test"
for d in ${DIAGS:-0 1}; do
  DSY_BLOOM_DIAG=$d timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/trace_$d -o t --output-format csv -- $SW > $OUT/trace_$d.log 2>&1 &&
  DSY_BLOOM_DIAG=$d timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU -d $OUT/pmc_$d -o p --output-format csv -- $SW > $OUT/pmc_$d.log 2>&1 || exit 1
done
echo done
