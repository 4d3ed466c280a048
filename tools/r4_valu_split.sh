#!/bin/bash
# VALU instructions per headline k_pair_test launch: the product (DSY_PAIR_DIAG=0) against the build without the
# compression (DSY_PAIR_DIAG=2: loads, staging, probes, task setup -- the non-hash work) -- one PMC pass each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for d in 0 2; do
  DSY_PAIR_DIAG=$d timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH -d gpurun_out/valu_split/pmc_$d -o p --output-format csv -- python bench.py --steps 5 --warmup 1 --extra none --cpu-claims 0 > gpurun_out/valu_split_$d.log 2>&1 || exit 1
done
