#!/bin/bash
# Instruction mix per k_pair_test launch, product (DSY_PAIR_DIAG=0) against the build without the compression (2):
# the headline (bench.py --extra none) and config 5 (tools/leg_run.py 5), one PMC pass each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU"
for d in 0 2; do
  DSY_PAIR_DIAG=$d timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmc_split/head_$d -o p --output-format csv -- python bench.py --steps 5 --warmup 1 --extra none --cpu-claims 0 > gpurun_out/pmc_split_head_$d.txt 2>&1 || exit 1
  python tools/pmc_split.py gpurun_out/pmc_split/head_$d/p_counter_collection.csv | tee gpurun_out/pmc_split_head_$d.json || exit 1
  DSY_PAIR_DIAG=$d timeout -s KILL 240 rocprofv3 --pmc $C -d gpurun_out/pmc_split/cfg5_$d -o p --output-format csv -- python tools/leg_run.py 5 --steps 4 > gpurun_out/pmc_split_cfg5_$d.txt 2>&1 || exit 1
  python tools/pmc_split.py gpurun_out/pmc_split/cfg5_$d/p_counter_collection.csv | tee gpurun_out/pmc_split_cfg5_$d.json || exit 1
done
