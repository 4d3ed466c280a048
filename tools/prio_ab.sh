#!/bin/bash
# k_pair_test wave priority by wave-task length (DSY_PAIR_PRIO) x pooled SHA-1 (DSY_POOL=2), same box, twice
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/prio || exit 1
for r in 1 2; do
  for c in ${CASES:-0:0 1:0 0:2 1:2}; do
    IFS=: read pr pl <<< "$c"
    DSY_PAIR_PRIO=$pr DSY_POOL=$pl timeout -k 10 200 python bench.py --steps 30 --extra ${EXTRA:-sha1,5} --cpu-claims 0 --sim-peers 0 > gpurun_out/prio/p${pr}_$pl.json 2> gpurun_out/prio/p${pr}_$pl.err || exit 1
    python tools/pool_summary.py "prio=$pr pool=$pl" gpurun_out/prio/p${pr}_$pl.json || exit 1
  done
done
