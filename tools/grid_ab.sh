#!/bin/bash
# k_pair_test grid cap (DSY_PAIR_GRID) on the headline and the SHA-1 responder leg, one bench run per value in $GRIDS
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/grid || exit 1
for r in 1 2; do
  for g in ${GRIDS:-512 768 1024 2048}; do
    DSY_PAIR_GRID=$g timeout -k 10 200 python bench.py --steps 30 --extra sha1 --cpu-claims 0 --sim-peers 0 > gpurun_out/grid/g$g.json 2> gpurun_out/grid/g$g.err || exit 1
    python tools/pool_summary.py "grid=$g" gpurun_out/grid/g$g.json || exit 1
  done
done
