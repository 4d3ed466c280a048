#!/bin/bash
# The single-filter kernels' ceilings on the GPU box (run through gpurun from the repo root): the product kernel
# (DSY_BLOOM_DIAG=0), its compute alone (1: no packet loads) and its gather alone (2: no compression), one JSON line
# each from tools/hash_sweep.py into gpurun_out/ceil_<diag>.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for d in ${DIAGS:-0 1 2}; do
  DSY_BLOOM_DIAG=$d timeout -k 10 120 python tools/hash_sweep.py --packets ${PACKETS:-4000000} --reps ${REPS:-5} \
    --families md5,sha1 --ops test,add > gpurun_out/ceil_$d.json 2> gpurun_out/ceil_$d.err || exit 1
done
echo ok
