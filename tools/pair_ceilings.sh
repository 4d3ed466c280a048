#!/bin/bash
# The responder's k_pair_test ceilings on the GPU box (run through gpurun from the repo root): the headline step
# (MD5 claims) and the SHA-1 leg with the product kernel (DSY_PAIR_DIAG=0), its compute alone (1: no packet loads)
# and its gather alone (2: no compression); one bench line each into gpurun_out/pair_<diag>.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for d in ${DIAGS:-0 1 2}; do
  DSY_PAIR_DIAG=$d timeout -k 10 200 python bench.py --extra sha1 --cpu-claims 0 --steps 20 \
    > gpurun_out/pair_$d.json 2> gpurun_out/pair_$d.err || exit 1
done
echo ok
