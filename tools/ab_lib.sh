#!/bin/bash
# Same-box A/B of a kernel change (run through gpurun from the repo root): the headline and the SHA-1 responder leg of
# bench.py with a baseline build of the library (DSY_LIB_PATH, e.g. dispersy_amd/libdsybloom_base.so built from an
# earlier commit in a git worktree: make -C <worktree>/dispersy_amd/csrc OUT=$PWD/dispersy_amd/libdsybloom_base.so)
# and with the current build, alternated ROUNDS times so box drift hits both.  Boxes differ by 3-5 %, so kernel
# changes of that size are only judged this way.  Results: gpurun_out/ab/{base,new}<i>.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ab || exit 1
BASE=${BASE:-$PWD/dispersy_amd/libdsybloom_base.so}
ROUNDS=${ROUNDS:-2}
EXTRA=${EXTRA:-sha1}  # bench.py --extra legs beside the headline
for i in $(seq 1 "$ROUNDS"); do
  DSY_LIB_PATH=$BASE timeout -k 10 200 python bench.py --steps 30 --extra "$EXTRA" --cpu-claims 0 \
      > gpurun_out/ab/base$i.json 2> gpurun_out/ab/base$i.err &&
  timeout -k 10 200 python bench.py --steps 30 --extra "$EXTRA" --cpu-claims 0 \
      > gpurun_out/ab/new$i.json 2> gpurun_out/ab/new$i.err || exit 1
done
