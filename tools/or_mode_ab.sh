#!/bin/bash
# A/B of the filter-build atomics (DSY_OR_MODE, filter_set_all in dsy_message.h) on the GPU box: config 1's
# saturating 100 k-key add, a 10 M-key add (MD5 MTU filter and SHA-1 m=4096), config 4 (2^20..2^24 HBM filters)
# and config 3's claim build (k_sim_build_claims), once per mode.  Every step has its own time limit; && chains them.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/or_ab || exit 1
for mode in 0 1 2; do
  DSY_OR_MODE=$mode timeout -k 10 120 python tools/hash_sweep.py --packets 100000 --reps 50 --ops add \
      --families md5,sha1 > gpurun_out/or_ab/add100k_m$mode.json 2>&1 &&
  DSY_OR_MODE=$mode timeout -k 10 120 python tools/hash_sweep.py --packets 10000000 --reps 5 --ops add \
      --families md5,sha1 > gpurun_out/or_ab/add10m_m$mode.json 2>&1 &&
  DSY_OR_MODE=$mode timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-claims 0 --extra 1,3,4 \
      --sim-rounds 4 --sim-warmup 1 > gpurun_out/or_ab/bench_m$mode.json 2> gpurun_out/or_ab/bench_m$mode.err || exit 1
done
