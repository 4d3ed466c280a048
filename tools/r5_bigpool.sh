#!/bin/bash
# Config 5 with bigger window pools (DSY_BIG_POOL pairs shared by the windows after the first): fewer windows per
# step; the leg alone, same box.
set -o pipefail
mkdir -p gpurun_out
for bp in 0 67108864 134217728 0; do
  DSY_BIG_POOL=$bp timeout -k 10 300 python tools/leg_run.py 5 --steps 8 > gpurun_out/r5_bp_$bp.json 2> gpurun_out/r5_bp_$bp.err || { tail -20 gpurun_out/r5_bp_$bp.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r5_bp_$bp.json').read().strip().splitlines()[-1]);print('big_pool $bp', d['ms_per_step'], d['serial_ms_per_step'], json.dumps(d['pair_test']), d['lane_utilization'])" || exit 1
done
