#!/bin/bash
# Config 5's responder ceilings: k_pair_test as built (diag 0), without its packet loads (1: compute ceiling) and
# without its compression (2: gather ceiling); the leg alone, same box.  Diag runs' answers are meaningless.
set -o pipefail
mkdir -p gpurun_out
for d in 0 1 2; do
  DSY_PAIR_DIAG=$d timeout -k 10 300 python tools/leg_run.py 5 --steps 8 > gpurun_out/r5_cfg5_diag$d.json 2> gpurun_out/r5_cfg5_diag$d.err || { tail -20 gpurun_out/r5_cfg5_diag$d.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r5_cfg5_diag$d.json').read().strip().splitlines()[-1]);print('diag $d', d['ms_per_step'], d['serial_ms_per_step'], json.dumps(d['pair_test']), d['lane_utilization'])" || exit 1
done
