#!/bin/bash
# k_sim_respond with 8 or 4 claims per workgroup (DSY_SIM_WAVES) on the config-3 simulator, twice each
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/sim || exit 1
for r in 1 2; do
  for w in 4 8; do
    DSY_SIM_WAVES=$w timeout -k 10 300 python bench.py --steps 3 --extra 3 --cpu-claims 0 > gpurun_out/sim/w$w.json 2> gpurun_out/sim/w$w.err || exit 1
    python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['gossip_sim'];k=d['kernels']['k_sim_respond<md5>'];print('waves', sys.argv[2], d['value'], d['ms_per_round'], k['ms_per_round'], k['lane_utilization'], d['store_checksum'])" gpurun_out/sim/w$w.json $w || exit 1
  done
done
