#!/bin/bash
# Round 5 baseline on a fresh box: the headline (config 2) alone, three runs, then the config-5 leg once.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 40 --extra none --cpu-claims 0 > gpurun_out/r5_base_head$i.json 2> gpurun_out/r5_base_head$i.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r5_base_head$i.json').read().strip().splitlines()[-1]);print('head', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])" || exit 1
done
timeout -k 10 400 python bench.py --steps 5 --extra 5 --cpu-claims 0 --sim-peers 0 > gpurun_out/r5_base_cfg5.json 2> gpurun_out/r5_base_cfg5.err || exit 1
python -c "import json;d=json.loads(open('gpurun_out/r5_base_cfg5.json').read().strip().splitlines()[-1]);print(json.dumps(d.get('heavy_tail',{}))[:1500])"
