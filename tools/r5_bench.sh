#!/bin/bash
# Round 5: the default bench line (as the driver runs it) on one box.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python bench.py > gpurun_out/r5_bench.json 2> gpurun_out/r5_bench.err || { tail -30 gpurun_out/r5_bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r5_bench.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac']); print(json.dumps(d.get('heavy_tail',{}).get('ms_per_step')), d.get('gpu_matches_oracle'))"
