#!/bin/bash
# The N > 1 path on one GPU: bench.py with two ranks over gloo (claims sharded, the simulator's all-to-all(v), the
# sharded large-filter build); the simulator's store checksum must equal the one-rank run's.
set -o pipefail
mkdir -p gpurun_out
DSY_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 5 --extra 3,4 --cpu-claims 0 > gpurun_out/r5_gloo2.json 2> gpurun_out/r5_gloo2.err || { tail -20 gpurun_out/r5_gloo2.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r5_gloo2.json').read().strip().splitlines()[-1]);print(d['n_gpus'], d['value'], d.get('gossip_n_gpus'), d.get('gossip_store_checksum'), d.get('gossip_rounds_per_s'))"
