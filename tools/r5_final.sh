#!/bin/bash
# Round 5 check on one box: the whole -m gpu suite, smoke(), then the default bench line (as the driver runs them).
set -o pipefail
mkdir -p gpurun_out
date -u +"tests start %T" > gpurun_out/r5_final_tests.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread >> gpurun_out/r5_final_tests.txt 2>&1 || { tail -40 gpurun_out/r5_final_tests.txt; exit 1; }
tail -1 gpurun_out/r5_final_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_final_smoke.txt 2>&1 || { tail -20 gpurun_out/r5_final_smoke.txt; exit 1; }
tail -1 gpurun_out/r5_final_smoke.txt
timeout -k 10 900 python bench.py > gpurun_out/r5_final_bench.json 2> gpurun_out/r5_final_bench.err || { tail -30 gpurun_out/r5_final_bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r5_final_bench.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline'].get('traffic'), d.get('gpu_matches_oracle'))"
