#!/bin/bash
# Round 5: k_pair_pipe (software-pipelined responder hashing) -- responder parity tests with it, then same-box A/B
# of the headline and config 5 against k_pair_test (DSY_PAIR_PIPE=0).  Each GPU step under its own limit, && chained.
set -o pipefail
mkdir -p gpurun_out
T="${TESTS:-tests/test_sync_golden.py tests/test_respond_scale_gpu.py tests/test_heavy_tail_gpu.py tests/test_respond_order_gpu.py tests/test_respond_refs_gpu.py tests/test_pipeline_gpu.py}"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $T > gpurun_out/r5_pipe_tests.log 2>&1 || { tail -40 gpurun_out/r5_pipe_tests.log; exit 1; }
tail -2 gpurun_out/r5_pipe_tests.log
for i in 1 2; do
  for p in 1 0; do
    DSY_PAIR_PIPE=$p timeout -k 10 300 python bench.py --steps 40 --extra none --cpu-claims 0 > gpurun_out/r5_head_p${p}_$i.json 2> gpurun_out/r5_head_p${p}_$i.err || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/r5_head_p${p}_$i.json').read().strip().splitlines()[-1]);print('head pipe=$p', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])" || exit 1
  done
done
for p in 1 0; do
  DSY_PAIR_PIPE=$p timeout -k 10 400 python bench.py --steps 5 --extra 5 --cpu-claims 0 --sim-peers 0 > gpurun_out/r5_cfg5_p$p.json 2> gpurun_out/r5_cfg5_p$p.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r5_cfg5_p$p.json').read().strip().splitlines()[-1]);h=d['heavy_tail'];print('cfg5 pipe=$p', h['ms_per_step'], h['pair_test'], h['lane_utilization'])" || exit 1
done
