#!/bin/bash
# Same-box A/B: k_fill_sort reading each split-window pair's row record once (offset held in registers, 98 VGPRs)
# against re-reading it at placement (70 VGPRs): split-window parity tests, then the config-5 leg alternated twice.
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_heavy_tail_gpu.py tests/test_respond_order_gpu.py > gpurun_out/r5_ab_sortrec_tests.txt 2>&1 || { tail -30 gpurun_out/r5_ab_sortrec_tests.txt; exit 1; }
tail -1 gpurun_out/r5_ab_sortrec_tests.txt
B=$PWD/dispersy_amd/libdsybloom_base.so
for i in 1 2; do
  DSY_LIB_PATH=$B timeout -k 10 300 python tools/leg_run.py 5 --steps 8 > gpurun_out/ab/c5b$i.json 2> gpurun_out/ab/c5b$i.err || { tail -20 gpurun_out/ab/c5b$i.err; exit 1; }
  timeout -k 10 300 python tools/leg_run.py 5 --steps 8 > gpurun_out/ab/c5n$i.json 2> gpurun_out/ab/c5n$i.err || { tail -20 gpurun_out/ab/c5n$i.err; exit 1; }
done
for f in c5b1 c5n1 c5b2 c5n2; do
  python -c "import json;d=json.loads(open('gpurun_out/ab/$f.json').read().strip().splitlines()[-1]);print('$f', d['ms_per_step'], d['serial_ms_per_step'], json.dumps(d['pair_test']))" || exit 1
done
