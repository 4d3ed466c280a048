#!/bin/bash
# Same-box A/B of k_pair_test with a wave-uniform task index (readfirstlane: the task decode and the claim's state
# loads become scalar): responder parity tests on the new build, then the headline + SHA-1 legs and the config-5 leg
# alternating the base build (DSY_LIB_PATH) and the new one, twice.
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_respond_scale_gpu.py tests/test_heavy_tail_gpu.py tests/test_sync_golden.py tests/test_padded_lines_gpu.py tests/test_pool_gpu.py -k "not deal or 16384" > gpurun_out/r5_ab_uniform_tests.txt 2>&1 || { tail -30 gpurun_out/r5_ab_uniform_tests.txt; exit 1; }
tail -1 gpurun_out/r5_ab_uniform_tests.txt
B=$PWD/dispersy_amd/libdsybloom_base.so
for i in 1 2; do
  DSY_LIB_PATH=$B timeout -k 10 300 python bench.py --steps 30 --extra sha1 --cpu-claims 0 > gpurun_out/ab/hb$i.json 2> gpurun_out/ab/hb$i.err || { tail -20 gpurun_out/ab/hb$i.err; exit 1; }
  timeout -k 10 300 python bench.py --steps 30 --extra sha1 --cpu-claims 0 > gpurun_out/ab/hn$i.json 2> gpurun_out/ab/hn$i.err || { tail -20 gpurun_out/ab/hn$i.err; exit 1; }
  DSY_LIB_PATH=$B timeout -k 10 300 python tools/leg_run.py 5 --steps 8 > gpurun_out/ab/c5b$i.json 2> gpurun_out/ab/c5b$i.err || { tail -20 gpurun_out/ab/c5b$i.err; exit 1; }
  timeout -k 10 300 python tools/leg_run.py 5 --steps 8 > gpurun_out/ab/c5n$i.json 2> gpurun_out/ab/c5n$i.err || { tail -20 gpurun_out/ab/c5n$i.err; exit 1; }
done
for f in hb1 hn1 hb2 hn2; do python tools/pool_summary.py $f gpurun_out/ab/$f.json || exit 1; done
for f in c5b1 c5n1 c5b2 c5n2; do
  python -c "import json;d=json.loads(open('gpurun_out/ab/$f.json').read().strip().splitlines()[-1]);print('$f', d['ms_per_step'], d['serial_ms_per_step'], json.dumps(d['pair_test']))" || exit 1
done
