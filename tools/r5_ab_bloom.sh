#!/bin/bash
# Same-box A/B of the single-filter (config 1) and simulator (config 3) kernels: the MD5 tests run first on the
# new build, then bench.py --extra 1,3 alternating base (DSY_LIB_PATH) and new, twice.
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_bloom_gpu.py tests/test_sim_gpu.py tests/test_sync_golden.py > gpurun_out/r5_ab_bloom_tests.txt 2>&1 || { tail -30 gpurun_out/r5_ab_bloom_tests.txt; exit 1; }
tail -1 gpurun_out/r5_ab_bloom_tests.txt
for i in 1 2; do
  DSY_LIB_PATH=$PWD/dispersy_amd/libdsybloom_base.so timeout -k 10 300 python bench.py --steps 10 --extra 1,3 --cpu-claims 0 > gpurun_out/ab/bb$i.json 2> gpurun_out/ab/bb$i.err || { tail -20 gpurun_out/ab/bb$i.err; exit 1; }
  timeout -k 10 300 python bench.py --steps 10 --extra 1,3 --cpu-claims 0 > gpurun_out/ab/bn$i.json 2> gpurun_out/ab/bn$i.err || { tail -20 gpurun_out/ab/bn$i.err; exit 1; }
done
for f in bb1 bn1 bb2 bn2; do
  python -c "
import json;d=json.loads(open('gpurun_out/ab/$f.json').read().strip().splitlines()[-1])
sf=d.get('single_filter',{}); g=d.get('gossip_sim',{})
print('$f', 'md5 test', sf.get('md5',{}).get('test_keys_per_s'), 'sha1 test', sf.get('sha1',{}).get('test_keys_per_s'), 'md5 add', sf.get('md5',{}).get('add_keys_per_s'), 'gossip', g.get('value'), g.get('ms_per_round'))" || exit 1
done
