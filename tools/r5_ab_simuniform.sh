#!/bin/bash
# Same-box A/B of the simulator kernels with a wave-uniform wave index (readfirstlane): simulator parity tests on the
# new build, then the gossip leg alternating the base build (DSY_LIB_PATH) and the new one, twice.
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_sim_gpu.py tests/test_shard_gpu.py > gpurun_out/r5_ab_simu_tests.txt 2>&1 || { tail -30 gpurun_out/r5_ab_simu_tests.txt; exit 1; }
tail -1 gpurun_out/r5_ab_simu_tests.txt
B=$PWD/dispersy_amd/libdsybloom_base.so
for i in 1 2; do
  DSY_LIB_PATH=$B timeout -k 10 300 python bench.py --steps 5 --extra 3 --cpu-claims 0 > gpurun_out/ab/sb$i.json 2> gpurun_out/ab/sb$i.err || { tail -20 gpurun_out/ab/sb$i.err; exit 1; }
  timeout -k 10 300 python bench.py --steps 5 --extra 3 --cpu-claims 0 > gpurun_out/ab/sn$i.json 2> gpurun_out/ab/sn$i.err || { tail -20 gpurun_out/ab/sn$i.err; exit 1; }
done
for f in sb1 sn1 sb2 sn2; do
  python -c "import json;d=json.loads(open('gpurun_out/ab/$f.json').read().strip().splitlines()[-1])['gossip_sim'];k=d['kernels'];print('$f', d['ms_per_round'], d['store_checksum'], {n: (v['ms_per_round'], v['lane_utilization']) for n, v in k.items()})" || exit 1
done
