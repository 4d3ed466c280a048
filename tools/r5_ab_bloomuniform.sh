#!/bin/bash
# Same-box A/B of k_bloom with a wave-uniform wave index (readfirstlane): Bloom parity tests on the new build, then the
# config 1 and config 4 legs alternating the base build (DSY_LIB_PATH) and the new one, twice.
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_bloom_gpu.py tests/test_bitmod.py > gpurun_out/r5_ab_bloomu_tests.txt 2>&1 || { tail -30 gpurun_out/r5_ab_bloomu_tests.txt; exit 1; }
tail -1 gpurun_out/r5_ab_bloomu_tests.txt
B=$PWD/dispersy_amd/libdsybloom_base.so
for i in 1 2; do
  DSY_LIB_PATH=$B timeout -k 10 300 python bench.py --steps 5 --extra 1,4 --cpu-claims 0 > gpurun_out/ab/bb$i.json 2> gpurun_out/ab/bb$i.err || { tail -20 gpurun_out/ab/bb$i.err; exit 1; }
  timeout -k 10 300 python bench.py --steps 5 --extra 1,4 --cpu-claims 0 > gpurun_out/ab/bn$i.json 2> gpurun_out/ab/bn$i.err || { tail -20 gpurun_out/ab/bn$i.err; exit 1; }
done
