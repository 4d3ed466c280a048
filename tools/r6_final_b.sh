#!/bin/bash
# Round-6 final tree, call B: the default bench.py, then config 1's FETCH / WRITE passes (one family each, 10 M keys,
# default staging) for profiles/pmc_traffic_cfg1.json
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6f
timeout -k 10 600 python bench.py > gpurun_out/r6f/bench.json 2> gpurun_out/r6f/bench.err || { tail -20 gpurun_out/r6f/bench.err; exit 1; }
cat gpurun_out/r6f/bench.json | cut -c1-600
for fam in md5 sha1; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r6f/pmc_f_$fam -o p --output-format csv -- python tools/cfg1_run.py --family $fam --lines 3 --check 0 --reps 3 > gpurun_out/r6f/pmc_f_$fam.log 2>&1 || { tail -20 gpurun_out/r6f/pmc_f_$fam.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r6f/pmc_w_$fam -o p --output-format csv -- python tools/cfg1_run.py --family $fam --lines 3 --check 0 --reps 3 > gpurun_out/r6f/pmc_w_$fam.log 2>&1 || { tail -20 gpurun_out/r6f/pmc_w_$fam.log; exit 1; }
done
python tools/cfg1_traffic.py r6 dispersy_amd/libdsybloom.so \
  md5:$(find gpurun_out/r6f/pmc_f_md5 -name '*counter_collection.csv' -print -quit):$(find gpurun_out/r6f/pmc_w_md5 -name '*counter_collection.csv' -print -quit):10000000 \
  sha1:$(find gpurun_out/r6f/pmc_f_sha1 -name '*counter_collection.csv' -print -quit):$(find gpurun_out/r6f/pmc_w_sha1 -name '*counter_collection.csv' -print -quit):10000000 \
  > gpurun_out/r6f/pmc_traffic_cfg1.json && cat gpurun_out/r6f/pmc_traffic_cfg1.json
