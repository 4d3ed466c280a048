#!/bin/bash
# Headline (config 2, no CPU legs) at each pipeline depth in $DEPTHS, then a kernel trace at the last one for
# tools/pipe_timeline.py; TESTS: GPU tests to run first
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
  tail -2 gpurun_out/tests.log
fi
for d in ${DEPTHS:-3}; do
  timeout -k 10 300 python bench.py --steps 40 --extra ${EXTRA:-none} --cpu-claims 0 --pipeline $d ${BENCH_ARGS:-} > gpurun_out/head_p$d.json 2> gpurun_out/head_p$d.err || exit 1
  python -c "import json,sys;d=json.loads(open('gpurun_out/head_p$d.json').read().strip().splitlines()[-1]);print('depth $d', d['value'], d['ms_per_step'], d['serial_ms_per_step'], d['roofline']['avg_launch_us'])" || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pipe -o bench --output-format csv -- python bench.py --steps 20 --extra none --cpu-claims 0 --pipeline $d ${BENCH_ARGS:-} > gpurun_out/prof_pipe.log 2>&1
