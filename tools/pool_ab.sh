#!/bin/bash
# Pooled responder families (DSY_POOL = bitmask of hash kinds, DSY_POOL_QUEUE) on one box: optionally the GPU tests in
# $TESTS with $TEST_POOL (default 7: every poolable family pooled), then bench.py's headline and SHA-1 responder legs
# under each setting in $CASES ("pool:queue:deal" triples), summarised by tools/pool_summary.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -n "${TESTS+x}" ]; then
  DSY_POOL=${TEST_POOL:-7} timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests} > gpurun_out/pool_tests.log 2>&1 || { tail -30 gpurun_out/pool_tests.log; exit 1; }
  tail -2 gpurun_out/pool_tests.log
fi
for c in ${CASES:-0:0:0 2:0:0 2:0:1}; do
  IFS=: read p q dl <<< "$c"
  DSY_POOL=$p DSY_POOL_QUEUE=$q DSY_POOL_DEAL=$dl timeout -k 10 300 python bench.py --steps 40 --extra ${EXTRA:-sha1} --cpu-claims 0 --sim-peers 0 > gpurun_out/pool_${p}_${q}_${dl}.json 2> gpurun_out/pool_${p}_${q}_${dl}.err || { tail -20 gpurun_out/pool_${p}_${q}_${dl}.err; exit 1; }
  python tools/pool_summary.py "pool=$p queue=$q deal=$dl" gpurun_out/pool_${p}_${q}_${dl}.json || exit 1
done
