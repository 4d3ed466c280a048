#!/bin/bash
# Round 6: store_flush with the pending entries ordered on the host (pend_order_host) -- parity of every index test,
# then the ingest leg A/B on one box (host order vs DSY_FLUSH_ORDER=device), phases profiled once
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6i
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ingest.py tests/test_ingest_slack.py tests/test_undo.py tests/test_delete.py tests/test_sequence.py tests/test_dedup.py tests/test_claim_largest.py tests/test_claim_modulo.py > gpurun_out/r6i/tests.txt 2>&1 || { tail -40 gpurun_out/r6i/tests.txt; exit 1; }
tail -1 gpurun_out/r6i/tests.txt
for rep in 1 2; do
  for v in host device; do
    DSY_FLUSH_ORDER=$v timeout -k 10 400 python bench.py --steps 5 --warmup 1 --extra ingest --cpu-claims 0 --sim-peers 0 > gpurun_out/r6i/ingest_${v}_$rep.json 2> gpurun_out/r6i/ingest_${v}_$rep.err || { tail -20 gpurun_out/r6i/ingest_${v}_$rep.err; exit 1; }
    python -c "
import json;d=json.loads(open('gpurun_out/r6i/ingest_${v}_$rep.json').read().strip().splitlines()[-1]);w=d['ingest']['workloads']
print('$v', $rep, [(k, v['median_responder_step_after_an_append_ms'], v['responder_step_without_merge_ms'], v['median_ms_per_append']) for k,v in w.items()])"
  done
done
DSY_FLUSH_PROFILE=1 timeout -k 10 400 python bench.py --steps 5 --warmup 1 --extra ingest --cpu-claims 0 --sim-peers 0 > gpurun_out/r6i/prof.json 2> gpurun_out/r6i/prof.err || { tail -20 gpurun_out/r6i/prof.err; exit 1; }
grep flush_profile gpurun_out/r6i/prof.err | awk 'NR%5==2' | head -8
echo done
