#!/bin/bash
# Round 6: (1) the unaligned ds_read_b128 probe; (2) parity: single filter + ingest/index tests; (3) config-1 A/B
# (line staging: 208-byte rows, (slots, lag, e0) sort, dword-aligned b128 window reads) + FETCH/SQ passes; (4) the
# ingest leg with the fused small-batch flush, phases profiled.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6c1d
timeout -k 5 60 ./tools/lds_unaligned_probe > gpurun_out/r6c1d/probe.txt 2>&1 || { cat gpurun_out/r6c1d/probe.txt; exit 1; }
cat gpurun_out/r6c1d/probe.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_bloom_gpu.py tests/test_claim_largest.py tests/test_claim_modulo.py tests/test_ingest.py tests/test_ingest_slack.py tests/test_undo.py tests/test_delete.py tests/test_sequence.py > gpurun_out/r6c1d/tests.txt 2>&1 || { tail -40 gpurun_out/r6c1d/tests.txt; exit 1; }
tail -1 gpurun_out/r6c1d/tests.txt
for fam in md5 sha1; do
  timeout -k 10 300 python tools/cfg1_run.py --family $fam --lines 3,0,3,0 > gpurun_out/r6c1d/ab_$fam.json 2> gpurun_out/r6c1d/ab_$fam.err || { tail -20 gpurun_out/r6c1d/ab_$fam.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/r6c1d/ab_$fam.json'))
print('$fam', [(r['lines'], r['test_us'], r['add_us'], r['int32_frac'], r.get('gpu_vs_oracle',{}).get('membership_equal'), r['same_as_first']) for r in d['runs']])"
done
for fam in md5 sha1; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r6c1d/pmc_f_${fam}_3 -o p --output-format csv -- python tools/cfg1_run.py --family $fam --lines 3 --check 0 --reps 3 > gpurun_out/r6c1d/pmc_f_${fam}_3.log 2>&1 || { tail -20 gpurun_out/r6c1d/pmc_f_${fam}_3.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT -d gpurun_out/r6c1d/pmc_sq_${fam}_3 -o p --output-format csv -- python tools/cfg1_run.py --family $fam --lines 3 --check 0 --reps 3 > gpurun_out/r6c1d/pmc_sq_${fam}_3.log 2>&1 || { tail -20 gpurun_out/r6c1d/pmc_sq_${fam}_3.log; exit 1; }
done
DSY_FLUSH_PROFILE=1 timeout -k 10 400 python bench.py --steps 5 --warmup 1 --extra ingest --cpu-claims 0 --sim-peers 0 > gpurun_out/r6c1d/ingest.json 2> gpurun_out/r6c1d/ingest.err || { tail -20 gpurun_out/r6c1d/ingest.err; exit 1; }
grep flush_profile gpurun_out/r6c1d/ingest.err | awk 'NR%4==1' | head -12
python -c "
import json;d=json.loads(open('gpurun_out/r6c1d/ingest.json').read().strip().splitlines()[-1]);w=d['ingest']['workloads']
[print(k, v['median_responder_step_after_an_append_ms'], v['responder_step_without_merge_ms'], v['index_bytes_per_append_over_batch_index_bytes'], v['median_ms_per_append']) for k,v in w.items()]"
echo done
