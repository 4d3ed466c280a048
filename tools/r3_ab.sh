#!/bin/bash
# Responder / store parity tests, then a same-box A/B (tools/ab_lib.sh) of the current library against
# dispersy_amd/libdsybloom_base.so with the SHA-1 and drop-in legs, summarised one line per run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out || exit 1
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_sync_golden.py tests/test_respond_scale_gpu.py tests/test_heavy_tail_gpu.py tests/test_ingest.py tests/test_undo.py tests/test_sequence.py tests/test_delete.py} > gpurun_out/t2.log 2>&1 || { tail -30 gpurun_out/t2.log; exit 1; }
tail -2 gpurun_out/t2.log
ROUNDS=${ROUNDS:-3} EXTRA=${EXTRA:-sha1,dropin} bash tools/ab_lib.sh || exit 1
for f in gpurun_out/ab/*.json; do
  python tools/pool_summary.py "$f" "$f" || exit 1
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);x=d.get('dropin');print('dropin', x and (x['store_messages']['median_ms_per_batch'], x['respond']['median_ms_per_batch']))" "$f" || exit 1
done
