#!/bin/bash
# Round 6: every responder parity test with DSY_FILL_SKEW set for the whole process (waves 1-3 of every
# one-workgroup fill held back): a sweep for other late-wave orderings in the window's fill
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6sw
DSY_FILL_SKEW=32 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_sync_golden.py tests/test_respond_order_gpu.py tests/test_respond_scale_gpu.py tests/test_heavy_tail_gpu.py tests/test_pipeline_gpu.py tests/test_padded_lines_gpu.py tests/test_pool_gpu.py tests/test_respond_refs_gpu.py tests/test_fullsize_gpu.py tests/test_ingest.py tests/test_undo.py tests/test_delete.py > gpurun_out/r6sw/tests.txt 2>&1 || { tail -30 gpurun_out/r6sw/tests.txt; exit 1; }
tail -2 gpurun_out/r6sw/tests.txt
