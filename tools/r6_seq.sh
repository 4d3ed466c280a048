#!/bin/bash
# Round 6: the window sequence check (kStatusSeq) and the separate pinned area for later windows' active lists --
# responder parity tests, then ten pairs of concurrent config-5 legs (the condition of the rank-1 trip), audited.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6s
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_sync_golden.py tests/test_respond_order_gpu.py tests/test_pipeline_gpu.py tests/test_heavy_tail_gpu.py tests/test_respond_refs_gpu.py tests/test_padded_lines_gpu.py > gpurun_out/r6s/tests.txt 2>&1 || { tail -30 gpurun_out/r6s/tests.txt; exit 1; }
tail -1 gpurun_out/r6s/tests.txt
grep -h "dsybloom: window" gpurun_out/r6s/tests.txt | head -3
bash tools/r6_cfg5_audit.sh
grep -h "dsybloom: window" gpurun_out/r6ca/*.err | head -5
echo seq done
