#!/bin/bash
# DSY_PACK_STREAM A/B on one build: the responder tests (in flight and synchronous) with the pack on its own stream,
# then bench.py's headline + SHA-1 + config 5 alternating 0 / 1, twice.
set -o pipefail
mkdir -p gpurun_out/ab
DSY_PACK_STREAM=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_sync_golden.py tests/test_pipeline_gpu.py tests/test_respond_order_gpu.py tests/test_respond_refs_gpu.py tests/test_padded_lines_gpu.py tests/test_heavy_tail_gpu.py > gpurun_out/r5_ps_tests.txt 2>&1 || { tail -30 gpurun_out/r5_ps_tests.txt; exit 1; }
tail -1 gpurun_out/r5_ps_tests.txt
for i in 1 2; do
  for ps in 0 1; do
    DSY_PACK_STREAM=$ps timeout -k 10 300 python bench.py --steps 30 --extra sha1,5,dropin --cpu-claims 0 > gpurun_out/ab/ps${ps}_$i.json 2> gpurun_out/ab/ps${ps}_$i.err || { tail -20 gpurun_out/ab/ps${ps}_$i.err; exit 1; }
    python -c "
import json;d=json.loads(open('gpurun_out/ab/ps${ps}_$i.json').read().strip().splitlines()[-1])
s=d.get('sha1_respond',{}); h=d.get('heavy_tail',{}); dr=d.get('dropin',{}).get('respond',{})
print('ps=$ps', d['value'], d['ms_per_step'], d['serial_ms_per_step'], d['roofline']['avg_launch_us'], 'sha1', s.get('ms_per_step'), 'cfg5', h.get('ms_per_step'), 'dropin', dr.get('median_ms_per_batch'))" || exit 1
  done
done
