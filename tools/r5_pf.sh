#!/bin/bash
# DSY_LINE_PF (each stage also loads one dword of every key's next line) A/B on one build: responder tests with it
# on, then bench.py's headline + SHA-1 + config 5 alternating off / on, twice.
set -o pipefail
mkdir -p gpurun_out/ab
DSY_LINE_PF=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_sync_golden.py tests/test_padded_lines_gpu.py tests/test_respond_scale_gpu.py tests/test_heavy_tail_gpu.py > gpurun_out/r5_pf_tests.txt 2>&1 || { tail -30 gpurun_out/r5_pf_tests.txt; exit 1; }
tail -1 gpurun_out/r5_pf_tests.txt
for i in 1 2; do
  for pf in 0 1; do
    DSY_LINE_PF=$pf timeout -k 10 300 python bench.py --steps 30 --extra sha1,5 --cpu-claims 0 > gpurun_out/ab/pf${pf}_$i.json 2> gpurun_out/ab/pf${pf}_$i.err || { tail -20 gpurun_out/ab/pf${pf}_$i.err; exit 1; }
    python -c "
import json;d=json.loads(open('gpurun_out/ab/pf${pf}_$i.json').read().strip().splitlines()[-1])
s=d.get('sha1_respond',{}); h=d.get('heavy_tail',{})
print('pf=$pf', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], 'sha1', s.get('ms_per_step'), (s.get('roofline') or {}).get('avg_launch_us'), 'cfg5', h.get('ms_per_step'), (h.get('pair_test') or {}).get('avg_launch_us'))" || exit 1
  done
done
