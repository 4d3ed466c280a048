#!/bin/bash
# Round 5 kernel step: the whole -m gpu suite on the new build, then a same-box A/B against the previous build
# (dispersy_amd/libdsybloom_base.so): headline + SHA-1 leg + config 5, two alternations.
set -o pipefail
mkdir -p gpurun_out
date -u +"tests start %T" > gpurun_out/r5_ab_tests.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread >> gpurun_out/r5_ab_tests.txt 2>&1 || { tail -40 gpurun_out/r5_ab_tests.txt; exit 1; }
date -u +"tests end %T" >> gpurun_out/r5_ab_tests.txt
tail -2 gpurun_out/r5_ab_tests.txt
ROUNDS=2 EXTRA=sha1,5 bash tools/ab_lib.sh || exit 1
date -u +"ab end %T"
for f in gpurun_out/ab/base1 gpurun_out/ab/new1 gpurun_out/ab/base2 gpurun_out/ab/new2; do
  python -c "
import json,sys;d=json.loads(open('$f.json').read().strip().splitlines()[-1])
s=d.get('sha1_respond',{}); h=d.get('heavy_tail',{})
print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], 'sha1', s.get('ms_per_step'), (s.get('roofline') or {}).get('avg_launch_us'), 'cfg5', h.get('ms_per_step'), (h.get('pair_test') or {}).get('avg_launch_us'))" || exit 1
done
