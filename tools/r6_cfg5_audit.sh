#!/bin/bash
# Round 6: config 5 with two processes on the card (the condition under which k_pair_test's task-record check tripped),
# now with the audit that names the first bad record (k_task_audit).  A tripped check is a clean DSY_EINTERNAL (exit 1);
# any other failure ends the script.  Twelve pairs at most (both on rank 1's claims, where it tripped).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6ca
for rep in 1 2 3 4 5 6 7 8 9 10 11 12; do
  DSY_BULK_AUDIT=1 DSY_LEG_RANK=1 timeout -k 10 300 python tools/leg_run.py 5 --steps 12 > gpurun_out/r6ca/c${rep}_r0.json 2> gpurun_out/r6ca/c${rep}_r0.err &
  p0=$!
  DSY_BULK_AUDIT=1 DSY_LEG_RANK=1 timeout -k 10 300 python tools/leg_run.py 5 --steps 12 > gpurun_out/r6ca/c${rep}_r1.json 2> gpurun_out/r6ca/c${rep}_r1.err &
  p1=$!
  wait $p0; rc0=$?
  wait $p1; rc1=$?
  echo "conc $rep rc0=$rc0 rc1=$rc1"
  grep -h "bounds check\|bulk_audit" gpurun_out/r6ca/c${rep}_r*.err | cut -c1-1500 | head -6
  { [ $rc0 -le 1 ] && [ $rc1 -le 1 ]; } || exit 1
done
echo done
