#!/bin/bash
# Round 6: the 2-rank gloo rehearsal (tools/r6_gloo2.sh) tripped k_pair_test's task-record bounds check in config 5 on
# rank 1 (its claims: seed 5 + 1000).  Replay that rank's claims in one process; a tripped check is a clean
# DSY_EINTERNAL (exit 1), anything else ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6r1
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python tools/leg_run.py 5 --steps 12 > gpurun_out/r6r1/$name.json 2> gpurun_out/r6r1/$name.err
  local rc=$?
  echo "$name rc=$rc $(grep -o 'bounds check[^"]*' gpurun_out/r6r1/$name.err | head -1) $(cut -c1-160 gpurun_out/r6r1/$name.json)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
}
run rank1 DSY_LEG_RANK=1
run rank1_again DSY_LEG_RANK=1
run rank0 DSY_LEG_RANK=0
run rank2 DSY_LEG_RANK=2
run rank3 DSY_LEG_RANK=3
echo done
