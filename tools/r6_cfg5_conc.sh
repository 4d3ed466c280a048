#!/bin/bash
# Round 6: does config 5's task-record bounds trip (2-rank gloo rehearsal, rank 1) need two processes on the card?
# (a) two concurrent single-process legs (ranks 0 and 1's claims), twice; (b) the 2-rank gloo bench with config 5 only.
# A tripped check is a clean DSY_EINTERNAL (exit 1); any other failure ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6cc
for rep in 1 2; do
  DSY_LEG_RANK=0 timeout -k 10 300 python tools/leg_run.py 5 --steps 12 > gpurun_out/r6cc/c${rep}_r0.json 2> gpurun_out/r6cc/c${rep}_r0.err &
  p0=$!
  DSY_LEG_RANK=1 timeout -k 10 300 python tools/leg_run.py 5 --steps 12 > gpurun_out/r6cc/c${rep}_r1.json 2> gpurun_out/r6cc/c${rep}_r1.err &
  p1=$!
  wait $p0; rc0=$?
  wait $p1; rc1=$?
  echo "conc $rep rc0=$rc0 rc1=$rc1 $(grep -ho 'bounds check[^"]*' gpurun_out/r6cc/c${rep}_r*.err | head -2)"
  { [ $rc0 -le 1 ] && [ $rc1 -le 1 ]; } || exit 1
done
DSY_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 5 --warmup 2 --extra 5 --cpu-claims 0 > gpurun_out/r6cc/g2_cfg5.json 2> gpurun_out/r6cc/g2_cfg5.err
rc=$?
echo "gloo2 extra5 rc=$rc $(grep -o 'bounds check[^"]*' gpurun_out/r6cc/g2_cfg5.err | head -2)"
cut -c1-300 gpurun_out/r6cc/g2_cfg5.json
echo done
