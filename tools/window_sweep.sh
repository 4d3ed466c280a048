cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for w in 384 512 640 768; do
  timeout -k 10 120 python bench.py --extra none --cpu-claims 0 --window $w > gpurun_out/w_$w.json 2>&1 || exit 1
done
