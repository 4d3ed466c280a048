#!/bin/bash
# headline (config 2) with the responder's window capped (bench.py --window, dsy_ctx_set_window) at each value in
# $WINDOWS (0: the default growing window), pipelined and one batch at a time
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/win || exit 1
for r in 1 2; do
  for w in ${WINDOWS:-0 640 704 768 896}; do
    timeout -k 10 200 python bench.py --steps 40 --extra none --cpu-claims 0 --sim-peers 0 --window $w > gpurun_out/win/w$w.json 2> gpurun_out/win/w$w.err || exit 1
    python - "$w" <<'PY' || exit 1
import json, sys
w = sys.argv[1]
d = json.loads(open("gpurun_out/win/w%s.json" % w).read().strip().splitlines()[-1])
r = d["roofline"]
print("window %s: %.3f G useful/s, %.3f ms/step (serial %.3f), hashed/step %.0f, pair_test %.1f us x %d launches / %d steps" % (
    w, d["value"] / 1e9, d["ms_per_step"], d["serial_ms_per_step"], d["pairs_hashed_per_s"] * d["ms_per_step"] / 1e3,
    r["avg_launch_us"], r["launches"], d["steps"]))
PY
  done
done
