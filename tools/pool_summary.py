"""One line per bench.py result: the headline's and the SHA-1 responder's step, k_pair_test launch and lane use."""
import json
import sys

label, path = sys.argv[1], sys.argv[2]
d = json.loads(open(path).read().strip().splitlines()[-1])
r = d["roofline"]
out = ["%s: headline %.3f ms/step %.1f us/launch frac %.3f util %.3f" % (
    label, d["ms_per_step"], r["avg_launch_us"], r["frac"], r.get("lane_utilization", 0))]
s = d.get("sha1_respond")
if s:
    sr = s["roofline"]
    out.append("sha1 %.3f ms/step %.1f us/launch valu %.3f util %.3f" % (
        s["ms_per_step"], sr["avg_launch_us"], sr["frac"], sr["lane_utilization"]))
h = d.get("heavy_tail")
if h:
    out.append("cfg5 %.2f ms/step pair_test %.0f us x %.1f util %.3f" % (
        h["ms_per_step"], h["pair_test"]["avg_launch_us"], h["pair_test"]["launches_per_step"], h["lane_utilization"]))
print(" | ".join(out))
