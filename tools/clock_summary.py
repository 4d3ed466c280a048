#!/usr/bin/env python3
"""Summarise tools/profile_hash.sh output: per kernel and diag build, the average dispatch time (kernel trace), the
shader clock it ran at (GRBM_GUI_ACTIVE summed over the 8 XCDs, over the dispatches' total time), the cycles per
dispatch, the VALU instructions per dispatch and the INT32 fraction against the spec peak and against the same
peak at the measured clock.

usage: clock_summary.py OUT_DIR [--match KERNEL_SUBSTRING] > profiles/<name>.json   (default k_bloom)"""
import collections
import csv
import glob
import json
import os
import sys

XCDS = 8


def main():
    root = sys.argv[1]
    match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else "k_bloom"
    out = {}
    for trace in sorted(glob.glob(os.path.join(root, "trace_*"))):
        if not os.path.isdir(trace):
            continue
        d = trace.rsplit("_", 1)[1]
        stats = glob.glob(os.path.join(trace, "**", "*kernel_stats.csv"), recursive=True)
        pmc = glob.glob(os.path.join(root, "pmc_%s" % d, "**", "*counter_collection.csv"), recursive=True)
        if not stats or not pmc:
            continue
        durs = {}
        for r in csv.DictReader(open(stats[0])):
            if match in r["Name"]:
                durs[r["Name"].split("(")[0].replace("void ", "")] = (int(r["Calls"]), float(r["AverageNs"]))
        acc = collections.defaultdict(lambda: collections.defaultdict(float))
        disp = collections.defaultdict(set)
        for r in csv.DictReader(open(pmc[0])):
            name = r.get("Kernel_Name", "").split("(")[0].replace("void ", "")
            if match not in name:
                continue
            acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[name].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
        for name, c in acc.items():
            if name not in durs:
                continue
            calls, avg_ns = durs[name]
            n = max(len(disp[name]), 1)
            clock = c["GRBM_GUI_ACTIVE"] / XCDS / (n * avg_ns * 1e-9)
            out["%s diag%s" % (name, d)] = {
                "avg_us": round(avg_ns / 1e3, 1), "dispatches": n,
                "shader_clock_ghz": round(clock / 1e9, 3),
                "cycles_per_dispatch": round(c["GRBM_GUI_ACTIVE"] / XCDS / n),
                "valu_insts_per_dispatch": round(c["SQ_INSTS_VALU"] / n),
                "salu_insts_per_dispatch": round(c["SQ_INSTS_SALU"] / n),
                "busy_cycles_per_dispatch_all_se": round(c["SQ_BUSY_CYCLES"] / n)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
