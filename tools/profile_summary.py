#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output of bench.py into profiles/ (tracked).

usage: profile_summary.py ROUND TRACE_DIR [PMC_DIR ...]
  TRACE_DIR: rocprofv3 --kernel-trace --stats output (…_kernel_stats.csv)
  PMC_DIR:   rocprofv3 --pmc output (…_counter_collection.csv), one directory per pass

Writes profiles/<ROUND>_kernel_stats.csv (copy), profiles/<ROUND>_pmc.json (per-kernel counter averages per
dispatch) and profiles/pmc_traffic_<hash>.json with the HBM bytes per k_pair_test launch, corrected as
MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE (KiB) reads exactly half the bytes of a wide (16 B/lane)
streaming read on gfx950, so bytes_read = 2 * FETCH_SIZE * 1024; WRITE_SIZE * 1024 is exact for 16-B stores
and is reported as measured.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    return name.split("(")[0].replace("void ", "")[:80]


def main():
    rnd, trace = sys.argv[1], sys.argv[2]
    pmc_dirs = [d for d in sys.argv[3:] if not d.startswith("--full=")]
    full = [d[len("--full="):] for d in sys.argv[3:] if d.startswith("--full=")]
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    stats = glob.glob(os.path.join(trace, "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(out, "%s_kernel_stats.csv" % rnd))
        print(open(stats[0]).read()[:3000])
    for d in full:
        fs = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
        if fs:
            shutil.copy(fs[0], os.path.join(out, "%s_full_kernel_stats.csv" % rnd))
    per = defaultdict(lambda: defaultdict(list))
    for d in pmc_dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                per[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    summary = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}
    with open(os.path.join(out, "%s_pmc.json" % rnd), "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    for k, cs in summary.items():
        if "k_pair_test" in k and "FETCH_SIZE" in cs:
            kind = "md5" if "Md5" in k else "sha1" if "Sha1" in k else "sha256" if "Sha256" in k else "sha512"
            sys.path.insert(0, ROOT)
            from tools.kernel_hash import HEADLINE, kernel_sha
            lib = os.environ.get("DSY_LIB_PATH") or os.path.join(ROOT, "dispersy_amd", "libdsybloom.so")
            rec = {"kernel": k, "fetch_size_kib": cs["FETCH_SIZE"], "write_size_kib": cs.get("WRITE_SIZE"),
                   "kernel_sha": kernel_sha(lib, HEADLINE) if kind == "md5" else None,
                   "hbm_bytes_per_launch": 2 * cs["FETCH_SIZE"] * 1024 + (cs.get("WRITE_SIZE") or 0) * 1024,
                   "correction": "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950: FETCH_SIZE counts half of a "
                                 "16 B/lane streaming read, MI355X_MICROARCH.md §HBM)",
                   "round": rnd}
            with open(os.path.join(out, "pmc_traffic_%s.json" % kind), "w") as f:
                json.dump(rec, f, indent=1)
            print(json.dumps(rec))
    print(json.dumps(summary, indent=1)[:4000])


if __name__ == "__main__":
    main()
