#!/usr/bin/env python3
"""profiles/pmc_traffic_cfg1.json from single-size PMC passes of tools/cfg1_run.py (one family per pass, 10 M keys):
per test launch of k_bloom<H, 2, TEST, line-staged>, HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes; the gfx950
half count of FETCH_SIZE, MI355X_MICROARCH.md section HBM), bound to the sha256 of the kernel's machine code in the
library the passes ran (tools/kernel_hash.py) -- bench.py's single_filter leg reports the figure only for that code.

usage: python tools/cfg1_traffic.py ROUND LIB md5:FETCH_CSV:WRITE_CSV:KEYS sha1:FETCH_CSV:WRITE_CSV:KEYS
"""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.kernel_hash import kernel_sha  # noqa: E402

SYMBOLS = {"md5": ("k_bloom<dsy::Md5, 2, 1, 2, 0, 0>", "k_bloomINS_3Md5ELi2ELi1ELi2ELi0ELi0E"),
           "sha1": ("k_bloom<dsy::Sha1, 2, 1, 2, 0, 0>", "k_bloomINS_4Sha1ELi2ELi1ELi2ELi0ELi0E")}


def per_dispatch(path, kernel, counter):
    per = defaultdict(float)
    for row in csv.DictReader(open(path)):
        if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
            per[row["Dispatch_Id"]] += float(row["Counter_Value"])
    return list(per.values())


def main():
    rnd, lib = sys.argv[1], sys.argv[2]
    out = {}
    for spec in sys.argv[3:]:
        fam, fcsv, wcsv, keys = spec.split(":")
        kernel, symbol = SYMBOLS[fam]
        f, w = per_dispatch(fcsv, kernel, "FETCH_SIZE"), per_dispatch(wcsv, kernel, "WRITE_SIZE")
        fk, wk = sum(f) / len(f), sum(w) / len(w)
        out[fam] = {"kernel": kernel, "symbol": symbol, "kernel_sha": kernel_sha(lib, symbol), "keys": int(keys),
                    "dispatches": [len(f), len(w)], "fetch_size_kib": fk, "write_size_kib": wk,
                    "hbm_bytes_per_launch": int(2 * fk * 1024 + wk * 1024),
                    "correction": "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950: FETCH_SIZE counts half of a "
                                  "16 B/lane streaming read, MI355X_MICROARCH.md section HBM)",
                    "round": rnd}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
