#!/usr/bin/env python3
"""Per-dispatch averages of a rocprofv3 --pmc CSV (p_counter_collection.csv) over the kernels whose name contains a
substring (default k_pair_test).  usage: python tools/pmc_split.py <csv> [substring]  -> one JSON line"""
import csv
import json
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "k_pair_test"
    per = defaultdict(lambda: defaultdict(float))  # dispatch -> counter -> value (summed over dimensions)
    for row in csv.DictReader(open(path)):
        if sub not in row["Kernel_Name"]:
            continue
        per[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
    names = sorted({c for d in per.values() for c in d})
    n = len(per)
    out = {"kernel_substring": sub, "dispatches": n}
    for c in names:
        out[c] = sum(d.get(c, 0.0) for d in per.values()) / max(n, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
