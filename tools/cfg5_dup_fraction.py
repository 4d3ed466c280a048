#!/usr/bin/env python3
"""Config 5 (heavy tail): how many of a responder step's (claim, packet) pairs hash the same message -- the same
(prefix, row) -- as another claim's pair.  The digest of prefix || packet is the same for every claim with that
1-byte prefix (community.py:773, :911 draw it per claim), so a step could hash each distinct (prefix, row) once and
probe every owning claim's filter (round-4 verdict, Next 2a).  This counts the pairs each claim walks when its
filter never spends the budget (an upper bound on the work: a claim that stops early walks fewer) and how many of
them are distinct (prefix, row) keys, over the whole step (an upper bound on what per-window sharing can save).

bench.py's config-5 store is drawn by torch's GPU generator; this draws the same distributions with numpy
(discretised Pareto(1.2) lengths are irrelevant here; Zipf(1.1) global times over 1..10^6, 10 M rows), and the
claims exactly as bench.py's heavy_tail does (PCG64(5): largest-style claims of ~capacity rows from a random row,
modulo-style claims over the whole store, a random 1-byte prefix each).  CPU only; prints one JSON line.
usage: python tools/cfg5_dup_fraction.py [--rows N] [--claims R]"""
import argparse
import json
import math

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--claims", type=int, default=1024)
    ap.add_argument("--capacity", type=int, default=1059)  # BloomFilter(10160, 0.01).get_capacity(0.01)
    args = ap.parse_args()
    N, R, G_MAX = args.rows, args.claims, 1_000_000
    rng0 = np.random.default_rng(5)
    w = np.arange(1, G_MAX + 1, dtype=np.float64) ** -1.1
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    gt = np.minimum(np.searchsorted(cdf, rng0.random(N)) + 1, G_MAX)
    gt.sort()
    starts = np.searchsorted(gt, np.arange(1, G_MAX + 2), side="left")
    rng = np.random.Generator(np.random.PCG64(5))
    modulo_m = int(math.ceil(N / float(args.capacity)))
    by_prefix = {}
    total = 0
    for i in range(R):
        if i % 2 == 0:
            a = int(rng.integers(0, N))
            lo, hi = int(gt[a]), int(gt[min(a + args.capacity - 1, N - 1)])
            iv = [(int(starts[lo - 1]), int(starts[hi]))]
        else:
            offset = int(rng.integers(0, modulo_m))
            first = (modulo_m - offset) % modulo_m or modulo_m
            iv = [(int(starts[g - 1]), int(starts[g])) for g in range(first, G_MAX + 1, modulo_m)]
        prefix = int(rng.integers(0, 256))
        n = sum(b - a for a, b in iv)
        rng.random(n)  # (bench.py draws the 1 % withheld rows here: keep the generator in step)
        total += n
        by_prefix.setdefault(prefix, []).extend(iv)
    distinct = 0
    for iv in by_prefix.values():  # the union of each prefix's row intervals
        iv.sort()
        cur_a, cur_b = iv[0]
        for a, b in iv[1:]:
            if a > cur_b:
                distinct += cur_b - cur_a
                cur_a, cur_b = a, b
            else:
                cur_b = max(cur_b, b)
        distinct += cur_b - cur_a
    print(json.dumps({"rows": N, "claims": R, "pairs_walked_upper_bound": total, "distinct_prefix_rows": distinct,
                      "duplicate_fraction": round(1 - distinct / max(total, 1), 4),
                      "note": "whole-step upper bound on what hashing each (prefix, row) once could save; the "
                              "claims' own stops and the windows' generations make the real share smaller"}))


if __name__ == "__main__":
    main()
