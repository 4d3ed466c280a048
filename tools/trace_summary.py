"""Summarise a DSY_PAIR_TRACE file (k_pair_test wave-task records, dsy_capi.hip job_window): per window, the launch
span, how the wave-tasks' start times spread, how busy every SIMD was, and the time per block of the tasks.

usage: python tools/trace_summary.py TRACE [--windows N]"""
import sys

import numpy as np

REC = np.dtype([("hw", "<u4"), ("xcc", "<u4"), ("t0", "<u8"), ("t1", "<u8"), ("blocks", "<u4"), ("task", "<u4")])


def windows(path):
    raw = open(path, "rb").read()
    at = 0
    while at + 16 <= len(raw):
        n, w = np.frombuffer(raw, "<u8", 2, at)
        at += 16
        yield int(w), np.frombuffer(raw, REC, int(n), at)
        at += int(n) * REC.itemsize


def simd_key(r):
    hw = r["hw"].astype(np.int64)
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    return ((r["xcc"].astype(np.int64) * 8 + se) * 2 + sh) * 16 * 4 + cu * 4 + simd


def summary(w, r):
    t0, t1 = r["t0"].astype(np.int64), r["t1"].astype(np.int64)
    s0, s1 = t0.min(), t1.max()
    span = (s1 - s0) * 10e-3  # us (100 MHz)
    key = simd_key(r)
    simds, inv = np.unique(key, return_inverse=True)
    last = np.zeros(len(simds), np.int64)
    np.maximum.at(last, inv, t1 - s0)
    work = np.zeros(len(simds), np.int64)
    np.add.at(work, inv, r["blocks"].astype(np.int64))
    start_us = np.percentile((t0 - s0) * 10e-3, [50, 90, 99, 100])
    end_us = np.percentile(last * 10e-3, [0, 10, 50, 90, 100])
    dur = (t1 - t0) * 10e-3
    per_blk = dur / np.maximum(r["blocks"], 1)
    print("window W=%d: %d wave-tasks on %d SIMDs, span %.1f us" % (w, len(r), len(simds), span))
    print("  task start after launch start (p50/p90/p99/max us): %s" % " ".join("%.1f" % x for x in start_us))
    print("  SIMD last end (min/p10/p50/p90/max us): %s" % " ".join("%.1f" % x for x in end_us))
    print("  SIMD blocks (min/p10/p50/p90/max): %s  mean %.1f" % (
        " ".join("%d" % x for x in np.percentile(work, [0, 10, 50, 90, 100])), work.mean()))
    print("  tasks per SIMD (min/mean/max): %d %.2f %d" % (
        np.bincount(inv).min(), np.bincount(inv).mean(), np.bincount(inv).max()))
    print("  task us per block (p10/p50/p90): %s; task blocks (p10/p50/p90): %s" % (
        " ".join("%.2f" % x for x in np.percentile(per_blk, [10, 50, 90])),
        " ".join("%d" % x for x in np.percentile(r["blocks"], [10, 50, 90]))))
    # busy fraction: SIMD-time covered by at least one running task of that SIMD, over span x SIMDs
    busy = 0
    for k in range(len(simds)):
        m = inv == k
        iv = sorted(zip(t0[m], t1[m]))
        cur_a, cur_b = iv[0]
        for a, b in iv[1:]:
            if a > cur_b:
                busy += cur_b - cur_a
                cur_a, cur_b = a, b
            else:
                cur_b = max(cur_b, b)
        busy += cur_b - cur_a
    print("  SIMD occupied fraction of the span: %.3f" % (busy / float(len(simds) * (s1 - s0))))
    # the critical path: the longest wave-tasks (their serial digests) against the span
    top = np.argsort(dur)[::-1][:5]
    print("  longest tasks (us / blocks / start us): %s" % "; ".join(
        "%.1f / %d / %.1f" % (dur[i], r["blocks"][i], (t0[i] - s0) * 10e-3) for i in top))


def main():
    path = sys.argv[1]
    limit = int(sys.argv[sys.argv.index("--windows") + 1]) if "--windows" in sys.argv else 3
    for i, (w, r) in enumerate(windows(path)):
        if i >= limit:
            break
        if len(r):
            summary(w, r)


if __name__ == "__main__":
    main()
