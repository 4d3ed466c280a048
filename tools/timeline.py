"""Print the device timeline of a few steady-state responder steps from a rocprofv3 kernel/memory-copy trace
(tools/profile_round.sh layout): each dispatch or copy with its start relative to the step's first kernel, its
duration and the idle gap before it.  Usage: python tools/timeline.py <trace dir> [first step] [steps]"""
import csv
import glob
import sys


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                out.append(r)
    return out


def main():
    d = sys.argv[1]
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    ev = []
    for r in rows(d + "/**/*kernel_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:48]))
    for r in rows(d + "/**/*memory_copy_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "?")))
    ev.sort()
    starts = [i for i, e in enumerate(ev) if e[2].startswith("dsy::k_setup") or e[2].startswith("dsy::k_fill_first")]
    if len(starts) < first + nsteps + 1:
        first = max(0, len(starts) - nsteps - 1)
    for s in range(first, first + nsteps):
        a, b = starts[s], starts[s + 1]
        t0 = ev[a][0]
        print("step %d: %.1f us to the next step" % (s, (ev[b][0] - t0) / 1e3))
        prev_end = ev[a - 1][1] if a else t0
        for e in ev[a - 1:b]:
            print("  %+9.1f us  %8.1f us  gap %7.1f  %s" % ((e[0] - t0) / 1e3, (e[1] - e[0]) / 1e3,
                                                          (e[0] - prev_end) / 1e3, e[2]))
            prev_end = max(prev_end, e[1])


if __name__ == "__main__":
    main()
