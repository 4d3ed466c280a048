"""Device timeline of the pipelined responder from a rocprofv3 kernel trace: every dispatch between two k_fill_first
launches of the steady state, with its queue, start and duration.  Usage: python tools/pipe_timeline.py <trace dir> [from] [to]"""
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    lo = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    hi = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    ev = []
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:44],
                       r["Queue_Id"]))
    ev.sort()
    idx = [i for i, e in enumerate(ev) if "k_fill_first" in e[2]]
    a, b = idx[lo], idx[hi]
    t0 = ev[a][0]
    for e in ev[a:b]:
        print("%9.1f %8.1f  q%s %s" % ((e[0] - t0) / 1e3, (e[1] - e[0]) / 1e3, e[3], e[2]))
    print("%d fills in %.1f us: %.1f us per batch" % (hi - lo, (ev[b][0] - t0) / 1e3, (ev[b][0] - t0) / 1e3 / (hi - lo)))


if __name__ == "__main__":
    main()
