"""Per-kernel average duration (us) and calls from a rocprofv3 run_results.db (its top_kernels view).
usage: python tools/db_top.py DB [substring ...]"""
import sqlite3
import sys

db, keys = sys.argv[1], sys.argv[2:]
c = sqlite3.connect(db)
for name, calls, total, avg, pct in c.execute("select * from top_kernels"):
    if not keys or any(k in name for k in keys):
        print("%-90s calls %6d avg %10.3f us total %12.1f us" % (name[:90], calls, avg, total))
