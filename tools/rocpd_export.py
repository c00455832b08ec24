"""Export rocprofv3's rocpd SQLite output (its default format on this image) to the CSV
summaries kept under profiles/:

  python tools/rocpd_export.py stats    <results.db> <kernel_stats.csv>
  python tools/rocpd_export.py counters <results.db> <out_counter_collection.csv>
  python tools/rocpd_export.py trace    <results.db> <kernel_trace.csv> [name regex]

stats: per kernel name Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs, StdDev
(the columns of rocprofv3 --stats). counters: one row per dispatch and counter
(Kernel_Name, Counter_Name, Counter_Value), the input of tools/pmc_traffic.py.
"""
import csv
import math
import sqlite3
import sys
from collections import defaultdict


def stats(db, out):
    con = sqlite3.connect(db)
    d = defaultdict(list)
    for name, dur in con.execute("select name, duration from kernels"):
        d[name].append(float(dur))
    tot_all = sum(sum(v) for v in d.values()) or 1.0
    rows = []
    for name, v in d.items():
        n = len(v)
        tot = sum(v)
        avg = tot / n
        sd = math.sqrt(sum((x - avg) ** 2 for x in v) / n)
        rows.append([name, n, int(tot), f"{avg:.6f}", f"{100.0 * tot / tot_all:.2f}", int(min(v)), int(max(v)), f"{sd:.6f}"])
    rows.sort(key=lambda r: -r[2])
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        w.writerows(rows)


def counters(db, out):
    con = sqlite3.connect(db)
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        for row in con.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection"):
            w.writerow(row)


def trace(db, out, pattern=""):
    """one row per dispatch in start order: name, start (ns from the first), duration (ns)"""
    import re
    con = sqlite3.connect(db)
    rows = list(con.execute("select name, start, duration from kernels order by start"))
    t0 = rows[0][1] if rows else 0
    rx = re.compile(pattern) if pattern else None
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Name", "StartNs", "DurationNs"])
        for name, start, dur in rows:
            if rx is None or rx.search(name):
                w.writerow([name, int(start - t0), int(dur)])


if __name__ == "__main__":
    {"stats": stats, "counters": counters, "trace": trace}[sys.argv[1]](*sys.argv[2:])
