"""Per-kernel mean of every PMC counter in a rocprofv3 rocpd database (one JSON line per
kernel whose name matches the regex), for quick instruction-mix / cache summaries.

  python tools/pmc_summary.py <results.db> [kernel_regex]
"""
import json
import re
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
rx = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
con = sqlite3.connect(db)
acc = defaultdict(lambda: defaultdict(list))
for name, ctr, val in con.execute("select kernel_name, counter_name, value from counters_collection"):
    if rx.search(name):
        acc[name][ctr].append(float(val))
for name, d in acc.items():
    print(json.dumps({"kernel": name[:80], "dispatches": max(len(v) for v in d.values()),
                      **{k: sum(v) / len(v) for k, v in sorted(d.items())}}))
