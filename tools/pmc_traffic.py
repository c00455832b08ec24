"""Summarise rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE, KB per dispatch) into HBM
bytes per launch per kernel, with the gfx950 correction of MI355X_MICROARCH.md (HBM
section): FETCH_SIZE reports half of the bytes of wide coalesced reads -> x2.

  python tools/pmc_traffic.py <fetch_dir> <write_dir> <out.json> [kernel=regex ...]
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def load(d, counter):
    rows = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") != counter:
                    continue
                rows[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return rows


def main():
    fetch_dir, write_dir, out = sys.argv[1:4]
    kmap = dict(a.split("=", 1) for a in sys.argv[4:])
    fe, wr = load(fetch_dir, "FETCH_SIZE"), load(write_dir, "WRITE_SIZE")
    res = {}
    for key, rx in kmap.items():
        f = [v for k, vs in fe.items() if re.search(rx, k) for v in vs]
        w = [v for k, vs in wr.items() if re.search(rx, k) for v in vs]
        if not f or not w:
            continue
        fetch = 2.0 * 1024.0 * sum(f) / len(f)   # KB -> B, x2 gfx950 correction
        write = 1024.0 * sum(w) / len(w)
        res[key] = {"bytes_per_launch": fetch + write, "fetch_bytes_corrected": fetch, "write_bytes": write,
                    "dispatches": len(f)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
