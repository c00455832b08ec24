"""HBM bytes per consensus pass per kernel role from two rocprofv3 PMC passes over
`tools/phase_timing.py <cfg> 1` (one reset + DivideRounds + DecideFame + FindOrder):
FETCH_SIZE (KB, x2 gfx950 correction, MI355X_MICROARCH.md HBM section) + WRITE_SIZE (KB).

  python tools/pmc_pass.py <fetch_counters.csv> <write_counters.csv> <out.json>

The roles are bench.py's kernel names (hgx_kernel_stats); bench.py reads `bytes_per_pass` of
the dominant role into roofline.traffic.
"""
import csv
import json
import re
import sys
from collections import defaultdict

ROLES = {
    "layout": r"k_layout",
    "la_sweep": r"k_la_sweep|k_la_wave",
    "fd_build": r"k_fd_build",
    "round_gather": r"k_round_gather|k_round_k_gather|k_wcoin",
    "round_search": r"k_round_k<|k_round_step",
    "fame": r"k_fame",
    "threshold": r"k_threshold|k_wla_transpose",
    "round_received": r"k_round_received",
    "cts_median": r"k_cts",
    "order_sort": r"k_radix|k_sort_small|k_tie|k_keys|k_scan|k_minmax|k_finish_order",
}


def load(path, counter):
    per = defaultdict(list)
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if r["Counter_Name"] == counter:
                per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return per


def main():
    fe, wr, out = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE"), sys.argv[3]
    res = {}
    for role, rx in ROLES.items():
        f = [v for k, vs in fe.items() if re.search(rx, k) for v in vs]
        w = [v for k, vs in wr.items() if re.search(rx, k) for v in vs]
        if not f:
            continue
        fetch = 2.0 * 1024.0 * sum(f)
        write = 1024.0 * sum(w)
        res[role] = {"bytes_per_pass": fetch + write, "fetch_bytes_corrected": fetch, "write_bytes": write,
                     "dispatches": len(f), "bytes_per_launch": (fetch + write) / len(f)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
