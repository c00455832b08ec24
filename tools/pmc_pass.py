"""HBM bytes per consensus pass per kernel role from two rocprofv3 PMC passes over
`tools/phase_timing.py <cfg> 1` (one reset + DivideRounds + DecideFame + FindOrder):
FETCH_SIZE (KB) + WRITE_SIZE (KB). MI355X_MICROARCH.md (HBM): FETCH_SIZE reports half the
bytes of a WIDE COALESCED STREAMING read (16 B per lane), so only the streaming roles
(STREAMING below) get the x2 correction; gathers and hand-off reads are counted as read.
FETCH_SIZE comes from the L2's memory-side requests: Infinity-Cache hits are included, so
the figure is L2-miss traffic, an upper bound on HBM bytes.

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
    "layout": r"k_layout|k_ck_pack",
    "la_sweep": r"k_la_sweep|k_la_wave|k_la_small|k_la_seg",
    "fd_build": r"k_fd_build",
    "round_gather": r"k_round_gather|k_round_k_gather|k_wcoin|k_round_p_post|k_round_p_tail|k_round_p_init|k_round_pb_init|k_round_pb_silent",
    "round_search": r"k_round_k<|k_round_step|k_round_p<|k_round_pb<|k_round_g<",
    "fame": r"k_fame",
    "threshold": r"k_threshold|k_wla_transpose",
    "round_received": r"k_round_received",
    "cts_median": r"k_cts",
    "order_sort": r"k_radix|k_sort_small|k_sort_rank|k_sort_place|k_tie|k_keys|k_scan|k_minmax|k_seg_|k_finish_order",
    # ingest legs (bench.py p256_leg / ingest_leg; not in a consensus pass)
    "p256_verify": r"k_p256_verify",
    "sha256": r"k_sha256",
}


# roles whose reads are wide coalesced streams (16-byte lanes or LDS-DMA rows)
STREAMING = {"layout", "la_sweep", "fd_build", "order_sort"}


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
        # the whole-graph recurrence reads nothing but its 16-byte LDS-DMA staging
        stream = role in STREAMING or (role == "round_search" and all("k_round_g<" in k for k in fe if re.search(rx, k)))
        corr = 2.0 if stream else 1.0
        fetch = corr * 1024.0 * sum(f)
        write = 1024.0 * sum(w)
        res[role] = {"bytes_per_pass": fetch + write, "fetch_bytes": fetch, "fetch_correction": corr,
                     "write_bytes": write, "dispatches": len(f), "bytes_per_launch": (fetch + write) / len(f),
                     "note": "L2 memory-side traffic (Infinity-Cache hits included)"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
