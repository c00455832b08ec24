"""Summarise tools/gpurun/r06_fame.sh: per config and tally, the k_fame_tile PMC counters of one DecideFame
and the device fame time (tools/phase_timing.py, last rep) -> one JSON.

  python tools/fame_pmc.py <dir> <out.json>
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict


def fame_counters(path):
    tot = defaultdict(float)
    disp = set()
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if "k_fame_tile" in row["Kernel_Name"]:
                tot[row["Counter_Name"]] += float(row["Counter_Value"])
                disp.add(row["Dispatch_Id"])
    return dict(sorted(tot.items())), len(disp)


def fame_ms(path):
    last = None
    with open(path) as fh:
        for line in fh:
            m = re.search(r"device: .*?\bfame_ms=([0-9.]+)", line) or re.search(r"\bfame=([0-9.]+)ms", line)
            if m:
                last = float(m.group(1))
    return last


def fame_avg_ns(path):
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if "k_fame_tile" in row["Name"]:
                return float(row["AverageNs"])
    return None


d, out = sys.argv[1], sys.argv[2]
res = {}
for cfg in ("c5", "c3"):
    for t in ("popc", "mfma"):
        p = os.path.join(d, f"{cfg}_{t}_counters.csv")
        if not os.path.exists(p):
            continue
        ctr, nd = fame_counters(p)
        r = {"counters": ctr, "dispatches": nd,
             "kernel_avg_ms_profiled": (fame_avg_ns(os.path.join(d, f"{cfg}_{t}_stats.csv")) or 0) / 1e6,
             "fame_ms_device": fame_ms(os.path.join(d, f"{cfg}_{t}_phases.log"))}
        busy = ctr.get("SQ_BUSY_CU_CYCLES", 0)
        if busy:
            r["mfma_busy_share"] = ctr.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / busy
        res[f"{cfg} k_fame_tile ({t} tally)"] = r
res["_note"] = ("rocprofv3 --kernel-trace --pmc (8 SQ counters, one pass) over one consensus pass "
                "(tools/phase_timing.py <cfg> 1, HGX_NO_WARMUP=1, HGX_FAME_TALLY=<tally>); fame_ms_device = the "
                "DecideFame phase time (HIP events) of the last of 3 unprofiled reps; tools/gpurun/r06_fame.sh")
with open(out, "w") as fh:
    json.dump(res, fh, indent=1)
print(json.dumps(res, indent=1))
