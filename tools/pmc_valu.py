"""VALU instruction issue per consensus pass per kernel role, from one rocprofv3 PMC pass
(SQ_INSTS_VALU, wave instructions) with the kernel trace of the same run (durations):

  python tools/pmc_valu.py <counters.csv> <kernel_stats.csv> <out.json>

valu_insts_per_pass x 64 lanes / duration = the achieved lane-op rate; its fraction of the
MI355X VALU peak (32 lanes/clk x 4 SIMD x 256 CU x 2.4 GHz = 78.6 T lane-op/s) is the VALU
roofline beside the HBM one (bench.py reads `valu_insts_per_pass` of the dominant role).
The profiled duration includes the counter collection's overhead: frac_profiled is a
lower bound, bench.py recomputes the fraction over its own timed ms_per_pass.
"""
import csv
import json
import re
import sys
from collections import defaultdict

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
from pmc_pass import ROLES  # noqa: E402

PEAK = 32 * 4 * 256 * 2.4e9


def main():
    cnt, stats, out = sys.argv[1], sys.argv[2], sys.argv[3]
    per = defaultdict(list)
    with open(cnt) as fh:
        for r in csv.DictReader(fh):
            if r["Counter_Name"] == "SQ_INSTS_VALU":
                per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    dur = defaultdict(float)
    with open(stats) as fh:
        for r in csv.DictReader(fh):
            dur[r["Name"]] += float(r["TotalDurationNs"])
    res = {}
    for role, rx in ROLES.items():
        v = [x for k, xs in per.items() if re.search(rx, k) for x in xs]
        if not v:
            continue
        d = sum(x for k, x in dur.items() if re.search(rx, k))
        insts = sum(v)
        res[role] = {"valu_insts_per_pass": insts, "dispatches": len(v), "profiled_ns": d,
                     "frac_profiled": (64.0 * insts / (d * 1e-9) / PEAK) if d > 0 else None}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
