"""Dev tool: the DESIGN §4 tables from the final evidence (profiles/r06_final/<cfg>_bench.json, traffic_<cfg>.json,
valu_<cfg>.json): per kernel group ms per pass, algorithmic GB, PMC GB, VALU fraction; per config the step line.

    python tools/r06_table.py [dir]
"""
import json
import os
import sys

D = sys.argv[1] if len(sys.argv) > 1 else "profiles/r06_final"


def line(cfg):
    p = os.path.join(D, f"{cfg}_bench.json")
    return json.loads([ln for ln in open(p) if ln.startswith("{")][-1])


d = line("c3")
tr = json.load(open(os.path.join(D, "traffic_c3.json")))
va = json.load(open(os.path.join(D, "valu_c3.json")))
print("c3 kernels (ms / pass, launches, algorithmic GB, PMC GB, VALU frac):")
for k, v in sorted(d["kernels_per_pass"].items(), key=lambda kv: -kv[1]["ms"]):
    ab = v.get("algorithmic_bytes")
    pmc = tr.get(k, {}).get("bytes_per_pass")
    print(f"  {k:15s} {v['ms']:7.3f} {v['launches']:2d} {'' if ab is None else round(ab / 1e9, 2):>6} "
          f"{'' if pmc is None else round(pmc / 1e9, 2):>6} {round(va.get(k, {}).get('frac_profiled', 0), 2)}")
rf = d["roofline"]
print("roofline", rf["kernel"], round(rf["ms_per_pass"], 2), "frac", round(rf["frac"], 4), "latency frac",
      round(rf.get("latency", {}).get("frac", 0), 3), "valu", round(rf.get("valu", {}).get("frac", 0), 3))
print("\nconfig | ms/step | M ev/s host RAM | HBM-resident M | CPU | rounds ms | chunked ms/call (worst)")
for c in ("c1", "c2", "c3", "c4", "c5"):
    try:
        x = line(c)
    except (OSError, IndexError):
        continue
    ph = x["config"].get("phase_ms_last_step", {})
    hb = x.get("hbm_resident", {})
    cs = x.get("chunked_sync", {})
    cb = x.get("cpu_baseline", {})
    print(f"{c} | {x['ms_per_step']:.2f} | {x['value'] / 1e6:.2f} | {hb.get('value', 0) / 1e6:.2f} | "
          f"{cb.get('value', 0):.4g} | {ph.get('rounds_ms', 0):.2f} | "
          f"{cs.get('ms_per_call', 0):.3f} ({cs.get('worst_call_ms', 0):.2f}) | phases "
          f"{ {k: round(ph[k], 2) for k in ('coords_ms', 'rounds_ms', 'fame_ms', 'order_ms') if k in ph} }")
