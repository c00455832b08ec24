"""One-line summary of a bench.py JSON line (tools/gpurun/r06_*.sh)."""
import json
import sys

d = json.loads([ln for ln in open(sys.argv[1]) if ln.startswith("{")][-1])
p = d["config"].get("phase_ms_last_step", {})
out = {"cfg": d["config"].get("config"), "n_gpus": d.get("n_gpus"), "ms": round(d["ms_per_step"], 3),
       "M_ev_s": round(d["value"] / 1e6, 2),
       "phases": {k: round(p[k], 2) for k in ("coords_ms", "rounds_ms", "fame_ms", "order_ms") if k in p}}
rf = d.get("roofline") or {}
if rf:
    out["dom"] = (rf.get("kernel"), round(rf.get("ms_per_pass", 0), 3), round(rf.get("frac", 0), 4))
    if rf.get("latency"):
        out["latency"] = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in rf["latency"].items() if k != "note"}
if d.get("hbm_resident"):
    out["hbm_ms"] = round(d["hbm_resident"]["ms_per_step"], 3)
if d.get("packed_columns"):
    pc = d["packed_columns"]
    out["packed"] = {k: round(pc[k], 3) for k in ("ms_per_step_incl_pack", "pack_ms", "ms_per_step_excl_pack")}
k = d.get("kernels_per_pass") or {}
out["kernels"] = {x: v["ms"] for x, v in sorted(k.items(), key=lambda kv: -kv[1]["ms"])[:8]}
for x in ("round_received", "threshold", "order_sort"):
    if x in k:
        out[x] = k[x]["ms"]
if d.get("sharded"):
    s = d["sharded"]
    out["sharded"] = s if "error" in s or "skipped" in s else {
        "shards": s["shards"], "n_gpus": s["n_gpus"], "ms": round(s["ms_per_step"], 3),
        "M_ev_s": round(s["value"] / 1e6, 2), "rounds_ms": round(s["config"]["phase_ms_last_step"]["rounds_ms"], 3),
        "fallbacks": s["config"]["phase_ms_last_step"]["round_p_fallbacks"]}
print(json.dumps(out))
