"""Probe: the SyncLimit-chunked schedule (Core.Sync + RunConsensus per 1 000 events) at a config's
shape: host wall time per API call (insert, DivideRounds, DecideFame, FindOrder) and the device
phase times, averaged over calls after a warm-up; optional kernel timing per call.
Usage: python tools/probe/chunked_profile.py [cfg] [calls] [sync_limit] [warm-up calls]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import bench  # noqa: E402
from babble_amd.hashgraph import Hashgraph  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
sl = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
warm = int(sys.argv[4]) if len(sys.argv) > 4 else calls // 10
n, E, G, *_ = bench.CONFIGS[cfg]
tr, G = bench.make_trace(cfg, 0)
h = Hashgraph(n, capacity=tr.E, device=0, n_graphs=G)
acc = {k: [] for k in ("insert", "divide", "fame", "order", "total")}
ph_acc = {}
for c in range(calls):
    lo = c * sl
    if lo >= tr.E:
        break
    t0 = time.perf_counter(); h.insert_trace(tr, lo, min(tr.E, lo + sl)); t1 = time.perf_counter()
    h.DivideRounds(); t2 = time.perf_counter()
    ph = h.phase_times()
    h.DecideFame(); t3 = time.perf_counter()
    h.FindOrder(); t4 = time.perf_counter()
    if c >= warm:
        for k, v in (("insert", t1 - t0), ("divide", t2 - t1), ("fame", t3 - t2), ("order", t4 - t3), ("total", t4 - t0)):
            acc[k].append(v * 1e3)
        for k in ("coords_ms", "rounds_ms"):
            ph_acc.setdefault(k, []).append(ph[k])
        ph2 = h.phase_times()
        for k in ("fame_ms", "order_ms"):
            ph_acc.setdefault(k, []).append(ph2[k])
print(f"{cfg}: {len(acc['total'])} calls of {sl} events (after {warm} warm-up calls)")
for k, v in acc.items():
    q = len(v) // 4
    print(f"  host {k:7s} mean {np.mean(v):.3f} ms  p50 {np.median(v):.3f}  max {np.max(v):.3f}"
          f"  first-quarter {np.mean(v[:q]):.3f}  last-quarter {np.mean(v[-q:]):.3f}")
for k, v in ph_acc.items():
    print(f"  device {k:10s} mean {np.mean(v):.3f} ms")
tot = np.asarray(acc["total"])
for w in np.argsort(-tot)[:5]:
    print(f"  worst call {w + warm}: " + " ".join(f"{k} {acc[k][w]:.3f}" for k in acc))
