"""Dev probe: host wall time of each call of bench.py's step (clear, device insert, DivideRounds,
DecideFame, FindOrder, count) against the device phase clocks, c3 by default.

  python tools/probe/step_calls.py [cfg] [reps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from babble_amd.hashgraph import DeviceTrace, Hashgraph  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n, E, G, *_ = bench.CONFIGS[cfg]
tr, G = bench.make_trace(cfg, 0)
h = Hashgraph(n, capacity=tr.E, device=0, n_graphs=G)
dtr = DeviceTrace(tr, device=0)
for rep in range(reps):
    t = {}
    for name, fn in (("clear", h.clear), ("insert", lambda: h.insert_device(dtr)), ("divide", h.DivideRounds),
                     ("fame", h.DecideFame), ("order", h.FindOrder),
                     ("count", lambda: [int(h.L.hgx_consensus_events_count(h.ctx, g)) for g in range(G)])):
        t0 = time.perf_counter()
        fn()
        t[name] = (time.perf_counter() - t0) * 1e3
    print(f"rep {rep}: " + " ".join(f"{k}={v:.2f}ms" for k, v in t.items()) + f" | total={sum(t.values()):.1f}ms | "
          + " ".join(f"{k}={v:.2f}" for k, v in h.phase_times().items() if k.endswith("_ms")), flush=True)
