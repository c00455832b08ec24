"""Dev tool: host wall time of each drop-in call vs the device phase times, one config.

  python tools/phase_timing.py [c3|c2|c4|c5] [reps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from babble_amd.hashgraph import Hashgraph  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n, E, G, *_ = bench.CONFIGS[cfg]
tr, G = bench.make_trace(cfg, 0)
h = Hashgraph(n, capacity=tr.E, device=0, n_graphs=G)
if os.environ.get("HGX_FAME_TALLY"):   # (A/B of DecideFame's tally: popc, vote, mfma)
    h.set_fame_tally(os.environ["HGX_FAME_TALLY"])
h.insert_trace(tr)
for rep in range(reps):
    t = {}
    t0 = time.perf_counter(); h.reset_consensus(); t["reset"] = time.perf_counter() - t0
    t0 = time.perf_counter(); h.DivideRounds(); t["divide"] = time.perf_counter() - t0
    t0 = time.perf_counter(); h.DecideFame(); t["fame"] = time.perf_counter() - t0
    t0 = time.perf_counter(); h.FindOrder(); t["order"] = time.perf_counter() - t0
    ph = h.phase_times()
    print(f"rep {rep}: " + " ".join(f"{k}={v*1e3:.2f}ms" for k, v in t.items()) +
          f" | total={sum(t.values())*1e3:.1f}ms | device: " +
          " ".join(f"{k}={v:.2f}" for k, v in ph.items()), flush=True)
