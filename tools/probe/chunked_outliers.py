"""Probe: the chunked schedule's slow DivideRounds calls at a config (phase times of each call
slower than a threshold). Usage: python tools/probe/chunked_outliers.py [cfg] [calls] [ms]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from babble_amd.hashgraph import Hashgraph  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
lim = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
n, E, G, *_ = bench.CONFIGS[cfg]
tr, G = bench.make_trace(cfg, 0)
h = Hashgraph(n, capacity=tr.E, device=0, n_graphs=G)
for c in range(calls):
    lo = c * 1000
    h.insert_trace(tr, lo, min(tr.E, lo + 1000))
    t0 = time.perf_counter()
    h.DivideRounds()
    dt = (time.perf_counter() - t0) * 1e3
    ph = h.phase_times()
    if dt > lim:
        print(f"call {c}: divide {dt:.2f} ms", {k: ph[k] for k in ("coords_ms", "rounds_ms", "la_sweeps", "rebuild",
                                                              "la_wave", "la_wave_fallbacks", "r_lo", "rounds")}, flush=True)
    h.DecideFame()
    h.FindOrder()
