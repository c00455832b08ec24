"""Probe: the chunked schedule's slow calls at a config: every call whose insert + DivideRounds +
DecideFame + FindOrder took longer than a threshold, with each part's host time and the device
phase times. Usage: python tools/probe/chunked_outliers.py [cfg] [calls] [ms]"""
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
tot = []
for c in range(calls):
    lo = c * 1000
    if lo >= tr.E:
        break
    t0 = time.perf_counter()
    h.insert_trace(tr, lo, min(tr.E, lo + 1000))
    t1 = time.perf_counter()
    h.DivideRounds()
    t2 = time.perf_counter()
    ph = h.phase_times()
    h.DecideFame()
    t3 = time.perf_counter()
    h.FindOrder()
    t4 = time.perf_counter()
    ph2 = h.phase_times()
    dt = (t4 - t0) * 1e3
    tot.append(dt)
    if dt > lim:
        print(f"call {c}: total {dt:.2f} ms: insert {(t1 - t0) * 1e3:.2f} divide {(t2 - t1) * 1e3:.2f} "
              f"fame {(t3 - t2) * 1e3:.2f} order {(t4 - t3) * 1e3:.2f} |",
              {k: round(ph[k], 3) if isinstance(ph[k], float) else ph[k]
               for k in ("coords_ms", "rounds_ms", "la_sweeps", "rebuild", "la_wave", "la_small", "r_lo", "rounds",
                         "round_p_runs", "round_g_runs")},
              {k: round(ph2[k], 3) for k in ("fame_ms", "order_ms")}, flush=True)
tot.sort()
print(f"{len(tot)} calls: mean {sum(tot) / len(tot):.3f} ms, p50 {tot[len(tot) // 2]:.3f}, p99 {tot[int(len(tot) * .99)]:.3f}, "
      f"max {tot[-1]:.3f}")
