"""Probe: the chunked schedule's first calls on fresh contexts (per-process one-time costs vs per-context
ones): two contexts in turn, each created, then three 1 000-event calls (insert / DivideRounds /
DecideFame / FindOrder host times). Usage: python tools/probe/first_call.py [cfg]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from babble_amd.hashgraph import Hashgraph  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
warm = len(sys.argv) > 2 and sys.argv[2] == "warm"
n, E, G, *_ = bench.CONFIGS[cfg]
tr, G = bench.make_trace(cfg, 0)
if warm:   # a tiny context of another size first: is the first call's cost per process or per size?
    t1 = bench.make_trace("c1", 0)[0]
    t0 = time.perf_counter()
    hw = Hashgraph(4, capacity=t1.E, device=0)
    hw.insert_trace(t1)
    hw.RunConsensus()
    del hw
    print(f"warm-up context (n = 4, {t1.E} events): {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
for ctx in range(2):
    t0 = time.perf_counter()
    h = Hashgraph(n, capacity=tr.E, device=0, n_graphs=G)
    print(f"context {ctx}: create {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
    for c in range(3):
        lo = c * 1000
        t0 = time.perf_counter()
        h.insert_trace(tr, lo, lo + 1000)
        t1 = time.perf_counter()
        h.DivideRounds()
        t2 = time.perf_counter()
        ph = h.phase_times()
        h.DecideFame()
        t3 = time.perf_counter()
        h.FindOrder()
        t4 = time.perf_counter()
        print(f"  call {c}: total {(t4 - t0) * 1e3:.2f} ms: insert {(t1 - t0) * 1e3:.2f} divide {(t2 - t1) * 1e3:.2f} "
              f"fame {(t3 - t2) * 1e3:.2f} order {(t4 - t3) * 1e3:.2f} | coords {ph['coords_ms']:.2f} "
              f"rounds {ph['rounds_ms']:.2f} rebuild {ph['rebuild']} round_p_runs {ph['round_p_runs']}", flush=True)
    del h
