"""lastAncestors build time on a C3-shaped trace by dataflow time segments (hgx_set_la_kernel
modes: 1 = sweeps, m >= 2 = m segments, 0 = auto)."""
import sys
import time
sys.path.insert(0, ".")
from babble_amd import trace as gtrace
from babble_amd.hashgraph import Hashgraph

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
E = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
modes = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0, 1, 4, 8, 16, 32, 64]
t = gtrace.gossip(n, E, 1)
for m in modes:
    h = Hashgraph(n, capacity=E)
    h.set_la_kernel(m)
    h.set_incremental(False)
    h.insert_trace(t)
    best = None
    for rep in range(3):
        h.DivideRounds()
        pt = h.phase_times()
        best = pt if best is None or pt["coords_ms"] < best["coords_ms"] else best
    print(f"mode {m}: coords {best['coords_ms']:.2f} ms  segs {best['la_wave_segs']} sweeps {best['la_sweeps']} "
          f"rows {best['la_rows']} fallbacks {best['la_wave_fallbacks']}", flush=True)
    del h
