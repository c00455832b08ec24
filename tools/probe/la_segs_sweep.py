"""Probe: coordinates phase time of a full DivideRounds against the lastAncestors time-segment
count (hgx_set_la_kernel mode >= 2). Usage: python tools/probe/la_segs_sweep.py [cfg] [segs...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from babble_amd.hashgraph import Hashgraph  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
segs = [int(x) for x in sys.argv[2:]] or [0, 8, 16, 24, 32, 48]
n, E, G, *_ = bench.CONFIGS[cfg]
tr, G = bench.make_trace(cfg, 0)
h = Hashgraph(n, capacity=tr.E, device=0, n_graphs=G)
h.insert_trace(tr)
for s in segs:
    best = 1e9
    for rep in range(3):
        h.L.hgx_set_la_kernel(h.ctx, s)
        h.reset_consensus()
        h.DivideRounds()
        ph = h.phase_times()
        best = min(best, ph["coords_ms"])
    print(f"segs {s}: coords_ms {best:.3f} (used {ph['la_wave_segs']}, sweeps {ph['la_sweeps']}, fallbacks {ph['la_wave_fallbacks']})", flush=True)
h.L.hgx_set_la_kernel(h.ctx, 0)
