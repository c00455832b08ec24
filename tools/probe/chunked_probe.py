"""Per-call cost of the incremental schedule: RunConsensus every `chunk` inserted events
(SyncLimit), on a config's trace or a prefix of it."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from babble_amd import trace as gtrace  # noqa: E402
from babble_amd.hashgraph import Hashgraph, DeviceTrace  # noqa: E402

n, E, chunk = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
full = int(sys.argv[4]) if len(sys.argv) > 4 else 0
timing = int(sys.argv[5]) if len(sys.argv) > 5 else 0
t = gtrace.gossip(n, E, 1)
h = Hashgraph(n, capacity=E)
if full:
    h.set_incremental(False)
dt = DeviceTrace(t)
if timing:
    h.set_kernel_timing(True)
calls, worst, t0 = 0, 0.0, time.perf_counter()
phase = np.zeros(4)
for lo in range(0, E, chunk):
    c0 = time.perf_counter()
    h.insert_device(dt, lo, min(E, lo + chunk))
    h.RunConsensus()
    c1 = time.perf_counter()
    worst = max(worst, c1 - c0)
    p = h.phase_times()
    phase += [p["coords_ms"], p["rounds_ms"], p["fame_ms"], p["order_ms"]]
    calls += 1
    if calls % 500 == 0:
        print(f"{calls} calls, {lo + chunk} events, {time.perf_counter() - t0:.2f}s", flush=True)
el = time.perf_counter() - t0
ordered = len(h.ConsensusEvents())
print(f"n={n} E={E} chunk={chunk} full={full}: {calls} calls in {el:.3f}s = {el / calls * 1e3:.3f} ms/call "
      f"(worst {worst * 1e3:.2f} ms), {E / el / 1e6:.3f} M inserted ev/s, {ordered} ordered; "
      f"device ms/call coords {phase[0] / calls:.3f} rounds {phase[1] / calls:.3f} fame {phase[2] / calls:.3f} "
      f"order {phase[3] / calls:.3f}", flush=True)
if timing:
    for k, v in h.kernel_stats().items():
        print(f"  {k:15s} {v['ms'] / calls * 1e3:8.1f} us/call  {v['launches'] / calls:6.2f} launches/call", flush=True)
