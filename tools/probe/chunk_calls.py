"""Host wall time per call of the chunked schedule, by call (insert / DivideRounds / DecideFame /
FindOrder), against the device phase times."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from babble_amd import trace as gtrace  # noqa: E402
from babble_amd.hashgraph import DeviceTrace, Hashgraph  # noqa: E402

n, E, chunk = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
t = gtrace.gossip(n, E, 1)
h = Hashgraph(n, capacity=E)
dt = DeviceTrace(t)
acc = np.zeros(8)
calls = 0
for lo in range(0, E, chunk):
    t0 = time.perf_counter(); h.insert_device(dt, lo, min(E, lo + chunk))
    t1 = time.perf_counter(); h.DivideRounds()
    t2 = time.perf_counter(); h.DecideFame()
    t3 = time.perf_counter(); h.FindOrder()
    t4 = time.perf_counter()
    p = h.phase_times()
    if lo >= E // 4:
        acc += [t1 - t0, t2 - t1, t3 - t2, t4 - t3, p["coords_ms"] * 1e-3, p["rounds_ms"] * 1e-3, p["fame_ms"] * 1e-3,
                p["order_ms"] * 1e-3]
        calls += 1
acc = acc / calls * 1e6
print(f"n={n} E={E} chunk={chunk}: us/call host insert {acc[0]:.0f} divide {acc[1]:.0f} fame {acc[2]:.0f} "
      f"order {acc[3]:.0f} | device coords {acc[4]:.0f} rounds {acc[5]:.0f} fame {acc[6]:.0f} order {acc[7]:.0f}",
      flush=True)
