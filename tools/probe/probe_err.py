import sys, time
sys.path.insert(0, '.')
from babble_amd import trace
from babble_amd.hashgraph import Hashgraph
for E in (200_000, 2_000_000):
    for timing in (False, True):
        t = trace.gossip(256, E, 1)
        h = Hashgraph(256, capacity=t.E)
        h.set_kernel_timing(timing)
        h.insert_trace(t)
        for nm in ("DivideRounds", "DecideFame", "FindOrder"):
            try:
                getattr(h, nm)()
                print(E, timing, nm, "ok", flush=True)
            except Exception as e:
                print(E, timing, nm, "FAILED", e, flush=True)
                break
        print(h.phase_times(), flush=True)
        h.close()
