"""Probe: the persistent round recurrence on one large graph (c3 shape) at growing sizes;
prints phase times (round_p_runs / fallbacks / give-up round and chain) per call and every
error raised. Usage: python tools/probe/round_p_sizes.py [n] [E1,E2,...] [passes]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from babble_amd import trace  # noqa: E402
from babble_amd.hashgraph import Hashgraph  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
sizes = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1000000,3000000,10000000").split(",")]
passes = int(sys.argv[3]) if len(sys.argv) > 3 else 2
for E in sizes:
    t = trace.gossip(n, E, 1)
    h = Hashgraph(n, capacity=E)
    for p in range(passes):
        t0 = time.time()
        try:
            h.clear()
            h.insert_trace(t)
            h.DivideRounds()
            ph = h.phase_times()
            h.DecideFame()
            h.FindOrder()
            print(f"E={E} pass {p}: {time.time() - t0:.3f}s ordered {len(h.ConsensusEvents())} "
                  f"rounds_ms {ph['rounds_ms']:.2f} runs {ph['round_p_runs']} fallbacks {ph['round_p_fallbacks']} "
                  f"give-up round {ph['round_p_fail_round']} chain {ph['round_p_fail_chain']} R {ph['rounds']}",
                  flush=True)
        except Exception as e:
            print(f"E={E} pass {p}: ERROR {e!r} phases {h.phase_times()}", flush=True)
            break
    h.close()
