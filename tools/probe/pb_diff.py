"""Probe: k_round_pb ("auto") against the per-launch steps ("auto-steps") on a grid of traces; for
each mismatch the first differing (round, chain) and both boundary rows around it."""
import sys

import numpy as np

from babble_amd import trace as gtrace
from babble_amd.hashgraph import Hashgraph


def run(t, mode):
    h = Hashgraph(t.n, capacity=max(64, t.E))
    h.set_round_kernel(mode)
    h.insert_trace(t)
    h.RunConsensus()
    return h


def bounds(rnd, creator, n):
    """per chain: first index of each round (from the per-event rounds, gid order = index order)"""
    out = {}
    for c in range(n):
        r = rnd[creator == c]
        out[c] = r
    return out


def main():
    grid = [(258, 16000, 0.0), (258, 16000, 0.2), (300, 16000, 0.0), (300, 16000, 0.2), (320, 16000, 0.2),
            (384, 16000, 0.0), (384, 16000, 0.2), (448, 16000, 0.2), (512, 16000, 0.0), (512, 16000, 0.2),
            (384, 60000, 0.0), (700, 60000, 0.2)]
    if len(sys.argv) > 1:
        grid = [tuple(float(x) if "." in x else int(x) for x in a.split(",")) for a in sys.argv[1:]]
    for (n, E, stale) in grid:
        t = gtrace.gossip(n, E, 103, stale_prob=stale, stale_depth=4)
        hp, hk = run(t, "auto"), run(t, "auto-steps")
        ph = hp.phase_times()
        a, b = np.asarray(hp.results()["round"]), np.asarray(hk.results()["round"])
        bad = np.nonzero(a != b)[0]
        print(f"n={n} E={E} stale={stale} runs={ph['round_p_runs']} fb={ph['round_p_fallbacks']} "
              f"ovf={ph.get('round_p_ovf')} last={hp.results()['last_round']}/{hk.results()['last_round']} "
              f"mismatch={len(bad)}", flush=True)
        if len(bad):
            cr = np.asarray(t.creator)
            g0 = int(bad[0])
            c = int(cr[g0])
            idx = np.nonzero(cr == c)[0]
            k = int(np.searchsorted(idx, g0))
            lo, hi = max(0, k - 40), min(len(idx), k + 10)
            print(f"  first gid {g0} chain {c} index {k}: pb {a[idx[lo:hi]].tolist()}", flush=True)
            print(f"  {' ' * (len(str(g0)) + len(str(c)) + len(str(k)) + 27)}steps {b[idx[lo:hi]].tolist()}", flush=True)
            # the lowest differing round over all chains
            rmin = int(min(a[bad].min(), b[bad].min()))
            chains = sorted(set(int(cr[g]) for g in bad if min(a[g], b[g]) == rmin))
            print(f"  lowest differing round {rmin}: chains {chains[:20]} ({len(chains)})", flush=True)


if __name__ == "__main__":
    main()
