"""Dev probe (CPU): how predictable is a chain's boundary advance per round? The oracle's rounds of a
c3-shaped trace (256 peers, seed 1, E events); Bm[s][c] = first offset of chain c with round >= s.
    python tools/probe/round_advance.py [E]"""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT]
import hgref, bench
from babble_amd import trace
n, E = 256, int(sys.argv[1]) if len(sys.argv) > 1 else 120000
cfg = bench.CONFIGS['c3']
_, _, _, silent, stale, depth, _ = cfg
t = trace.gossip(n, E, 1, n_silent=silent, stale_prob=stale, stale_depth=depth)
o = hgref.Oracle(n)
t0 = time.time(); o.insert_trace(t); o.divide_rounds(); print("oracle", time.time() - t0, file=sys.stderr)
L = o.L
L.hgo_round.restype = C.c_int
rnd = np.array([L.hgo_round(o.h, x) for x in range(t.E)])
cr = np.asarray(t.creator)
R = rnd.max() + 1
# boundary Bm[s][c] = first offset on chain c with round >= s
Bm = np.zeros((R + 1, n), np.int64)
for c in range(n):
    rc = rnd[cr == c]
    Bm[:, c] = np.searchsorted(np.maximum.accumulate(rc), np.arange(R + 1), side='left')
d = np.diff(Bm, axis=0)   # advance per round
print("rounds", R, "mean adv", d.mean(), "pct", np.percentile(d, [5, 25, 50, 75, 95, 99]))
prev = d[:-1]; cur = d[1:]
for k in (0, 1, 2):
    print("|cur-prev|<=", k, np.mean(np.abs(cur - prev) <= k))
# predictor: median of the chain's last 4 advances / global previous-round median
