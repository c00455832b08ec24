"""Dev probe (CPU): would a per-chain incremental median pay for the consensus timestamps?

The timestamp of x is the upper median of ts(FD[x][d]) over the famous witnesses w_d of rr(x) that see x.
Along x's chain (fixed rr) an incremental median would keep the member multiset and apply, per step
x_p -> x_{p+1}, one replace for every d whose FD moved and one delete for every d that stopped seeing
x. This counts, over a c3-shaped trace (256 peers, seed 1), how many of the n values move per step, and
whether the timestamps along a chain are monotone (the reference does not require it: Event timestamps
are the creator's clock, event.go:44-52, so a median structure cannot assume sorted inputs).

    python tools/probe/cts_change_rate.py [E]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from babble_amd import trace  # noqa: E402

n = 256
E = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
_, _, _, silent, stale, depth, _ = bench.CONFIGS["c3"]
t = trace.gossip(n, E, 1, n_silent=silent, stale_prob=stale, stale_depth=depth)
cr = np.asarray(t.creator)
idx = np.asarray(t.index)
# lastAncestors in gid order (parents precede children): LA[x][d] = max over parents, own slot = Index
LA = np.full((E, n), -1, np.int32)
for x in range(E):
    row = LA[x]
    if t.sp[x] >= 0:
        np.maximum(row, LA[t.sp[x]], out=row)
    if t.op[x] >= 0:
        np.maximum(row, LA[t.op[x]], out=row)
    row[cr[x]] = idx[x]
# firstDescendants by the closed form: FD[x][d] = min{k on chain d : LA[(d,k)][cr(x)] >= Index(x)}
chains = [np.nonzero(cr == c)[0] for c in range(n)]
moved = []
tail_pos = []
for c in range(n):
    xs = chains[c]
    if len(xs) < 3:
        continue
    FDc = np.full((len(xs), n), -1, np.int64)
    for d in range(n):
        col = LA[chains[d], c]              # non-decreasing along chain d
        k = np.searchsorted(col, idx[xs], side="left")
        FDc[:, d] = np.where(k < len(col), k, -1)
    both = (FDc[1:] >= 0) & (FDc[:-1] >= 0)
    ch = (FDc[1:] != FDc[:-1]) & both
    denom = both.sum(axis=1)
    ok = denom > n // 2            # steps well inside the DAG (both events seen by most chains)
    moved.extend((ch.sum(axis=1)[ok] / denom[ok]).tolist())
mono = np.mean([np.all(np.diff(np.asarray(t.ts)[chains[c]]) >= 0) for c in range(n) if len(chains[c]) > 1])
m = np.asarray(moved)
print(f"E={E} n={n} steps={m.size}: fraction of the n firstDescendants that move per chain step: "
      f"mean {m.mean():.3f}, pct5/50/95 {np.percentile(m, [5, 50, 95]).round(3).tolist()}")
print(f"chains whose synthetic timestamps are monotone: {mono:.3f} (the reference does not require it)")
