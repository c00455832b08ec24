"""Probe (CPU, numpy): distribution of the per-candidate first-seeing probe K(w) and of the
chain boundaries in the round recurrence on a prefix of a gossip trace, to
size search shortcuts for k_round_p.  python tools/probe/kdist.py [n] [events]"""
import sys
import os

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from babble_amd import trace  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
E = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
t = trace.gossip(n, E, 1)
sm = 2 * n // 3 + 1
cr = t.creator.astype(np.int64)
idx = t.index.astype(np.int64)
LA = np.full((E, n), -1, np.int32)
for x in range(E):
    row = LA[t.sp[x]].copy() if t.sp[x] >= 0 else np.full(n, -1, np.int32)
    if t.op[x] >= 0:
        np.maximum(row, LA[t.op[x]], out=row)
    row[cr[x]] = idx[x]
    LA[x] = row
chains = [np.nonzero(cr == c)[0] for c in range(n)]
L = np.array([len(ch) for ch in chains])
MAX = np.iinfo(np.int32).max
FD = np.full((E, n), MAX, np.int64)
for d in range(n):
    lad = LA[chains[d]]            # [len_d, n]
    for c in range(n):
        j = np.arange(L[c])
        k = np.searchsorted(lad[:, c], j, side="left")
        v = np.where(k < L[d], k, MAX)
        FD[chains[c], d] = v
P = 31
B = np.zeros(n, np.int64)
Ks, Bs, strides = [], [], []
r = 0
prev_stride = None
while True:
    live = B < L
    if not live.any():
        break
    cands = np.array([chains[c][B[c]] for c in range(n) if B[c] < L[c]])
    candc = np.array([c for c in range(n) if B[c] < L[c]])
    Fc = FD[cands]                                   # [m, n]
    Bn = B.copy()
    for c in range(n):
        if B[c] >= L[c]:
            continue
        k0 = B[c]
        found = None
        kb = k0
        while kb < L[c] and found is None:
            pr = chains[c][kb:kb + P]
            cnt = (LA[pr][:, None, :] >= Fc[None, :, :]).sum(-1) >= sm      # [np, m]
            self_ = (candc == c)
            if kb == k0:
                cnt[0, self_] = False
            K = np.where(cnt.any(0), cnt.argmax(0), P)
            h = np.bincount(np.minimum(K, P), minlength=P + 1)[:P].cumsum()
            bb = np.nonzero(h >= sm)[0]
            if kb == k0:
                Ks.append(K)
            if len(bb):
                found = kb + bb[0]
            else:
                kb += len(pr)
        Bn[c] = found if found is not None else L[c]
        if found is not None and kb == k0:
            Bs.append(found - k0)
    B = Bn
    r += 1
K = np.concatenate(Ks)
Bs = np.array(Bs)
print(f"n={n} E={E} rounds={r} chain-rounds={len(Bs)}")
print("boundary offset B: mean %.2f  pct 10/50/90 %s" % (Bs.mean(), np.percentile(Bs, [10, 50, 90])))
print("K(w) histogram (0..31):", np.bincount(K, minlength=P + 1).tolist())
print("frac K=0 %.3f  K=31(none) %.3f" % ((K == 0).mean(), (K == P).mean()))
