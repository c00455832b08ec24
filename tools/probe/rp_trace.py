"""Dev probe: per-(round, chain) stamps of the persistent round launch (prof build, HGX_RP_TRACE_FILE)
and what sets each round's period.  HGX_LIB=libhgx_prof.so python tools/probe/rp_trace.py c3"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from babble_amd.hashgraph import Hashgraph  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
out = os.path.join(ROOT, "gpurun_out", f"rp_trace_{cfg}.bin")
os.environ["HGX_RP_TRACE_FILE"] = out
n, E, G, *_ = bench.CONFIGS[cfg]
tr, G = bench.make_trace(cfg, 0)
h = Hashgraph(n, capacity=tr.E, device=0, n_graphs=G)
h.insert_trace(tr)
for rep in range(2):
    h.reset_consensus()
    h.DivideRounds()
print("phases", h.phase_times(), flush=True)
R = int(h.phase_times()["rounds"])
C = n * G
TT = np.fromfile(out, np.uint32).reshape(4096, 256, 8)[:R, :C].astype(np.int64)
T = TT[:, :, :4]
W1 = TT[:, :, 4:]
rnd = h.results()["round"] if hasattr(h, "results") else None
# Bm[r][c] from the event rounds
cr = tr.creator
Bm = np.zeros((R + 1, C), np.int64)
for c in range(C):
    rc = np.sort(rnd[cr == c])
    Bm[:, c] = np.searchsorted(rc, np.arange(R + 1), side="left")
t0, t1, t2, t3 = (T[:, :, k] for k in range(4))
base = t2.min()
ok = (t2 > 0).all(axis=1)
lo, hi = 10, R - 10
rs = np.arange(lo, hi)
pmax = t2[rs].max(1)
period = np.diff(t2[lo - 1:hi].max(1))
print(f"rounds {R}, period (10 ns ticks): median {np.median(period):.0f} mean {period.mean():.1f} "
      f"p10 {np.percentile(period, 10):.0f} p90 {np.percentile(period, 90):.0f}")
skew = t2[rs].max(1) - t2[rs].min(1)
print(f"publish skew per round: median {np.median(skew):.0f} p90 {np.percentile(skew, 90):.0f}")
# per chain, per round: hop = poll done - last publish of the previous round
prevmax = t2[rs - 1].max(1)[:, None]
hop = t0[rs] - prevmax
search = t1[rs] - t0[rs]
pub = t2[rs] - t1[rs]
endb = t3[rs] - t2[rs]
for nm, a in (("poll-done - prev last publish", hop), ("poll->boundary", search), ("boundary->publish", pub),
              ("publish->end", endb), ("end->next poll done", t0[rs + 1] - t3[rs])):
    print(f"{nm:32s} median {np.median(a):6.0f} mean {a.mean():7.1f} p90 {np.percentile(a, 90):6.0f} max {a.max():6.0f}")
# the slowest publisher of each round: its breakdown and what distinguishes it
am = t2[rs].argmax(1)
sl = lambda a: a[np.arange(len(rs)), am]
print("slowest chain per round: hop %.0f search %.0f publish %.0f" % (np.median(sl(hop)), np.median(sl(search)), np.median(sl(pub))))
adv = (Bm[rs + 1] - Bm[rs])
staged = ((Bm[rs] // 32 + 3) > (Bm[rs - 1] // 32 + 3))   # a new ring segment this round
print("slowest: adv median %.1f (all %.1f); staged frac %.2f (all %.2f)" % (
    np.median(sl(adv)), np.median(adv), sl(staged).mean(), staged.mean()))
print("search time staged vs not: %.0f / %.0f" % (np.median(search[staged]), np.median(search[~staged])))
xcd = np.arange(C) % 8
print("search median by blockIdx %% 8:", [int(np.median(search[:, xcd == k])) for k in range(8)])
print("hop median by blockIdx %% 8:", [int(np.median(hop[:, xcd == k])) for k in range(8)])

# wave 1 (a rebasing wave): its poll completion vs wave 0's, its (e) length
w0p, w1p = t0[rs], W1[rs, :, 0]
w1e = W1[rs, :, 2] - W1[rs, :, 1]
print("wave1 poll done - wave0 poll done: median %.0f p90 %.0f" % (np.median(w1p - w0p), np.percentile(w1p - w0p, 90)))
print("wave1 (e) (S row + rebase) median %.0f p90 %.0f; wave0 (e) (publish) median %.0f" % (
    np.median(w1e), np.percentile(w1e, 90), np.median(t2[rs] - t1[rs])))
print("wave1: end -> its poll done median %.0f; wave0: end -> poll done median %.0f" % (
    np.median(W1[rs + 1, :, 0] - W1[rs, :, 3]), np.median(t0[rs + 1] - t3[rs])))

# every wave of rounds [100, 164): poll done and end of round
Wv = np.fromfile(out + ".waves", np.uint32).reshape(64, 256, 16, 2)[:, :C].astype(np.int64)
pd, en = Wv[..., 0], Wv[..., 1]
late = pd - pd.min(axis=2, keepdims=True)
print("per-wave poll done - first wave's (median over rounds/chains):", [int(np.median(late[:, :, w])) for w in range(min(16, late.shape[2]))])
last = pd.argmax(axis=2)
print("which wave polls last (counts):", np.bincount(last.ravel(), minlength=16).tolist())
ee = en[:-1] - en[:-1].min(axis=2, keepdims=True)
print("per-wave end of (e) - first (median):", [int(np.median(ee[:, :, w])) for w in range(16)])
wait = pd[1:] - en[:-1]
print("per-wave end -> next poll done (median):", [int(np.median(wait[:, :, w])) for w in range(16)])
