"""Test-only numpy model of the GPU formulation used by libhgx.

It restates, in plain array code, the data-parallel reformulation the HIP kernels
implement -- NOT the reference loop structure (that is the oracle's job):
  * lastAncestors  = max over ancestors (fixed point)        (hashgraph.go:448-499)
  * firstDescendants via lower_bound on monotone LA columns   
  * rounds via per-chain boundaries B_r(c) against candidate sets W'_r
  * fame via strongly-see bit matrices and vote tallies      
  * round-received via per-(round, creator) thresholds      
  * consensus timestamp = upper median of first-descendant timestamps
  * order = sort by (rr, cts, S) ; blocks by rr
and the host bookkeeping (UndecidedRounds, LastConsensusRound, late witnesses) for
batch and chunked schedules. tests/test_parallel_model.py checks it against the oracle.
"""
from __future__ import annotations

import numpy as np

MAXI32 = 2147483647


def super_majority(n):
    return 2 * n // 3 + 1


class Model:
    def __init__(self, n):
        self.n = n
        self.sm = super_majority(n)
        self.E = 0
        self.creator = np.zeros(0, np.int64)
        self.index = np.zeros(0, np.int64)
        self.sp = np.zeros(0, np.int64)
        self.op = np.zeros(0, np.int64)
        self.ts = np.zeros(0, np.int64)
        self.S = np.zeros((0, 32), np.uint8)
        self.coin = np.zeros(0, bool)
        self.ntx = np.zeros(0, np.int64)
        self.loaded = np.zeros(0, bool)
        self.txnil = np.zeros(0, bool)
        # persistent host state (Go bookkeeping)
        self.rr = np.zeros(0, np.int64)
        self.cts = np.zeros(0, np.int64)
        self.undecided = [0]
        self.queued_upto = -1            # rounds <= queued_upto have been queued
        self.fame = {}                   # (round, chain) -> 0/1/2, host state (frozen once decided)
        self.lcr = None
        self.lcre = 0
        self.consensus = []
        self.consensus_tx = 0
        self.pending_loaded = 0
        self.divided = 0                 # events registered by DivideRounds
        self.blocks = []

    def insert(self, t, lo, hi):
        sl = slice(lo, hi)
        cat = np.concatenate
        self.creator = cat([self.creator, t.creator[sl].astype(np.int64)])
        self.index = cat([self.index, t.index[sl].astype(np.int64)])
        self.sp = cat([self.sp, t.sp[sl].astype(np.int64)])
        self.op = cat([self.op, t.op[sl].astype(np.int64)])
        self.ts = cat([self.ts, t.ts[sl].astype(np.int64)])
        self.S = cat([self.S, t.s[sl]])
        self.coin = cat([self.coin, t.hash[sl, 16] != 0])
        self.ntx = cat([self.ntx, t.ntx[sl].astype(np.int64)])
        self.txnil = cat([self.txnil, t.txnil[sl] != 0])
        ld = (t.index[sl] == 0) | ((t.txnil[sl] == 0) & (t.ntx[sl] > 0))
        self.loaded = cat([self.loaded, ld])
        self.rr = cat([self.rr, np.full(hi - lo, -1, np.int64)])
        self.cts = cat([self.cts, np.zeros(hi - lo, np.int64)])
        self.pending_loaded += int(ld.sum())
        self.E = len(self.creator)

    # ------------------------------------------------------------------ pure (DAG) part
    def coordinates(self):
        n, E = self.n, self.E
        LA = np.full((E, n), -1, np.int64)
        for x in range(E):                       # fixed point of max over parents
            row = LA[self.sp[x]].copy() if self.sp[x] >= 0 else np.full(n, -1)
            if self.op[x] >= 0:
                row = np.maximum(row, LA[self.op[x]])
            row[self.creator[x]] = self.index[x]
            LA[x] = row
        self.chains = [np.where(self.creator == c)[0] for c in range(n)]
        self.base = np.array([self.index[ch[0]] if len(ch) else 0 for ch in self.chains])
        FD = np.full((E, n), MAXI32, np.int64)
        for c in range(n):
            ch = self.chains[c]
            if not len(ch):
                continue
            for d in range(n):
                col = LA[ch, d]                  # monotone non-decreasing along chain c
                yd = self.chains[d]
                if not len(yd):
                    continue
                k = np.searchsorted(col, self.index[yd], side="left")
                ok = k < len(ch)
                FD[yd[ok], c] = self.index[ch[k[ok]]]
        self.LA, self.FD = LA, FD

    def ss(self, x, w):
        return int((self.LA[x] >= self.FD[w]).sum()) >= self.sm

    def rounds(self):
        n = self.n
        L = [len(ch) for ch in self.chains]
        B = [0] * n
        rnd = np.full(self.E, -1, np.int64)
        wit = np.zeros(self.E, bool)
        self.cand = []                           # per round: {chain: gid} of W'_r
        self.W = []                              # per round: {chain: gid} witnesses
        r = 0
        while True:
            cands = {c: int(self.chains[c][B[c]]) for c in range(n) if B[c] < L[c]}
            if not cands:
                break
            Bn = []
            for c in range(n):
                k = B[c]
                while k < L[c]:
                    x = int(self.chains[c][k])
                    cnt = sum(1 for w in cands.values() if w != x and self.ss(x, w))
                    if cnt >= self.sm:
                        break
                    k += 1
                Bn.append(k)
            wr = {}
            for c in range(n):
                if B[c] < L[c]:
                    rnd[self.chains[c][B[c]:Bn[c]]] = r
                    if Bn[c] > B[c]:
                        wit[self.chains[c][B[c]]] = True
                        wr[c] = int(self.chains[c][B[c]])
            self.cand.append(cands)
            self.W.append(wr)
            B = Bn
            r += 1
        self.round, self.witness = rnd, wit
        self.last_round = r - 1

    # ------------------------------------------------------------------ fame (per call)
    def fame_decisions(self):
        """Device fame for every witness given the current DAG: 1/2 decided, 0 not."""
        n, sm, LR = self.n, self.sm, self.last_round
        dec = {}
        for i in range(LR + 1):
            xs = self.W[i]
            und = set(xs)
            if i + 1 > LR:
                for c in xs:
                    dec[(i, c)] = 0
                continue
            # j = i+1: votes = See(y, x)
            V = {c: {yc for yc, y in self.W[i + 1].items() if self.LA[y, self.creator[x]] >= self.index[x]}
                 for c, x in xs.items()}
            res = {c: 0 for c in xs}
            for j in range(i + 2, LR + 1):
                if not und:
                    break
                diff = j - i
                prev = self.W[j - 1]
                Sj = {yc: {wc for wc, w in prev.items() if self.ss(y, w)} for yc, y in self.W[j].items()}
                newV = {}
                for c in list(und):
                    vote = set()
                    decided = None
                    for yc, y in self.W[j].items():
                        ss = Sj[yc]
                        yays = len(ss & V[c])
                        nays = len(ss) - yays
                        v = yays >= nays
                        t = yays if v else nays
                        if diff % n > 0:
                            if t >= sm:
                                decided = v
                                break
                            if v:
                                vote.add(yc)
                        else:
                            if (v if t >= sm else bool(self.coin[y])):
                                vote.add(yc)
                    if decided is not None:
                        res[c] = 1 if decided else 2
                        und.discard(c)
                    else:
                        newV[c] = vote
                for c in und:
                    V[c] = newV[c]
            for c in xs:
                dec[(i, c)] = res[c]
        return dec

    # ------------------------------------------------------------------ Go calls
    def divide_rounds(self):
        self.coordinates()
        self.rounds()
        self.divided = self.E
        for r in range(self.queued_upto + 1, self.last_round + 1):
            self.undecided.append(r)
        self.queued_upto = max(self.queued_upto, self.last_round)

    def round_events(self, r):
        return int((self.round[:self.divided] == r).sum()) if r >= 0 else 0

    def witnesses_decided(self, r):
        if r < 0 or r > self.last_round:
            return True
        return all(self.fame.get((r, c), 0) != 0 for c in self.W[r])

    def decide_fame(self):
        dec = self.fame_decisions()
        decided_rounds = set()
        for pos, i in enumerate(self.undecided):
            if i > self.last_round:
                raise RuntimeError(f"{i}, Not Found")
            for c in self.W[i]:
                if self.fame.get((i, c), 0) == 0 and dec[(i, c)] != 0:
                    self.fame[(i, c)] = dec[(i, c)]
            if self.witnesses_decided(i):
                decided_rounds.add(i)
                if self.lcr is None or i > self.lcr:
                    self.lcr = i
                    self.lcre = self.round_events(i - 1)
        self.undecided = [r for r in self.undecided if r not in decided_rounds]

    def find_order(self):
        n = self.n
        U0 = self.undecided[0] if self.undecided else None
        LR = self.last_round
        elig = [U0 is not None and i < U0 and self.witnesses_decided(i) for i in range(LR + 1)]
        # thresholds T[i][d] = (m//2+1)-th largest LA[w][d] over famous w of round i
        T = {}
        FW = {}
        for i in range(LR + 1):
            if not elig[i]:
                continue
            fws = [w for c, w in self.W[i].items() if self.fame.get((i, c), 0) == 1]
            FW[i] = fws
            m = len(fws)
            for d in range(n):
                vals = sorted((self.LA[w, d] for w in fws), reverse=True)
                T[(i, d)] = vals[m // 2] if m // 2 < m else -1
        newc = []
        for x in range(self.divided):
            if self.rr[x] >= 0:
                continue
            d, j = self.creator[x], self.index[x]
            for i in range(self.round[x] + 1, LR + 1):
                if U0 is None:
                    raise RuntimeError("runtime error: index out of range")
                if elig[i] and j <= T[(i, d)]:
                    self.rr[x] = i
                    tl = []
                    for w in FW[i]:
                        if self.LA[w, d] >= j:
                            c = self.creator[w]
                            fd = self.FD[x, c]
                            a = self.chains[c][fd - self.base[c]]
                            tl.append(self.ts[a])
                    tl.sort()
                    self.cts[x] = tl[len(tl) // 2]
                    newc.append(x)
                    break
        newc.sort(key=lambda x: (self.rr[x], self.cts[x], self.S[x].tobytes()))
        for x in newc:
            self.consensus.append(x)
            self.consensus_tx += int(self.ntx[x])
            if self.loaded[x]:
                self.pending_loaded -= 1
            if self.blocks and self.blocks[-1]["first_call"] == len(self.calls_marker) and \
                    self.blocks[-1]["rr"] == self.rr[x]:
                b = self.blocks[-1]
            else:
                b = dict(rr=int(self.rr[x]), ev=[], ntx=0, nil=bool(self.txnil[x]),
                         first_call=len(self.calls_marker))
                self.blocks.append(b)
            b["ev"].append(x)
            b["ntx"] += int(self.ntx[x])
            if self.ntx[x] > 0:
                b["nil"] = False
        self.calls_marker.append(1)

    calls_marker: list

    def run_consensus(self):
        if not hasattr(self, "calls_marker") or self.calls_marker is Model.__dict__.get("calls_marker"):
            self.calls_marker = []
        self.divide_rounds()
        self.decide_fame()
        self.find_order()


def model_run(t, chunk=None):
    m = Model(t.n)
    m.calls_marker = []
    if chunk is None:
        m.insert(t, 0, t.E)
        m.divide_rounds(); m.decide_fame(); m.find_order()
    else:
        for lo in range(0, t.E, chunk):
            m.insert(t, lo, min(t.E, lo + chunk))
            m.divide_rounds(); m.decide_fame(); m.find_order()
    return m
