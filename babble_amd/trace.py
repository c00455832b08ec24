"""Synthetic gossip traces (structure of arrays) produced by libhgx's generator.

The generator models the reference's deterministic gossip harness
(node/core_test.go:514-537, node/core.go:215-227); see include/hgx.h
hgx_trace_gossip for the exact rules.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from . import _lib


@dataclass
class GossipTrace:
    n: int
    creator: np.ndarray   # int32 [E]
    index: np.ndarray     # int64 [E]
    sp: np.ndarray        # int64 [E] (-1 = "")
    op: np.ndarray        # int64 [E]
    ts: np.ndarray        # int64 [E] unix ns
    hash: np.ndarray      # uint8 [E, 32]
    s: np.ndarray         # uint8 [E, 32]
    ntx: np.ndarray       # int32 [E]
    txnil: np.ndarray     # int32 [E]
    tx_seq: np.ndarray    # int64 [E] (-1 = no payload)

    @property
    def E(self) -> int:
        return int(self.creator.shape[0])

    def tx_payload(self, i: int) -> List[bytes]:
        if self.ntx[i] == 0:
            return []
        return [payload(int(self.creator[i]), int(self.tx_seq[i]))]

    def txs(self, i: int) -> Optional[List[bytes]]:
        return None if self.txnil[i] else self.tx_payload(i)


def payload(creator: int, seq: int) -> bytes:
    L = _lib.lib()
    buf = (_lib.C.c_uint8 * 64)()
    n = L.hgx_trace_tx_payload(creator, seq, buf, 64)
    return bytes(buf[:n])


def gossip(n: int, n_events: int, seed: int, n_silent: int = 0, stale_prob: float = 0.0,
           stale_depth: int = 1) -> GossipTrace:
    L = _lib.lib()
    E = int(n_events)
    t = GossipTrace(
        n=n,
        creator=np.zeros(E, np.int32), index=np.zeros(E, np.int64), sp=np.zeros(E, np.int64),
        op=np.zeros(E, np.int64), ts=np.zeros(E, np.int64), hash=np.zeros((E, 32), np.uint8),
        s=np.zeros((E, 32), np.uint8), ntx=np.zeros(E, np.int32), txnil=np.zeros(E, np.int32),
        tx_seq=np.zeros(E, np.int64))
    P = _lib.ptr
    rc = L.hgx_trace_gossip(n, n_silent, E, seed & 0xFFFFFFFFFFFFFFFF, float(stale_prob), int(stale_depth),
                            P(t.creator), P(t.index), P(t.sp), P(t.op), P(t.ts), P(t.hash), P(t.s),
                            P(t.ntx), P(t.txnil), P(t.tx_seq))
    if rc != 0:
        raise ValueError(f"hgx_trace_gossip failed ({rc})")
    return t


def concat_graphs(traces: List[GossipTrace]) -> GossipTrace:
    """Batch of independent graphs for a batched context: graph g's participants become
    g*n .. g*n+n-1 and its parent gids are offset by the events before it."""
    n = traces[0].n
    off = 0
    parts = []
    for g, t in enumerate(traces):
        assert t.n == n
        sp = np.where(t.sp >= 0, t.sp + off, t.sp)
        op = np.where(t.op >= 0, t.op + off, t.op)
        parts.append((t.creator + g * n, t.index, sp, op, t.ts, t.hash, t.s, t.ntx, t.txnil, t.tx_seq))
        off += t.E
    cat = [np.concatenate([p[k] for p in parts]) for k in range(10)]
    return GossipTrace(n, *cat)
