"""The incremental DivideRounds/FindOrder schedule against the oracle.

The real caller runs consensus after every sync (Core.Sync + RunConsensus, node/core.go:
190-303; at most SyncLimit = 1000 events per sync, cmd/babble/main.go:83-85). Each call
extends lastAncestors/firstDescendants for the new events only, resumes the round steps at
the lowest round that can change, decides fame from the first undecided round and computes
roundReceived for the events not received yet. The oracle runs the same chunked schedule
(hgref.oracle_run(t, chunk)); the GPU results must be bit-exact, and equal to the
recompute-everything schedule (hgx_set_incremental(ctx, 0))."""
import numpy as np
import pytest

import hgref
from babble_amd import trace as gtrace
from test_gpu_parity import compare

pytestmark = pytest.mark.gpu


def _run_chunked(t, chunk, incremental=True, cap=None, graphs=1, stats=None):
    from babble_amd.hashgraph import Hashgraph
    h = Hashgraph(t.n, capacity=cap or max(64, t.E), n_graphs=graphs)
    h.set_incremental(incremental)
    for lo in range(0, t.E, chunk):
        h.insert_trace(t, lo, min(t.E, lo + chunk))
        h.RunConsensus()
        if stats is not None:
            stats.append(h.phase_times())
    return h


@pytest.mark.parametrize("n,E,seed,chunk,silent,stale", [
    (64, 20000, 41, 1000, 0, 0.0),     # SyncLimit chunks
    (64, 12000, 42, 333, 0, 0.25),     # stale other-parents
    (128, 20000, 45, 1000, 20, 0.0),   # silent peers (chains that never grow)
    (256, 40000, 43, 1000, 0, 0.0),    # C3's n, compact coordinates
    (600, 30000, 47, 2000, 150, 0.2),  # n > 256: candidate chunks, silent and stale peers
    (16, 2000, 44, 1, 0, 0.1),         # one event per call
    (5, 900, 46, 17, 1, 0.3)])
def test_chunked_matches_oracle(n, E, seed, chunk, silent, stale):
    t = gtrace.gossip(n, E, seed, n_silent=silent, stale_prob=stale, stale_depth=3)
    stats = []
    h = _run_chunked(t, chunk, stats=stats)
    compare(h, hgref.oracle_run(t, chunk=chunk), t, hashes=E <= 6000)
    # after the first call, no call rebuilt the layout, and each recomputed only the
    # lastAncestors rows of the units holding its new events, once per sweep (~10 sweeps)
    assert stats[0]["rebuild"] == 1
    assert all(s["rebuild"] == 0 for s in stats[1:])
    seg = 16
    bound = chunk + n * seg
    assert max(s["la_rows"] for s in stats[1:]) <= 16 * bound
    assert stats[-1]["r_lo"] > 0 or stats[-1]["rounds"] < 3


@pytest.mark.parametrize("n,E,seed,chunk", [(64, 8000, 51, 500), (256, 30000, 52, 1000)])
def test_incremental_equals_full_recompute(n, E, seed, chunk):
    t = gtrace.gossip(n, E, seed, stale_prob=0.1, stale_depth=2)
    a = _run_chunked(t, chunk, incremental=True).results()
    b = _run_chunked(t, chunk, incremental=False).results()
    for k in ("round", "witness", "famous", "rr", "cts"):
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k
    assert list(a["order"]) == list(b["order"])
    for k in ("last_round", "undecided", "lcr", "lcre", "consensus_tx", "pending_loaded", "blocks"):
        assert a[k] == b[k], k


def _interleave(traces, per_call):
    """One batched-context stream: call k inserts the k-th slice (per_call[g] events) of
    every graph g, gids renumbered in that order; returns the stream, the gid of every
    graph event and the number of events per call."""
    n = traces[0].n
    G = len(traces)
    pos = [0] * G
    gid_of = [np.zeros(t.E, np.int64) for t in traces]
    cols = {k: [] for k in ("creator", "index", "sp", "op", "ts", "hash", "s", "ntx", "txnil", "tx_seq")}
    calls, nxt = [], 0
    while any(pos[g] < traces[g].E for g in range(G)):
        start = nxt
        for g, t in enumerate(traces):
            lo, hi = pos[g], min(t.E, pos[g] + per_call[g])
            for i in range(lo, hi):
                gid_of[g][i] = nxt
                nxt += 1
            sl = slice(lo, hi)
            cols["creator"].append(t.creator[sl] + g * n)
            for k in ("index", "ts", "hash", "s", "ntx", "txnil", "tx_seq"):
                cols[k].append(getattr(t, k)[sl])
            for k in ("sp", "op"):
                v = getattr(t, k)[sl]
                cols[k].append(np.where(v >= 0, gid_of[g][np.maximum(v, 0)], v))
            pos[g] = hi
        calls.append(nxt - start)
    st = gtrace.GossipTrace(n, **{k: np.concatenate(v) for k, v in cols.items()})
    return st, gid_of, calls


def test_chunked_layout_rebuild_on_slot_overflow():
    """Batched graphs growing at very different rates: the big graph's chains outgrow the
    slack of the layout, which is rebuilt (events received earlier keep their rr)."""
    from babble_amd.hashgraph import Hashgraph
    n, per_call, calls = 16, [600, 20, 20, 20], 20
    traces = [gtrace.gossip(n, p * calls, 600 + g) for g, p in enumerate(per_call)]
    st, gid_of, sizes = _interleave(traces, per_call)
    G = len(traces)
    h = Hashgraph(n, capacity=st.E, n_graphs=G)
    oracles = [hgref.Oracle(n) for _ in range(G)]
    rebuilds, lo = 0, 0
    for k, m in enumerate(sizes):
        h.insert_trace(st, lo, lo + m)
        h.RunConsensus()
        rebuilds += h.phase_times()["rebuild"]
        lo += m
        for g, t in enumerate(traces):
            oracles[g].insert_trace(t, k * per_call[g], min(t.E, (k + 1) * per_call[g]))
            oracles[g].run_consensus()
    assert rebuilds >= 2
    for g, t in enumerate(traces):
        r = oracles[g].results()
        inv = {int(x): i for i, x in enumerate(gid_of[g])}
        assert [inv[int(x)] for x in h.ConsensusEvents(g)] == list(r["order"]), g
        assert h.UndecidedRounds(g) == r["undecided"], g
        assert h.LastConsensusRound(g) == r["lcr"], g
        assert h.ConsensusTransactions(g) == r["consensus_tx"], g
