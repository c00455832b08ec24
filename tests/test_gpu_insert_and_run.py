"""hgx_insert_and_run: Bootstrap / Core.Sync + RunConsensus in one call, with the payload
columns (timestamps, hash, S, transactions) copied to HBM while DivideRounds runs
(hashgraph.go:1008-1037, node/core.go:190-303). Every output must equal the two-call path
(hgx_insert_events + hgx_run_consensus) and the oracle: the payload is committed before
DecideFame reads the coins, the layout's timestamps are rewritten, PendingLoadedEvents counts
the batch's loaded events, and an insert error leaves the accepted prefix inserted."""
import numpy as np
import pytest

import hgref
from babble_amd import trace as gtrace
from test_gpu_parity import compare

pytestmark = pytest.mark.gpu


def _hg(n, cap, graphs=1):
    from babble_amd.hashgraph import Hashgraph
    return Hashgraph(n, capacity=cap, n_graphs=graphs)


def _same(a, b, graphs=1):
    for g in range(graphs):
        x, y = a.results(g), b.results(g)
        for k in ("round", "witness", "famous", "rr", "cts"):
            assert np.array_equal(np.asarray(x[k]), np.asarray(y[k])), (g, k)
        assert list(x["order"]) == list(y["order"]), g
        for k in ("last_round", "undecided", "lcr", "lcre", "consensus_tx", "pending_loaded"):
            assert x[k] == y[k], (g, k)
        assert [(v["rr"], v["ntx"], v["tx_nil"], v["committed"]) for v in x["blocks"]] == \
            [(v["rr"], v["ntx"], v["tx_nil"], v["committed"]) for v in y["blocks"]], g


@pytest.mark.parametrize("n,E,seed", [(16, 70000, 1), (64, 120000, 2), (256, 200000, 3)])
def test_one_call_equals_two_calls_and_oracle(n, E, seed):
    t = gtrace.gossip(n, E, seed, stale_prob=0.1, stale_depth=3)
    a = _hg(n, E)
    assert a.insert_and_run(t) == E
    b = _hg(n, E)
    b.insert_trace(t)
    b.RunConsensus()
    _same(a, b)
    if n <= 64:
        compare(a, hgref.oracle_run(t), t, hashes=False)


def test_resumed_after_earlier_calls():
    """A context that already ran consensus: the split batch is laid out incrementally, its
    timestamps and the resumed rounds' coins come from the late payload."""
    n, E = 64, 150000
    t = gtrace.gossip(n, E, 4, stale_prob=0.2, stale_depth=3)
    a = _hg(n, E)
    a.insert_trace(t, 0, 40000)
    a.RunConsensus()
    assert a.insert_and_run(t, 40000, E) == E - 40000
    o = hgref.Oracle(n)
    o.insert_trace(t, 0, 40000)
    o.run_consensus()
    o.insert_trace(t, 40000, E)
    o.run_consensus()
    compare(a, o, t, hashes=False)


def test_insert_error_keeps_the_accepted_prefix():
    from babble_amd._lib import HgxError
    n, E, k0 = 32, 100000, 81234
    t = gtrace.gossip(n, E, 5)
    op = t.op.copy()
    op[k0] = -2   # HGX_UNKNOWN_PARENT
    bad = gtrace.GossipTrace(**{**t.__dict__, "op": op})
    a = _hg(n, E)
    with pytest.raises(HgxError) as ei:
        a.insert_and_run(bad)
    assert ei.value.msg == "CheckOtherParent: Other-parent not known" and ei.value.inserted == k0
    assert a.num_events() == k0
    a.RunConsensus()   # the prefix's payload is committed: consensus over it equals the two-call path
    b = _hg(n, E)
    b.insert_trace(t, 0, k0)
    b.RunConsensus()
    _same(a, b)


def test_batched_graphs():
    n, G, E1 = 16, 8, 12000
    t = gtrace.concat_graphs([gtrace.gossip(n, E1, 60 + g, stale_prob=0.1, stale_depth=2) for g in range(G)])
    a = _hg(n, t.E, graphs=G)
    assert a.insert_and_run(t) == t.E
    b = _hg(n, t.E, graphs=G)
    b.insert_trace(t)
    b.RunConsensus()
    _same(a, b, graphs=G)


# ---- the compact columns (hgx_events32: int32 Index / parents, the coin byte, ntx -1 = nil) ----

def _with_nil(t, every=7):
    """Some events with Body.Transactions == nil (the generator only makes empty non-nil ones)."""
    nil = t.txnil.copy()
    ntx = t.ntx.copy()
    k = np.arange(0, t.E, every)
    nil[k], ntx[k] = 1, 0
    return gtrace.GossipTrace(**{**t.__dict__, "txnil": nil, "ntx": ntx})


@pytest.mark.parametrize("n,E,seed", [(16, 70000, 11), (64, 120000, 12)])
def test_compact_columns_equal_wide(n, E, seed):
    from babble_amd.hashgraph import compact_columns
    t = _with_nil(gtrace.gossip(n, E, seed, stale_prob=0.1, stale_depth=3))
    a = _hg(n, E)
    assert a.insert_and_run32(compact_columns(t)) == E
    b = _hg(n, E)
    assert b.insert_and_run(t) == E
    _same(a, b)
    if n <= 16:
        compare(a, hgref.oracle_run(t), t, hashes=False)


def test_compact_chunked_and_small_batches():
    """Batches under 65 536 events (one packed pinned copy) through hgx_insert_events32, then
    RunConsensus per sync, equal the wide columns' path."""
    from babble_amd.hashgraph import compact_columns
    n, E, chunk = 32, 30000, 1000
    t = _with_nil(gtrace.gossip(n, E, 13, stale_prob=0.2, stale_depth=3), every=5)
    cols = compact_columns(t)
    a, b = _hg(n, E), _hg(n, E)
    for lo in range(0, E, chunk):
        hi = min(E, lo + chunk)
        assert a.insert_events32(cols, lo, hi) == hi - lo
        a.RunConsensus()
        b.insert_trace(t, lo, hi)
        b.RunConsensus()
    _same(a, b)


@pytest.mark.parametrize("kind", ["other_parent", "passed_index"])
def test_compact_insert_error(kind):
    from babble_amd._lib import HgxError
    from babble_amd.hashgraph import compact_columns
    n, E, k0 = 32, 100000, 81234
    t = gtrace.gossip(n, E, 14)
    cols = compact_columns(t)
    if kind == "other_parent":
        cols["op"][k0] = -2
        want = "CheckOtherParent: Other-parent not known"
    else:
        cols["index"][k0] = cols["index"][k0] - 1   # the self-parent's Index again
        want = None
    a = _hg(n, E)
    with pytest.raises(HgxError) as ei:
        a.insert_and_run32(cols)
    assert ei.value.inserted == k0 and a.num_events() == k0
    b = _hg(n, E)
    bad = {k: v.copy() for k, v in cols.items()}
    wide = gtrace.GossipTrace(**{**t.__dict__, "op": bad["op"].astype(np.int64), "index": bad["index"].astype(np.int64)})
    with pytest.raises(HgxError) as ew:
        b.insert_and_run(wide)
    assert ei.value.msg == ew.value.msg and ei.value.code == ew.value.code
    if want:
        assert ei.value.msg == want


def test_compact_batched_graphs():
    from babble_amd.hashgraph import compact_columns
    n, G, E1 = 16, 8, 12000
    t = gtrace.concat_graphs([gtrace.gossip(n, E1, 70 + g, stale_prob=0.1, stale_depth=2) for g in range(G)])
    a = _hg(n, t.E, graphs=G)
    assert a.insert_and_run32(compact_columns(t)) == t.E
    b = _hg(n, t.E, graphs=G)
    b.insert_and_run(t)
    _same(a, b, graphs=G)


def test_compact_refused_after_reset():
    from babble_amd._lib import HgxError
    from babble_amd.hashgraph import compact_columns
    n = 4
    t = gtrace.gossip(n, 100, 15)
    a = _hg(n, 1000)
    a.Reset([5] * n, [2] * n, [0] * n)
    with pytest.raises(HgxError) as ei:
        a.insert_events32(compact_columns(t))
    assert "use hgx_insert_events" in ei.value.msg


# ---- the packed structure columns (hgx_events_packed: 10 bytes per event, decoded on the device) ----

def _far_parents(cols, every=997, back=70000):
    """Valid other-parents more than 65 534 events back (CheckOtherParent only asks that the parent
    is known): the packed form carries them in its exception list."""
    op = cols["op"].copy()
    cr = cols["creator"]
    for k in range(back + 1, len(op), every):
        j = k - back
        while cr[j] == cr[k]:
            j -= 1
        op[k] = j
    return {**cols, "op": op}


@pytest.mark.parametrize("n,E,seed", [(16, 70000, 21), (64, 160000, 22), (256, 200000, 23)])
def test_packed_equal_compact(n, E, seed):
    from babble_amd.hashgraph import compact_columns, pack_columns
    cols = compact_columns(_with_nil(gtrace.gossip(n, E, seed, stale_prob=0.1, stale_depth=3)))
    if E > 70001:
        cols = _far_parents(cols)
    pk = pack_columns(cols, 0)
    assert (E <= 70001) or len(pk["exc_pos"]) > 0
    a = _hg(n, E)
    assert a.insert_and_run_packed(pk) == E
    b = _hg(n, E)
    assert b.insert_and_run32(cols) == E
    _same(a, b)
    if n <= 16:
        t = gtrace.gossip(n, E, seed, stale_prob=0.1, stale_depth=3)
        compare(a, hgref.oracle_run(_with_nil(t)), _with_nil(t), hashes=False)


def test_packed_small_batches_and_batched_graphs():
    """Sync-sized batches (hgx_insert_events_packed, base = the context's event count) and a
    batched context equal the compact columns' path."""
    from babble_amd.hashgraph import compact_columns, pack_columns
    n, E, chunk = 32, 30000, 1000
    cols = compact_columns(_with_nil(gtrace.gossip(n, E, 24, stale_prob=0.2, stale_depth=3), every=5))
    a, b = _hg(n, E), _hg(n, E)
    for lo in range(0, E, chunk):
        hi = min(E, lo + chunk)
        sub = {k: v[lo:hi] for k, v in cols.items()}
        assert a.insert_events_packed(pack_columns(sub, a.num_events())) == hi - lo
        a.RunConsensus()
        assert b.insert_events32(cols, lo, hi) == hi - lo
        b.RunConsensus()
    _same(a, b)
    G, E1 = 8, 12000
    t = gtrace.concat_graphs([gtrace.gossip(16, E1, 80 + g, stale_prob=0.1, stale_depth=2) for g in range(G)])
    cols = compact_columns(t)
    a, b = _hg(16, t.E, graphs=G), _hg(16, t.E, graphs=G)
    assert a.insert_and_run_packed(pack_columns(cols, 0)) == t.E
    b.insert_and_run32(cols)
    _same(a, b, graphs=G)


@pytest.mark.parametrize("kind", ["other_parent", "passed_index", "self_parent", "escape_without_entry"])
def test_packed_insert_error(kind):
    """The errors of the decoded batch are those of hgx_insert_and_run32 on the same batch."""
    from babble_amd._lib import HgxError
    from babble_amd.hashgraph import compact_columns, pack_columns
    n, E, k0 = 32, 100000, 81234
    cols = compact_columns(gtrace.gossip(n, E, 25))
    if kind == "other_parent":
        cols["op"][k0] = -2
    elif kind == "passed_index":
        cols["index"][k0] -= 1
    elif kind == "self_parent":
        cols["sp"][k0] = cols["sp"][k0] - 1 if cols["sp"][k0] > 0 else 0
    pk = pack_columns(cols, 0)
    if kind == "escape_without_entry":   # reads as HGX_UNKNOWN_PARENT
        pk["op_back"] = pk["op_back"].copy()
        pk["op_back"][k0] = 0xFFFF
        cols["op"][k0] = -2
    a = _hg(n, E)
    with pytest.raises(HgxError) as ei:
        a.insert_and_run_packed(pk)
    assert ei.value.inserted == k0 and a.num_events() == k0
    b = _hg(n, E)
    with pytest.raises(HgxError) as ec:
        b.insert_and_run32(cols)
    assert ei.value.msg == ec.value.msg and ei.value.code == ec.value.code and ec.value.inserted == k0


def test_packed_bad_exception_list():
    from babble_amd._lib import HgxError
    from babble_amd.hashgraph import compact_columns, pack_columns
    cols = compact_columns(gtrace.gossip(8, 2000, 26))
    pk = pack_columns(cols, 0)
    a = _hg(8, 4000)
    for pos in ([5, 5], [2000], [-1]):
        bad = {**pk, "exc_pos": np.asarray(pos, np.int64), "exc_sp": np.full(len(pos), -1, np.int32),
               "exc_op": np.full(len(pos), -1, np.int32)}
        with pytest.raises(HgxError) as ei:
            a.insert_events_packed(bad)
        assert "bad arguments" in ei.value.msg
    assert a.num_events() == 0
    assert a.insert_events_packed(pk) == 2000


@pytest.mark.parametrize("back", ["gid_plus_1", "far_before_0"])
def test_packed_distance_before_the_first_event(back):
    """A parent distance that reaches before gid 0 names no event: the decoded parent is
    HGX_UNKNOWN_PARENT (CheckOtherParent / CheckSelfParent fail, hashgraph.go:404-445), never gid -1
    (the empty parent) -- ADVICE r05. Same error and accepted prefix as the compact columns with -2."""
    from babble_amd._lib import HgxError
    from babble_amd.hashgraph import compact_columns, pack_columns
    n, E, k0 = 16, 3000, 700
    cols = compact_columns(gtrace.gossip(n, E, 27))
    pk = pack_columns(cols, 0)
    pk["op_back"] = pk["op_back"].copy()
    pk["op_back"][k0] = k0 + 1 if back == "gid_plus_1" else 0xFFFE
    cols["op"][k0] = -2
    a = _hg(n, E)
    with pytest.raises(HgxError) as ei:
        a.insert_and_run_packed(pk)
    b = _hg(n, E)
    with pytest.raises(HgxError) as ec:
        b.insert_and_run32(cols)
    assert ei.value.inserted == k0 == ec.value.inserted and a.num_events() == k0
    assert ei.value.msg == ec.value.msg and ei.value.code == ec.value.code
