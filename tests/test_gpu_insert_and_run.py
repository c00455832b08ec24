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
