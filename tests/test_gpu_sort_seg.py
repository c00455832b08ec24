"""FindOrder's segmented sort (hgx_kernels.hip k_seg_count / k_seg_scatter / k_seg_sort: the received
events bucketed by (graph, roundReceived), every bucket sorted in LDS) against the LSD radix sort and the
oracle (consensus_sorter.go:5-52, hashgraph.go:822-823).

Every test asserts which sort ran (phase_times sort_seg), so a silent fallback to the radix passes
cannot pass for the segmented one."""
import numpy as np
import pytest

import hgref
from babble_amd import trace as gtrace

pytestmark = pytest.mark.gpu


def _run(t, sort="auto", graphs=1, chunk=None, n=None):
    from babble_amd.hashgraph import Hashgraph
    h = Hashgraph(n or t.n, capacity=max(64, t.E), n_graphs=graphs)
    h.set_sort_kernel(sort)
    if chunk is None:
        h.insert_trace(t)
        h.RunConsensus()
    else:
        for lo in range(0, t.E, chunk):
            h.insert_trace(t, lo, min(t.E, lo + chunk))
            h.RunConsensus()
    return h


def _same(a, b):
    ra, rb = a.results(), b.results()
    for k in ("round", "witness", "famous", "rr", "cts"):
        assert np.array_equal(np.asarray(ra[k]), np.asarray(rb[k])), k
    assert list(ra["order"]) == list(rb["order"]), "consensus order"


@pytest.mark.parametrize("n,E,seed,stale", [(16, 20000, 201, 0.0), (64, 60000, 202, 0.2), (256, 60000, 203, 0.0)])
def test_seg_sort_matches_radix_and_oracle(n, E, seed, stale):
    t = gtrace.gossip(n, E, seed, stale_prob=stale, stale_depth=3)
    hs, hr = _run(t), _run(t, "radix")
    assert hs.phase_times()["sort_seg"] >= 1, "the segmented sort did not run"
    assert hr.phase_times()["sort_seg"] == 0
    _same(hs, hr)
    o = hgref.oracle_run(t).results()
    assert list(hs.results()["order"]) == list(o["order"])


def test_seg_sort_many_graphs():
    """c4's shape: many independent graphs in one context, a bucket per (graph, roundReceived)."""
    n, G = 16, 32
    traces = [gtrace.gossip(n, 6000 + 100 * g, 210 + g, stale_prob=0.1 * (g % 3), stale_depth=3) for g in range(G)]
    t = gtrace.concat_graphs(traces)
    hs, hr = _run(t, graphs=G, n=n), _run(t, "radix", graphs=G, n=n)
    assert hs.phase_times()["sort_seg"] >= 1
    _same(hs, hr)
    off = 0
    for g, tg in enumerate(traces[:4]):
        o = hgref.oracle_run(tg).results()
        assert list(hs.ConsensusEvents(g) - off) == list(o["order"]), g
        off += tg.E


def test_seg_sort_equal_timestamps():
    """Runs of equal consensus timestamps inside a bucket: ordered by S afterwards (k_tiefix_rank), as
    after the radix sort."""
    t = gtrace.gossip(32, 30000, 221, stale_prob=0.0, stale_depth=1)
    t.ts[:] = 1_600_000_000_000_000_000 + 1000 * (np.arange(t.E, dtype=np.int64) // 64)   # 64 events per tick
    hs, hr = _run(t), _run(t, "radix")
    assert hs.phase_times()["sort_seg"] >= 1
    _same(hs, hr)
    assert list(hs.results()["order"]) == list(hgref.oracle_run(t).results()["order"])


def test_seg_sort_chunked_calls():
    """The chunked schedule: calls whose received list is over the small sort's size use the buckets."""
    t = gtrace.gossip(64, 40000, 231, stale_prob=0.1, stale_depth=2)
    hs, hr = _run(t, chunk=10000), _run(t, "radix", chunk=10000)
    assert hs.phase_times()["sort_seg"] >= 1
    _same(hs, hr)
