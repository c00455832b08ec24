"""Bit-exact parity at the bench's own full workloads (BASELINE.json configs c2 and c4): the same
seeded traces bench.py times (bench.make_trace), handed over as it hands them (the packed host
columns, hgx_insert_and_run_packed), against the C oracle (oracle/, hashgraph.go's loops) on every
event -- not only the 100 k-event prefix the bench line checks, block hashes included. c3 (10 M events
at 256 peers) and c5 are pinned in full by the oracle's digests (test_gpu_full_digests.py): the
single-threaded oracle needs ~25 / ~40 min for them."""
import os
import sys

import numpy as np
import pytest

import hgref
from test_gpu_parity import compare

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _bench_trace(cfg):
    import bench
    return bench.make_trace(cfg, 0)


def test_c2_full_workload_bit_exact():
    from babble_amd.hashgraph import Hashgraph, compact_columns, pack_columns
    t, G = _bench_trace("c2")
    assert G == 1 and t.E == 1 << 20
    h = Hashgraph(64, capacity=t.E)
    assert h.insert_and_run_packed(pack_columns(compact_columns(t), 0)) == t.E
    compare(h, hgref.oracle_run(t), t, hashes=True)


def test_c4_full_workload_bit_exact():
    """All 512 independent 16-peer graphs of one GPU's c4 batch (8.4 M events)."""
    from babble_amd import trace as gtrace
    from babble_amd.hashgraph import Hashgraph, compact_columns, pack_columns
    import bench
    n, E1, G, silent, stale, depth, _ = bench.CONFIGS["c4"]
    t, G2 = _bench_trace("c4")
    assert G2 == G and t.E == G * E1
    h = Hashgraph(n, capacity=t.E, n_graphs=G)
    assert h.insert_and_run_packed(pack_columns(compact_columns(t), 0)) == t.E
    rnd, wit, fam = (np.asarray(x) for x in h.rounds())
    rr, cts = (np.asarray(x) for x in h.received())
    cts = np.where(rr >= 0, cts, 0)
    for g in range(G):
        o = hgref.oracle_run(gtrace.gossip(n, E1, 1 + g, n_silent=silent, stale_prob=stale,
                                           stale_depth=depth)).results()
        sl = slice(g * E1, (g + 1) * E1)
        for k, v in (("round", rnd), ("witness", wit), ("famous", fam), ("rr", rr), ("cts", cts)):
            assert np.array_equal(v[sl], np.asarray(o[k])), (g, k)
        assert list(np.asarray(h.ConsensusEvents(g)) - g * E1) == list(o["order"]), g
        assert h.UndecidedRounds(g) == o["undecided"] and h.LastConsensusRound(g) == o["lcr"], g
        assert h.ConsensusTransactions(g) == o["consensus_tx"], g
        assert [(b["rr"], b["ntx"], b["tx_nil"]) for b in h.Blocks(g)] == [(b[0], b[1], b[2]) for b in o["blocks"]], g
