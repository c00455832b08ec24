"""Parity at the headline configuration's shape and on the paths small traces never reach.

* C3-shaped: 256 peers, 200k events (chains ~780 long, 57 rounds), compact uint16
  coordinates, the n <= 256 round step, k_cts_tile at n = 256 -- every output against the
  oracle (the oracle needs ~1 min here; bench.py adds the full-size property checks).
* Timestamps so far apart that the (graph, rr, cts - min) sort key needs more than 64 bits
  (two-pass sort, hgx_engine.cpp find_order) and the consensus-timestamp offsets overflow
  32 bits (k_cts_tile's 64-bit reselect), alone and mixed with ordinary events.
"""
import numpy as np
import pytest

import hgref
from babble_amd import trace as gtrace

pytestmark = pytest.mark.gpu


def _run(t, cap=None):
    from babble_amd.hashgraph import Hashgraph
    h = Hashgraph(t.n, capacity=cap or t.E)
    h.insert_trace(t)
    h.RunConsensus()
    return h


def _compare(h, o):
    a, b = h.results(), o.results()
    for k in ("round", "witness", "famous", "rr", "cts"):
        if not np.array_equal(np.asarray(a[k]), np.asarray(b[k])):
            bad = np.nonzero(np.asarray(a[k]) != np.asarray(b[k]))[0][:10]
            raise AssertionError(f"{k} differs at gids {bad.tolist()}")
    assert list(a["order"]) == list(b["order"]), "consensus order"
    for k in ("last_round", "undecided", "lcr", "lcre", "consensus_tx", "pending_loaded"):
        assert a[k] == b[k], k
    assert [(x["rr"], x["ntx"], x["tx_nil"]) for x in a["blocks"]] == [(x[0], x[1], x[2]) for x in b["blocks"]]
    return b


def test_c3_shaped_long_chains():
    t = gtrace.gossip(256, 200_000, 1)
    h = _run(t)
    assert h.phase_times()["compact"] == 1
    b = _compare(h, hgref.oracle_run(t))
    assert b["last_round"] >= 50 and len(b["order"]) > 150_000


def _wide(t, step_log2, every=1):
    ts = t.ts.copy()
    g = np.arange(t.E, dtype=np.int64)
    sel = (g % every) == 0
    ts[sel] = ts[sel] + (g[sel] << np.int64(step_log2))
    t.ts = ts
    return t


@pytest.mark.parametrize("n,E,seed,step,every", [
    (64, 12000, 201, 46, 1),    # ~60-bit cts range: key > 64 bits, every offset > 32 bits
    (64, 12000, 202, 40, 97),   # mixed: a few far-future events among ordinary ones
    (16, 4000, 203, 46, 1),     # n <= 32 (k_cts_small) with the two-pass sort
    (256, 20000, 204, 44, 3)])  # n = 256 tile path
def test_wide_timestamps(n, E, seed, step, every):
    t = _wide(gtrace.gossip(n, E, seed, stale_prob=0.1, stale_depth=3), step, every)
    h = _run(t)
    b = _compare(h, hgref.oracle_run(t))
    rr = np.asarray(b["rr"])
    cts = np.asarray(b["cts"])[rr >= 0]
    span = int(cts.max()) - int(cts.min()) if cts.size else 0
    assert len(b["order"]) > 0
    if every == 1:
        assert span.bit_length() + int(rr.max()).bit_length() > 64 or span.bit_length() > 56
