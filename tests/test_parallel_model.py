"""The data-parallel formulation (tests/parallel_model.py, mirrored by the HIP kernels)
equals the reference restatement (oracle) on fixtures and seeded gossip traces, in
batch and chunked schedules. CPU only; validates the math independent of the kernels."""
import numpy as np
import pytest

import hgref
from parallel_model import model_run
from babble_amd import trace as gtrace


def _compare(m, o):
    r = o.results()
    E = m.E
    assert np.array_equal(m.round, r["round"]), "round"
    assert np.array_equal(m.witness.astype(np.int8), r["witness"]), "witness"
    fam = np.zeros(E, np.int8)
    for (i, c), v in m.fame.items():
        fam[m.W[i][c]] = v
    assert np.array_equal(fam, r["famous"]), "famous"
    assert np.array_equal(m.rr, r["rr"]), "round received"
    assert np.array_equal(np.where(m.rr >= 0, m.cts, 0), r["cts"]), "consensus ts"
    assert list(m.consensus) == list(r["order"]), "order"
    assert m.undecided == r["undecided"], "UndecidedRounds"
    assert m.lcr == r["lcr"] and m.lcre == r["lcre"]
    assert m.consensus_tx == r["consensus_tx"] and m.pending_loaded == r["pending_loaded"]
    assert [(b["rr"], b["ntx"], b["nil"]) for b in m.blocks] == [(b[0], b[1], b[2]) for b in r["blocks"]]


@pytest.mark.parametrize("name", ["round_hashgraph", "consensus_hashgraph", "funky_hashgraph"])
def test_model_fixtures(name):
    t = hgref.fixture_trace(name)
    _compare(model_run(t), hgref.oracle_run(t))


@pytest.mark.parametrize("n,E,seed,silent,stale", [
    (4, 600, 1, 0, 0.0), (4, 600, 2, 0, 0.0), (5, 500, 3, 1, 0.0), (7, 700, 4, 2, 0.3),
    (16, 1500, 5, 0, 0.0), (16, 1500, 6, 5, 0.5), (2, 200, 7, 0, 0.0), (3, 300, 8, 0, 0.2),
    (1, 50, 9, 0, 0.0), (32, 2000, 10, 10, 0.0)])
def test_model_gossip_batch(n, E, seed, silent, stale):
    t = gtrace.gossip(n, E, seed, n_silent=silent, stale_prob=stale, stale_depth=4)
    _compare(model_run(t), hgref.oracle_run(t))


@pytest.mark.parametrize("n,E,seed,chunk,stale", [
    (4, 500, 11, 64, 0.0), (4, 500, 12, 7, 0.0), (5, 400, 13, 13, 0.4), (8, 600, 14, 50, 0.0),
    (3, 300, 15, 1, 0.0)])
def test_model_gossip_chunked(n, E, seed, chunk, stale):
    t = gtrace.gossip(n, E, seed, stale_prob=stale, stale_depth=3)
    _compare(model_run(t, chunk=chunk), hgref.oracle_run(t, chunk=chunk))
