"""The whole-graph round recurrence (hgx_round_g.hip: one workgroup per graph of n <= 16 chains
runs every round of a DivideRounds in one launch, chains exchange their candidates through LDS)
against the CPU oracle and against the per-launch round step.

Every test asserts that the whole-graph launch actually ran (phase_times round_g_runs), so a
silent fallback to another round kernel cannot pass for it."""
import numpy as np
import pytest

import hgref
from babble_amd import trace as gtrace
from test_gpu_round_p import _compare, bursty

pytestmark = pytest.mark.gpu


def _run(t, mode="graph", chunk=None, coord32=False, reserve=None):
    from babble_amd.hashgraph import Hashgraph
    h = Hashgraph(t.n, capacity=max(64, t.E))
    if coord32:
        h.set_coord_storage(1)
    h.set_round_kernel(mode)
    if reserve:
        h.reserve_rounds(reserve)
    if chunk is None:
        h.insert_trace(t)
        h.RunConsensus()
    else:
        for lo in range(0, t.E, chunk):
            h.insert_trace(t, lo, min(t.E, lo + chunk))
            h.RunConsensus()
    return h


def _check_graph(h, runs=1):
    ph = h.phase_times()
    assert ph["round_g_runs"] >= runs, "the whole-graph round launch did not run"
    assert ph["round_p_runs"] == 0
    return ph


CASES = [(1, 64, 1, 0, 0.0), (2, 300, 2, 0, 0.0), (3, 900, 3, 0, 0.1), (4, 2000, 3, 0, 0.0),
         (4, 1024, 9, 0, 0.0), (5, 1500, 4, 1, 0.3), (6, 3000, 10, 0, 0.2), (8, 4000, 5, 0, 0.2),
         (11, 4000, 11, 2, 0.1), (12, 6000, 12, 0, 0.0), (13, 5000, 6, 3, 0.0), (16, 6000, 7, 5, 0.5),
         (16, 16384, 8, 0, 0.0), (16, 30000, 13, 0, 0.3)]


@pytest.mark.parametrize("n,E,seed,silent,stale", CASES)
def test_graph_batch_matches_oracle(n, E, seed, silent, stale):
    t = gtrace.gossip(n, E, seed, n_silent=silent, stale_prob=stale, stale_depth=4)
    h = _run(t)
    _check_graph(h)
    _compare(h, hgref.oracle_run(t))


@pytest.mark.parametrize("n,E,seed", [(4, 3000, 21), (16, 12000, 22)])
def test_graph_equals_per_launch_steps(n, E, seed):
    """Round, witness and the strongly-see rows feeding fame: identical to k_round_k."""
    t = gtrace.gossip(n, E, seed, stale_prob=0.2, stale_depth=3)
    hg, hk = _run(t), _run(t, mode="candidate")
    _check_graph(hg)
    assert hk.phase_times()["round_g_runs"] == 0
    a, b = hg.results(), hk.results()
    for k in ("round", "witness", "famous", "rr", "cts"):
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k
    assert list(a["order"]) == list(b["order"])


@pytest.mark.parametrize("n,E,seed", [(5, 3000, 31), (16, 8000, 32)])
def test_graph_int32_coordinates(n, E, seed):
    t = gtrace.gossip(n, E, seed, stale_prob=0.2, stale_depth=3)
    h = _run(t, coord32=True)
    _check_graph(h)
    _compare(h, hgref.oracle_run(t))


@pytest.mark.parametrize("n,E,seed,chunk", [(4, 1024, 41, 64), (8, 3000, 42, 100), (16, 12000, 43, 1000)])
def test_graph_chunked_schedule(n, E, seed, chunk):
    """Core's schedule: consensus after every sync; each call resumes at the lowest round that
    can change (one whole-graph launch per call, the default for n <= 16)."""
    t = gtrace.gossip(n, E, seed, stale_prob=0.1, stale_depth=2)
    h = _run(t, mode="auto", chunk=chunk)
    _check_graph(h, (E + chunk - 1) // chunk)
    _compare(h, hgref.oracle_run(t, chunk))


@pytest.mark.parametrize("n,E,seed", [(4, 6000, 51), (16, 20000, 52)])
def test_graph_round_capacity_relaunch(n, E, seed):
    """Round tables reserved for one round: the launch stops at the capacity, the host grows the
    tables and relaunches from the round it stopped at (the state rebuilt from Bm)."""
    t = gtrace.gossip(n, E, seed, stale_prob=0.2, stale_depth=3)
    h = _run(t, reserve=1)
    _check_graph(h, 2)
    _compare(h, hgref.oracle_run(t))


def test_graph_batched_graphs():
    """Many graphs in one context (one workgroup each, more graphs than CUs allowed)."""
    n, G = 16, 300
    traces = [gtrace.gossip(n, 600 + 7 * g, 600 + g, stale_prob=0.1 * (g % 3), stale_depth=3) for g in range(G)]
    t = gtrace.concat_graphs(traces)
    from babble_amd.hashgraph import Hashgraph
    h = Hashgraph(n, capacity=t.E, n_graphs=G)
    h.insert_trace(t)
    h.RunConsensus()
    _check_graph(h)
    a = h.results()
    off = 0
    for g, tg in enumerate(traces):
        if g % 37 == 0 or g == G - 1:
            o = hgref.oracle_run(tg).results()
            sl = slice(off, off + tg.E)
            for k in ("round", "witness", "famous", "rr", "cts"):
                assert np.array_equal(np.asarray(a[k])[sl], np.asarray(o[k])), (g, k)
            assert list(h.ConsensusEvents(g) - off) == list(o["order"]), g
            assert h.LastRound(g) == o["last_round"], g
        off += tg.E


@pytest.mark.parametrize("n,E,seed,coord32", [(8, 6000, 71, False), (16, 9000, 72, False), (16, 9000, 74, True)])
def test_graph_bursty_chains(n, E, seed, coord32):
    """A chain that runs far ahead of what it sees (the trace that drives the other kernels'
    over-8-bit rows): raw compares need no fallback; the burst also pushes windows past the staged
    ring (synchronous staging, later windows)."""
    t = bursty(n, E, seed)
    h = _run(t, coord32=coord32)
    _check_graph(h)
    _compare(h, hgref.oracle_run(t))
