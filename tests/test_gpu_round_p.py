"""The persistent round recurrence (hgx_round_p.hip: one resident workgroup per chain runs
every round of a DivideRounds in one launch, candidates handed over by write-through
granules) against the CPU oracle and against the per-launch round step.

Every test asserts that the persistent launch actually ran (phase_times round_p_runs) and
never gave up (round_p_fallbacks), so a silent fallback to the per-launch kernel cannot pass
for it."""
import numpy as np
import pytest

import hgref
from babble_amd import trace as gtrace
from babble_amd.trace import GossipTrace

pytestmark = pytest.mark.gpu


def _run(t, mode="persistent", chunk=None, coord32=False, graphs=1, reserve=None):
    from babble_amd.hashgraph import Hashgraph
    h = Hashgraph(t.n // graphs if graphs > 1 else t.n, capacity=max(64, t.E), n_graphs=graphs)
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


def _check_persistent(h):
    ph = h.phase_times()
    assert ph["round_p_runs"] > 0, "the persistent round launch did not run"
    assert ph["round_p_fallbacks"] == 0, "the persistent round launch gave up"
    return ph


def _compare(h, o):
    a, b = h.results(), o.results()
    for k in ("round", "witness", "famous", "rr", "cts"):
        if not np.array_equal(np.asarray(a[k]), np.asarray(b[k])):
            bad = np.nonzero(np.asarray(a[k]) != np.asarray(b[k]))[0][:10]
            raise AssertionError(f"{k} differs at gids {bad.tolist()}")
    assert list(a["order"]) == list(b["order"]), "consensus order"
    for k in ("last_round", "undecided", "lcr", "lcre", "consensus_tx", "pending_loaded"):
        assert a[k] == b[k], k


CASES = [(1, 64, 1, 0, 0.0), (2, 300, 2, 0, 0.0), (4, 2000, 3, 0, 0.0), (5, 1500, 4, 1, 0.3),
         (8, 4000, 5, 0, 0.2), (13, 5000, 6, 3, 0.0), (16, 6000, 7, 5, 0.5), (32, 8000, 8, 0, 0.0),
         (48, 10000, 9, 10, 0.3), (64, 16000, 10, 21, 0.2), (100, 15000, 11, 0, 0.0),
         (128, 20000, 12, 0, 0.0), (200, 20000, 13, 60, 0.0), (256, 40000, 14, 0, 0.0),
         (256, 30000, 15, 85, 0.3)]


@pytest.mark.parametrize("n,E,seed,silent,stale", CASES)
def test_persistent_batch_matches_oracle(n, E, seed, silent, stale):
    t = gtrace.gossip(n, E, seed, n_silent=silent, stale_prob=stale, stale_depth=4)
    h = _run(t)
    _check_persistent(h)
    _compare(h, hgref.oracle_run(t))


@pytest.mark.parametrize("n,E,seed", [(16, 6000, 21), (64, 16000, 22), (256, 30000, 23)])
def test_persistent_equals_per_launch_steps(n, E, seed):
    """Round, witness and the strongly-see rows feeding fame: identical to k_round_k."""
    t = gtrace.gossip(n, E, seed, stale_prob=0.2, stale_depth=3)
    hp, hk = _run(t), _run(t, mode="candidate")
    _check_persistent(hp)
    assert hk.phase_times()["round_p_runs"] == 0
    a, b = hp.results(), hk.results()
    for k in ("round", "witness", "famous", "rr", "cts"):
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k
    assert list(a["order"]) == list(b["order"])


@pytest.mark.parametrize("n,E,seed", [(16, 5000, 31), (64, 12000, 32), (256, 30000, 33)])
def test_persistent_int32_coordinates(n, E, seed):
    t = gtrace.gossip(n, E, seed, stale_prob=0.2, stale_depth=3)
    h = _run(t, coord32=True)
    _check_persistent(h)
    _compare(h, hgref.oracle_run(t))


@pytest.mark.parametrize("n,E,seed,chunk", [(8, 3000, 41, 100), (64, 12000, 42, 1000), (256, 30000, 43, 1000)])
def test_persistent_chunked_schedule(n, E, seed, chunk):
    """Core's schedule: consensus after every sync; each call resumes at the lowest round
    that can change (one persistent launch per call)."""
    t = gtrace.gossip(n, E, seed, stale_prob=0.1, stale_depth=2)
    h = _run(t, chunk=chunk)
    ph = _check_persistent(h)
    assert ph["round_p_runs"] >= (E + chunk - 1) // chunk
    _compare(h, hgref.oracle_run(t, chunk))


def test_auto_schedule_persistent_on_rebuild_only():
    """The default: the persistent launch on the call that lays the DAG out, per-round steps on
    the calls that resume after a sync's inserts; bit-exact either way."""
    t = gtrace.gossip(64, 12000, 44, stale_prob=0.1, stale_depth=2)
    h = _run(t, mode="auto", chunk=3000)
    ph = h.phase_times()
    assert ph["round_p_runs"] == 1 and ph["round_p_fallbacks"] == 0
    _compare(h, hgref.oracle_run(t, 3000))


@pytest.mark.parametrize("n,E,seed", [(8, 6000, 51), (16, 20000, 52)])
def test_persistent_round_capacity_relaunch(n, E, seed):
    """Round tables reserved for one round: the launch stops at the capacity, the host grows
    the tables and relaunches from the round it stopped at."""
    t = gtrace.gossip(n, E, seed, stale_prob=0.2, stale_depth=3)
    h = _run(t, reserve=1)
    ph = _check_persistent(h)
    assert ph["round_p_runs"] >= 2
    _compare(h, hgref.oracle_run(t))


def test_persistent_batched_graphs():
    """Several graphs in one context (C = G n <= CUs): each graph's workgroups wait only for
    their own graph's granules and stop at their own last round."""
    n, G = 16, 8
    traces = [gtrace.gossip(n, 3000 + 500 * g, 60 + g, stale_prob=0.1 * (g % 3), stale_depth=3) for g in range(G)]
    t = gtrace.concat_graphs(traces)
    from babble_amd.hashgraph import Hashgraph
    h = Hashgraph(n, capacity=t.E, n_graphs=G)
    h.set_round_kernel("persistent")   # (the default runs n <= 16 by the whole-graph kernel)
    h.insert_trace(t)
    h.RunConsensus()
    _check_persistent(h)
    a = h.results()
    off = 0
    for g, tg in enumerate(traces):
        o = hgref.oracle_run(tg).results()
        sl = slice(off, off + tg.E)
        for k in ("round", "witness", "famous", "rr", "cts"):
            assert np.array_equal(np.asarray(a[k])[sl], np.asarray(o[k])), (g, k)
        assert list(h.ConsensusEvents(g) - off) == list(o["order"]), g
        assert h.UndecidedRounds(g) == o["undecided"] and h.LastConsensusRound(g) == o["lcr"], g
        assert h.LastRound(g) == o["last_round"], g
        off += tg.E


def bursty(n, E, seed, burst_peer=0, burst_len=160, every=600):
    """Gossip (node/core_test.go model) where one peer now and then creates a run of events
    without an other-parent (op ""): its chain runs far ahead of what it sees, so the other
    candidates' first descendants on that chain lie more than 125 events past the round's
    base and their rows do not fit the 8-bit rebasing (the exact-compare path)."""
    rng = np.random.default_rng(seed)
    creator, index, sp, op = [], [], [], []
    head = [-1] * n
    hidx = [-1] * n

    def emit(to, o):
        g = len(creator)
        creator.append(to)
        index.append(hidx[to] + 1)
        sp.append(head[to])
        op.append(o)
        head[to] = g
        hidx[to] += 1

    for p in range(n):
        emit(p, -1)
    step = 0
    while len(creator) < E:
        step += 1
        if step % every == 0:
            for _ in range(burst_len):
                if len(creator) >= E:
                    break
                emit(burst_peer, -1)
            continue
        to = int(rng.integers(n))
        fr = int(rng.integers(n - 1))
        fr += fr >= to
        emit(to, head[fr])
    E = len(creator)
    S = rng.integers(0, 256, (E, 32), dtype=np.uint8)
    S[:, :8] = np.arange(E, dtype=">u8").view(np.uint8).reshape(E, 8)   # unique
    return GossipTrace(n=n, creator=np.array(creator, np.int32), index=np.array(index, np.int64),
                       sp=np.array(sp, np.int64), op=np.array(op, np.int64),
                       ts=1_600_000_000_000_000_000 + 1000 * np.arange(E, dtype=np.int64),
                       hash=rng.integers(0, 256, (E, 32), dtype=np.uint8), s=S,
                       ntx=np.zeros(E, np.int32), txnil=np.zeros(E, np.int32), tx_seq=np.full(E, -1, np.int64))


@pytest.mark.parametrize("n,E,seed,coord32", [(8, 6000, 71, False), (16, 9000, 72, False), (64, 20000, 73, False),
                                              (16, 9000, 74, True)])
def test_persistent_exact_rows(n, E, seed, coord32):
    """Candidate rows over 8 bits are counted with exact compares, one candidate at a time."""
    t = bursty(n, E, seed)
    h = _run(t, coord32=coord32)
    ph = _check_persistent(h)
    assert ph["round_p_ovf"] > 0, "the trace did not exercise the exact-compare path"
    _compare(h, hgref.oracle_run(t))
