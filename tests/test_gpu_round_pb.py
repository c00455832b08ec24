"""The big-n persistent round recurrence (hgx_round_pb.hip: 256 < n <= 1024, one resident
workgroup per chain WITH events runs every round of a DivideRounds in one launch) against the CPU
oracle and against the per-launch round steps it replaces ("auto-steps").

Every test asserts that the persistent launch actually ran (phase_times round_p_runs) and never
gave up (round_p_fallbacks), so a silent fallback to the steps cannot pass for it."""
import numpy as np
import pytest

import hgref
from babble_amd import trace as gtrace

from test_gpu_round_p import _compare, _run, bursty

pytestmark = pytest.mark.gpu


def _check_pb(h):
    ph = h.phase_times()
    assert ph["round_p_runs"] > 0, "the persistent round launch did not run"
    assert ph["round_p_fallbacks"] == 0, "the persistent round launch gave up"
    return ph


# (n, E, seed, silent, stale): at most 768 chains with events (3 resident workgroups per CU); the
# oracle's cost grows as n E (~1.5 s per million at n = 1 024), so the long runs of rounds at large
# n are checked against the steps (below) and against the oracle's digests of the c5 prefix
CASES = [(258, 12000, 101, 0, 0.0), (300, 15000, 102, 20, 0.3), (384, 16000, 103, 0, 0.2),
         (512, 16000, 104, 0, 0.0), (514, 14000, 105, 100, 0.3), (700, 12000, 106, 0, 0.2),
         (1000, 9000, 107, 300, 0.3), (1024, 9000, 108, 341, 0.3)]


@pytest.mark.parametrize("n,E,seed,silent,stale", CASES)
def test_pb_matches_oracle(n, E, seed, silent, stale):
    t = gtrace.gossip(n, E, seed, n_silent=silent, stale_prob=stale, stale_depth=4)
    h = _run(t, mode="auto")
    _check_pb(h)
    _compare(h, hgref.oracle_run(t))


@pytest.mark.parametrize("n,E,seed,spread", [(600, 12000, 151, "random"), (520, 12000, 152, "every7"),
                                              (1024, 9000, 153, "every3")])
def test_pb_silent_chains_between_active_ones(n, E, seed, spread):
    """Silent peers spread over the chain order instead of a tail: the coordinate slots (the chains with
    events) are then not one run of consecutive chains, so a window row's 16-byte slot groups fall back
    to one gather per slot (every group for a random order, some groups for a regular spread). The
    trace's creators are relabelled; the hashgraph is the same up to that relabelling."""
    silent = n // 4 if spread == "random" else (n + 6) // 7 if spread == "every7" else (n + 2) // 3
    t = gtrace.gossip(n, E, seed, n_silent=silent, stale_prob=0.2, stale_depth=3)
    if spread == "random":
        perm = np.random.default_rng(seed).permutation(n)
    else:
        step = 7 if spread == "every7" else 3
        sil = [c for c in range(n) if c % step == 0][:silent]
        act = [c for c in range(n) if c not in set(sil)]
        perm = np.array(act + sil)   # active creator a -> chain act[a], silent ones -> every step-th chain
    t.creator = perm[t.creator].astype(np.int32)
    h = _run(t, mode="auto")
    _check_pb(h)
    _compare(h, hgref.oracle_run(t))


@pytest.mark.parametrize("n,E,seed,silent", [(300, 60000, 111, 0), (600, 100000, 112, 0), (1024, 200000, 113, 341)])
def test_pb_equals_per_launch_steps(n, E, seed, silent):
    """Round, witness and the strongly-see rows feeding fame: identical to the k_round_k steps."""
    t = gtrace.gossip(n, E, seed, n_silent=silent, stale_prob=0.2, stale_depth=3)
    hp, hk = _run(t, mode="auto"), _run(t, mode="auto-steps")
    _check_pb(hp)
    assert hk.phase_times()["round_p_runs"] == 0
    a, b = hp.results(), hk.results()
    for k in ("round", "witness", "famous", "rr", "cts"):
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k
    assert list(a["order"]) == list(b["order"])


@pytest.mark.parametrize("n,E,seed", [(300, 12000, 121), (767, 10000, 122)])
def test_pb_int32_coordinates(n, E, seed):
    t = gtrace.gossip(n, E, seed, stale_prob=0.2, stale_depth=3)
    h = _run(t, mode="auto", coord32=True)
    _check_pb(h)
    _compare(h, hgref.oracle_run(t))


def test_pb_chunked_schedule():
    """One persistent launch per call ("persistent" mode), each resuming at the lowest round that
    can change."""
    n, E, chunk = 512, 16000, 4000
    t = gtrace.gossip(n, E, 131, n_silent=40, stale_prob=0.1, stale_depth=2)
    h = _run(t, mode="persistent", chunk=chunk)
    ph = _check_pb(h)
    assert ph["round_p_runs"] >= E // chunk
    _compare(h, hgref.oracle_run(t, chunk))


def test_pb_round_capacity_relaunch():
    """More rounds than the tables hold at first (64): the launch stops at the capacity, the host grows
    the tables and relaunches from the round it stopped at (the silent chains' rows filled after).
    Against the steps (the oracle would take minutes at this size)."""
    t = gtrace.gossip(300, 300000, 141, n_silent=30, stale_prob=0.2, stale_depth=3)
    h, hk = _run(t, mode="auto", reserve=1), _run(t, mode="auto-steps")
    ph = _check_pb(h)
    assert ph["round_p_runs"] >= 2 and h.results()["last_round"] > 64
    a, b = h.results(), hk.results()
    for k in ("round", "witness", "famous", "rr", "cts"):
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k
    assert list(a["order"]) == list(b["order"])


def test_pb_exact_rows():
    """Candidate rows over 8 bits (a peer's run of events without other-parents) are counted with
    exact compares."""
    t = bursty(300, 20000, 151, burst_len=200, every=900)
    h = _run(t, mode="auto")
    ph = _check_pb(h)
    assert ph["round_p_ovf"] > 0, "the trace did not exercise the exact-compare path"
    _compare(h, hgref.oracle_run(t))


def test_pb_too_many_chains_falls_back():
    """More chains with events than resident workgroups fit: the steps run instead, same results."""
    t = gtrace.gossip(1024, 100000, 161, stale_prob=0.1, stale_depth=2)
    h, hk = _run(t, mode="auto"), _run(t, mode="auto-steps")
    ph = h.phase_times()
    assert ph["round_p_runs"] == 0 and ph["round_p_fallbacks"] == 1
    a, b = h.results(), hk.results()
    for k in ("round", "witness", "famous", "rr", "cts"):
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k


def test_pb_c5_prefix_golden():
    """bench.py's c5 workload (1 024 peers, 341 silent, 30% stale), its first E events: every output
    equals the oracle's (SHA-256 digests, tests/golden/make_c5_prefix.py)."""
    import json
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import make_c5_prefix as mk
    doc = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "c5_prefix.json")))
    t = gtrace.gossip(doc["n"], doc["E"], doc["seed"], n_silent=doc["silent"], stale_prob=doc["stale"],
                      stale_depth=doc["depth"])
    h = _run(t, mode="auto")
    _check_pb(h)
    got = mk.summarize(h.results())
    for k, v in doc["digests"].items():
        assert got[k] == v, k
