"""The dataflow lastAncestors pass (k_la_wave, hgx_la_wave.hip) against the Gauss-Seidel
sweeps (k_la_sweep) and the oracle: identical coordinates on sampled events and identical
consensus on the whole DAG, for both coordinate storages, batched graphs, odd n, n > 256
(4-byte column blocks), n > 896 (lanes for the chains with events only) and incremental calls
(rows of earlier calls read from HBM)."""
import numpy as np
import pytest

import hgref
from babble_amd import trace as gtrace

pytestmark = pytest.mark.gpu


def _run(t, la, coord32=False, graphs=1, chunk=None):
    from babble_amd.hashgraph import Hashgraph
    h = Hashgraph(t.n, capacity=max(64, t.E), n_graphs=graphs)
    h.set_la_kernel(la)
    if coord32:
        h.set_coord_storage(1)
    if chunk is None:
        h.insert_trace(t)
        h.RunConsensus()
    else:
        for lo in range(0, t.E, chunk):
            h.insert_trace(t, lo, min(t.E, lo + chunk))
            h.RunConsensus()
    return h


def _same_coords(h1, h2, E, seed, k=400):
    rng = np.random.default_rng(seed)
    for x in sorted(set(rng.integers(0, E, size=min(k, E)).tolist()) | {0, E - 1}):
        la1, fd1 = h1.coords(int(x))
        la2, fd2 = h2.coords(int(x))
        assert np.array_equal(la1, la2), f"lastAncestors of gid {x}"
        assert np.array_equal(fd1, fd2), f"firstDescendants of gid {x}"


def _same_results(h1, h2, graph=0):
    a, b = h1.results(graph), h2.results(graph)
    for key in ("round", "witness", "famous", "rr", "cts", "order"):
        assert np.array_equal(np.asarray(a[key]), np.asarray(b[key])), key


CASES = [(4, 1024, 1, 0, 0.0), (5, 800, 4, 1, 0.0), (16, 4000, 7, 5, 0.5), (64, 12000, 10, 21, 0.2),
         (100, 15000, 11, 0, 0.0), (256, 30000, 16, 0, 0.0), (300, 24000, 17, 0, 0.0), (512, 24000, 18, 100, 0.2),
         (896, 14000, 20, 0, 0.0),
         # n > 896: lanes only for the chains with events (silent peers have none)
         (1024, 16000, 19, 300, 0.0), (1000, 20000, 22, 330, 0.3)]


@pytest.mark.parametrize("n,E,seed,silent,stale", CASES)
def test_wave_matches_sweeps_and_oracle(n, E, seed, silent, stale):
    t = gtrace.gossip(n, E, seed, n_silent=silent, stale_prob=stale, stale_depth=4)
    hw = _run(t, "wave")
    pt = hw.phase_times()
    assert pt["la_wave"] == 1 and pt["la_wave_fallbacks"] == 0, pt
    hs = _run(t, "sweep")
    assert hs.phase_times()["la_wave"] == 0
    _same_coords(hw, hs, t.E, seed)
    _same_results(hw, hs)
    o = hgref.oracle_run(t)
    b = o.results()
    a = hw.results()
    for key in ("round", "rr", "cts"):
        assert np.array_equal(np.asarray(a[key]), np.asarray(b[key])), key
    assert list(a["order"]) == list(b["order"])


@pytest.mark.parametrize("n,E,seed", [(4, 1024, 1), (64, 12000, 10), (256, 30000, 16), (512, 24000, 18)])
def test_wave_int32_coordinates(n, E, seed):
    t = gtrace.gossip(n, E, seed, stale_prob=0.2, stale_depth=4)
    hw = _run(t, "wave", coord32=True)
    assert hw.phase_times()["compact"] == 0 and hw.phase_times()["la_wave"] == 1
    hs = _run(t, "sweep", coord32=True)
    _same_coords(hw, hs, t.E, seed)
    _same_results(hw, hs)


@pytest.mark.parametrize("n,E,seed,chunk", [(4, 1024, 21, 64), (5, 700, 23, 13), (16, 4000, 24, 333),
                                            (64, 12000, 25, 1000), (256, 30000, 26, 2500), (1024, 20000, 27, 4000)])
def test_wave_incremental_calls(n, E, seed, chunk):
    """Chunked RunConsensus: every call's pass starts at the chains' first new rows and reads
    the op rows of earlier calls from HBM."""
    t = gtrace.gossip(n, E, seed, stale_prob=0.3, stale_depth=4, n_silent=300 if n > 896 else 0)
    hw = _run(t, "wave", chunk=chunk)
    pt = hw.phase_times()
    assert pt["la_wave"] == 1 and pt["la_wave_fallbacks"] == 0 and pt["rebuild"] == 0, pt
    hs = _run(t, "sweep")
    _same_coords(hw, hs, t.E, seed)
    _same_results(hw, hs)


@pytest.mark.parametrize("n,E,seed,coord32", [(16, 20000, 30, False), (64, 100000, 31, False), (64, 60000, 32, True),
                                             (256, 200000, 33, False), (128, 150000, 34, False)])
def test_wave_time_segments(n, E, seed, coord32):
    """Large single graphs: the wavefront runs on time segments concurrently (lower bounds),
    then the verify sweep and the dirty sweeps complete the rows."""
    t = gtrace.gossip(n, E, seed, stale_prob=0.2, stale_depth=4)
    hw = _run(t, "wave", coord32=coord32)
    pt = hw.phase_times()
    assert pt["la_wave"] == 1 and pt["la_wave_segs"] > 1 and pt["la_wave_fallbacks"] == 0, pt
    hs = _run(t, "sweep", coord32=coord32)
    _same_coords(hw, hs, t.E, seed, k=300)
    _same_results(hw, hs)


@pytest.mark.parametrize("n,E,seed", [(256, 600000, 35), (64, 100000, 36)])
def test_wave_segments_exactness_check(n, E, seed):
    """The time-segmented pass on large gossip graphs (more than the 64 head rows per chain in each
    segment): the exactness check (k_la_seg_check) proves every row exact, so the verify sweep is
    skipped; coordinates and consensus equal the sweeps'."""
    t = gtrace.gossip(n, E, seed, stale_prob=0.2, stale_depth=4)
    hw = _run(t, "wave")
    pt = hw.phase_times()
    assert pt["la_wave_segs"] > 1 and pt["la_verify"] == 0 and pt["la_wave_fallbacks"] == 0, pt
    hv = _run(t, "wave+verify")
    assert hv.phase_times()["la_verify"] == 1
    hs = _run(t, "sweep")
    _same_coords(hw, hs, t.E, seed, k=3000)
    _same_coords(hw, hv, t.E, seed + 1, k=3000)
    _same_results(hw, hs)


@pytest.mark.parametrize("n,E,seed,segs", [(16, 20000, 37, 48), (32, 30000, 38, 200)])
def test_wave_segments_check_fails_safe(n, E, seed, segs):
    """Segments so short that head rows read other segments' head rows: the check fails and the verify
    sweep runs; the result still equals the sweeps'."""
    t = gtrace.gossip(n, E, seed, stale_prob=0.3, stale_depth=4)
    hw = _run(t, segs)
    pt = hw.phase_times()
    assert pt["la_wave_segs"] == segs and pt["la_verify"] == 1, pt
    hs = _run(t, "sweep")
    _same_coords(hw, hs, t.E, seed, k=1500)
    _same_results(hw, hs)


def test_wave_batched_graphs():
    """One workgroup per (graph, column block): 8 independent 16-peer graphs."""
    n, G, E = 16, 8, 3000
    ts = [gtrace.gossip(n, E, 100 + g, stale_prob=0.2, stale_depth=4) for g in range(G)]
    cat = gtrace.concat_graphs(ts)
    hw = _run(cat, "wave", graphs=G)
    assert hw.phase_times()["la_wave"] == 1
    hs = _run(cat, "sweep", graphs=G)
    _same_coords(hw, hs, cat.E, 5)
    for g in range(G):
        _same_results(hw, hs, g)


# ---- small graphs: the whole graph in one workgroup's LDS (k_la_small) ----------------------------
# (sized to the kernel's bound: a graph's events x (words per row + 1) x 4 bytes <= 150 KB)
SMALL = [(1, 64, 31, 0, 0.0), (2, 300, 32, 0, 0.0), (4, 1024, 1, 0, 0.0), (5, 1500, 33, 1, 0.3),
         (8, 4000, 34, 0, 0.2), (16, 3000, 35, 5, 0.5), (32, 1000, 36, 0, 0.1)]


@pytest.mark.parametrize("n,E,seed,silent,stale", SMALL)
def test_small_graph_matches_ring_sweeps_and_oracle(n, E, seed, silent, stale):
    t = gtrace.gossip(n, E, seed, n_silent=silent, stale_prob=stale, stale_depth=4)
    h = _run(t, "wave")
    assert h.phase_times()["la_small"] == 1, "the small-graph lastAncestors kernel did not run"
    hr = _run(t, "ring")
    assert hr.phase_times()["la_small"] == 0 and hr.phase_times()["la_wave"] == 1
    hs = _run(t, "sweep")
    _same_coords(h, hr, t.E, seed)
    _same_coords(h, hs, t.E, seed + 1)
    _same_results(h, hs)
    b, a = hgref.oracle_run(t).results(), h.results()
    for key in ("round", "rr", "cts"):
        assert np.array_equal(np.asarray(a[key]), np.asarray(b[key])), key
    assert list(a["order"]) == list(b["order"])


@pytest.mark.parametrize("n,E,seed,chunk,coord32", [(4, 1024, 41, 100, False), (8, 3000, 42, 250, False),
                                                    (5, 2000, 43, 300, True), (16, 1500, 44, 200, True)])
def test_small_graph_incremental(n, E, seed, chunk, coord32):
    """Calls that resume: the rows of earlier calls are read from HBM into LDS first."""
    t = gtrace.gossip(n, E, seed, stale_prob=0.2, stale_depth=3)
    h = _run(t, "wave", coord32=coord32, chunk=chunk)
    assert h.phase_times()["la_small"] == 1
    hs = _run(t, "sweep", coord32=coord32, chunk=chunk)
    _same_coords(h, hs, t.E, seed)
    _same_results(h, hs)
    o = hgref.oracle_run(t, chunk).results()
    assert list(h.results()["order"]) == list(o["order"])


def test_small_graph_batched():
    """One workgroup per graph of a batch."""
    n, G = 8, 40
    traces = [gtrace.gossip(n, 500 + 9 * g, 900 + g, stale_prob=0.1 * (g % 3), stale_depth=3) for g in range(G)]
    t = gtrace.concat_graphs(traces)
    from babble_amd.hashgraph import Hashgraph
    h = Hashgraph(n, capacity=t.E, n_graphs=G)
    h.insert_trace(t)
    h.RunConsensus()
    assert h.phase_times()["la_small"] == 1
    a = h.results()
    off = 0
    for g, tg in enumerate(traces):
        if g % 7 == 0 or g == G - 1:
            o = hgref.oracle_run(tg).results()
            sl = slice(off, off + tg.E)
            for k in ("round", "witness", "famous", "rr", "cts"):
                assert np.array_equal(np.asarray(a[k])[sl], np.asarray(o[k])), (g, k)
            assert list(h.ConsensusEvents(g) - off) == list(o["order"]), g
        off += tg.E
