"""Parity of the HIP path (libhgx through its C ABI) with the CPU oracle.

Bit-exact on every integer output: rounds, witnesses, fame, round-received,
consensus timestamps, consensus order, UndecidedRounds/LastConsensusRound
bookkeeping, counters and blocks (incl. Go-JSON block hashes)."""
import numpy as np
import pytest

import hgref
from babble_amd import trace as gtrace

pytestmark = pytest.mark.gpu


def _hg(n, cap=1 << 14, graphs=1):
    from babble_amd.hashgraph import Hashgraph
    return Hashgraph(n, capacity=cap, n_graphs=graphs)


def run_gpu(t, chunk=None, cap=None, coord32=False, fame=None, round_kernel=None, cts_kernel=None):
    h = _hg(t.n, cap or max(64, t.E))
    if coord32:
        h.set_coord_storage(1)
    if round_kernel:
        h.set_round_kernel(round_kernel)
    if cts_kernel:
        h.set_cts_kernel(cts_kernel)
    if fame:
        h.set_fame_tally(fame)
    if chunk is None:
        h.insert_trace(t)
        h.RunConsensus()
    else:
        for lo in range(0, t.E, chunk):
            h.insert_trace(t, lo, min(t.E, lo + chunk))
            h.RunConsensus()
    return h


def block_hashes_gpu(h, t, graph=0):
    from babble_amd.hashgraph import block_hash
    order = h.ConsensusEvents(graph)
    out = []
    for b in h.Blocks(graph):
        txs = []
        for g in order[b["first"]:b["first"] + b["n_events"]]:
            txs.extend((t.txs(int(g)) if callable(getattr(t, "txs", None)) else t.txs[int(g)]) or [])
        out.append(block_hash(b["rr"], txs, b["tx_nil"]))
    return out


def compare(h, o, t, graph=0, hashes=True):
    a = h.results(graph)
    b = o.results()
    for k in ("round", "witness", "famous", "rr", "cts"):
        if not np.array_equal(np.asarray(a[k]), np.asarray(b[k])):
            bad = np.nonzero(np.asarray(a[k]) != np.asarray(b[k]))[0][:10]
            raise AssertionError(f"{k} differs at gids {bad.tolist()}: gpu {np.asarray(a[k])[bad].tolist()} "
                                 f"oracle {np.asarray(b[k])[bad].tolist()}")
    assert list(a["order"]) == list(b["order"]), "consensus order"
    for k in ("last_round", "undecided", "lcr", "lcre", "consensus_tx", "pending_loaded"):
        assert a[k] == b[k], k
    ga = [(x["rr"], x["ntx"], x["tx_nil"], x["committed"]) for x in a["blocks"]]
    gb = [(x[0], x[1], x[2], x[3]) for x in b["blocks"]]
    assert ga == gb, "blocks"
    if hashes:
        assert block_hashes_gpu(h, t, graph) == [x[4] for x in b["blocks"]], "block hashes"


@pytest.mark.parametrize("name", ["round_hashgraph", "consensus_hashgraph", "funky_hashgraph", "init_hashgraph"])
def test_fixture_batch(name):
    t = hgref.fixture_trace(name)
    compare(run_gpu(t), hgref.oracle_run(t), t)


def test_kat_coordinates_and_primitives(kat):
    t = hgref.fixture_trace("round_hashgraph")
    h = run_gpu(t)
    ix = t.name_to_gid()
    for nm, ex in kat["insert_event"]["events"].items():
        la, fd = h.coords(ix[nm])
        assert list(la) == [c[0] for c in ex["la"]]
        assert list(fd) == [c[0] for c in ex["fd"]]
    for x, y in kat["strongly_see_true"]["pairs"]:
        assert h.StronglySee(ix[x], ix[y])
    for x, y in kat["strongly_see_false"]["pairs"]:
        assert not h.StronglySee(ix[x], ix[y])
    for nm in kat["witness"]["true"]:
        assert h.Witness(ix[nm])
    for nm in kat["witness"]["false"]:
        assert not h.Witness(ix[nm])
    for nm, r in kat["round"]["expect"].items():
        assert h.Round(ix[nm]) == r
    t2 = hgref.fixture_trace("consensus_hashgraph")
    h2 = run_gpu(t2)
    ix2 = t2.name_to_gid()
    for x, y, a in kat["oldest_self_ancestor_to_see"]["expect"]:
        assert h2.OldestSelfAncestorToSee(ix2[x], ix2[y]) == (ix2[a] if a else -1)
    ce = h2.ConsensusEvents()
    assert len(ce) == 7 and t2.names[ce[0]] == "e0" and t2.names[ce[6]] == "e02"
    assert h2.PendingLoadedEvents() == 2
    t3 = hgref.fixture_trace("funky_hashgraph")
    h3 = run_gpu(t3)
    assert h3.LastRound() == 5 and h3.UndecidedRounds() == [4, 5]
    assert {b["rr"]: b["ntx"] for b in h3.Blocks()} == {1: 6, 2: 7, 3: 7}


GOSSIP = [
    (4, 1024, 1, 0, 0.0), (4, 1024, 2, 0, 0.0), (3, 600, 3, 0, 0.3), (5, 800, 4, 1, 0.0), (7, 1500, 5, 2, 0.4),
    (16, 4000, 6, 0, 0.0), (16, 4000, 7, 5, 0.5), (32, 6000, 8, 0, 0.0), (64, 12000, 9, 0, 0.0),
    (64, 12000, 10, 21, 0.2), (100, 15000, 11, 0, 0.0), (128, 20000, 12, 0, 0.0), (2, 300, 13, 0, 0.0),
    (1, 64, 14, 0, 0.0), (200, 20000, 15, 60, 0.0), (256, 30000, 16, 0, 0.0),
    # n > 256: the per-candidate step with the candidates in chunks of 128
    (300, 24000, 17, 0, 0.0), (512, 24000, 18, 100, 0.2), (1024, 16000, 19, 300, 0.0), (1000, 30000, 20, 330, 0.3)]


@pytest.mark.parametrize("n,E,seed,silent,stale", GOSSIP)
def test_gossip_batch(n, E, seed, silent, stale):
    t = gtrace.gossip(n, E, seed, n_silent=silent, stale_prob=stale, stale_depth=4)
    compare(run_gpu(t), hgref.oracle_run(t), t, hashes=(E <= 6000))


@pytest.mark.parametrize("n,E,seed,silent,stale", [(4, 1024, 1, 0, 0.0), (7, 1500, 5, 2, 0.4), (64, 12000, 10, 21, 0.2),
                                                   (128, 20000, 12, 0, 0.0), (256, 30000, 16, 0, 0.0),
                                                   (300, 24000, 17, 0, 0.0), (1024, 16000, 19, 300, 0.0)])
def test_gossip_block_search_round_kernel(n, E, seed, silent, stale):
    """The block binary-search round step (hgx_set_round_kernel(ctx, 1); k_round_step_big
    above n = 256) against the oracle."""
    t = gtrace.gossip(n, E, seed, n_silent=silent, stale_prob=stale, stale_depth=4)
    compare(run_gpu(t, round_kernel="block"), hgref.oracle_run(t), t, hashes=False)


@pytest.mark.parametrize("n,E,seed,silent,stale,chunk", [(64, 12000, 10, 21, 0.2, None), (100, 15000, 11, 0, 0.0, None),
                                                         (256, 30000, 16, 0, 0.0, None), (512, 24000, 18, 100, 0.2, None),
                                                         (128, 20000, 12, 0, 0.0, 1000), (1000, 30000, 20, 330, 0.3, None)])
def test_gossip_pipelined_cts_kernel(n, E, seed, silent, stale, chunk):
    """The pipelined consensus timestamp kernel (hgx_set_cts_kernel(ctx, 2), k_cts_pipe +
    k_cts_redo) against the oracle; the default per-tile kernel runs in every other test."""
    t = gtrace.gossip(n, E, seed, n_silent=silent, stale_prob=stale, stale_depth=4)
    compare(run_gpu(t, chunk=chunk, cts_kernel="pipe"), hgref.oracle_run(t, chunk=chunk), t, hashes=False)


def _expect_compact(t):
    """Coordinate storage rule of DivideRounds (hgx_engine.cpp): uint16 iff n is even and
    every Index <= 65533."""
    return t.n % 2 == 0 and int(t.index.max(initial=0)) <= 65533


@pytest.mark.parametrize("n,E,seed,silent,stale", [(4, 1024, 1, 0, 0.0), (16, 4000, 7, 5, 0.5), (64, 12000, 10, 21, 0.2),
                                                   (128, 20000, 12, 0, 0.0), (256, 30000, 16, 0, 0.0),
                                                   (512, 24000, 18, 100, 0.2)])
def test_gossip_int32_coordinates(n, E, seed, silent, stale):
    """The int32 coordinate path (forced) gives the same results as the oracle."""
    t = gtrace.gossip(n, E, seed, n_silent=silent, stale_prob=stale, stale_depth=4)
    h = run_gpu(t, coord32=True)
    assert h.phase_times()["compact"] == 0
    compare(h, hgref.oracle_run(t), t, hashes=False)


@pytest.mark.parametrize("E,seed", [(120000, 31), (140000, 32)])
def test_compact_coordinate_threshold(E, seed):
    """Two peers with chains around the uint16 limit: the mode follows the rule and
    both paths match the oracle."""
    t = gtrace.gossip(2, E, seed)
    h = run_gpu(t)
    assert h.phase_times()["compact"] == int(_expect_compact(t))
    compare(h, hgref.oracle_run(t), t, hashes=False)


def test_gossip_batch_uses_compact_coordinates():
    t = gtrace.gossip(64, 12000, 9)
    h = run_gpu(t)
    assert h.phase_times()["compact"] == 1
    t = gtrace.gossip(7, 1500, 5)
    h = run_gpu(t)
    assert h.phase_times()["compact"] == 0


@pytest.mark.parametrize("n,E,seed,chunk", [(4, 1024, 21, 64), (4, 600, 22, 7), (5, 700, 23, 13), (16, 2000, 24, 100),
                                            (3, 200, 25, 1)])
def test_gossip_chunked(n, E, seed, chunk):
    t = gtrace.gossip(n, E, seed, stale_prob=0.2, stale_depth=3)
    compare(run_gpu(t, chunk=chunk), hgref.oracle_run(t, chunk=chunk), t)


def test_batched_graphs_match_independent_oracles():
    G, n, Es = 6, 16, 3000
    traces = [gtrace.gossip(n, Es, 100 + g, stale_prob=0.1 * (g % 3), stale_depth=2) for g in range(G)]
    cat = gtrace.concat_graphs(traces)
    h = _hg(n, cap=cat.E, graphs=G)
    h.insert_trace(cat)
    h.RunConsensus()
    off = 0
    for g, t in enumerate(traces):
        o = hgref.oracle_run(t).results()
        order = h.ConsensusEvents(g) - off
        assert list(order) == list(o["order"]), g
        assert h.UndecidedRounds(g) == o["undecided"]
        assert h.LastConsensusRound(g) == o["lcr"]
        assert h.ConsensusTransactions(g) == o["consensus_tx"]
        assert [(b["rr"], b["ntx"], b["tx_nil"]) for b in h.Blocks(g)] == [(b[0], b[1], b[2]) for b in o["blocks"]]
        off += t.E


class _GpuCore:
    def __init__(self, n):
        self.h = _hg(n, cap=4096)

    def insert(self, creator, index, sp, op, ts, hsh, s, txs):
        from babble_amd._lib import HgxError
        try:
            self.h.InsertEvent(creator, index, sp, op, ts, hsh, s, txs)
            return 0, ""
        except HgxError as e:
            return e.code, e.msg

    def run_consensus(self):
        from babble_amd._lib import HgxError
        try:
            self.h.RunConsensus()
            return 0, ""
        except HgxError as e:
            return e.code, e.msg

    def consensus_events(self):
        return self.h.ConsensusEvents()

    def last_consensus_round(self):
        return self.h.LastConsensusRound()

    def known(self):
        return self.h.Known()


@pytest.mark.parametrize("fx", ["core_consensus", "core_ff"])
def test_core_playbooks_gpu_vs_oracle(plays, fx):
    p = plays[fx]
    sg = hgref.CoreSim(fx, p["n"], _GpuCore)
    so = hgref.CoreSim(fx, p["n"], lambda n: hgref.Oracle(n))
    for frm, to, pl in p["playbook"]:
        sg.sync_and_run(frm, to, [x.encode() for x in pl])
        so.sync_and_run(frm, to, [x.encode() for x in pl])
    for c in range(p["n"]):
        assert sg.consensus_hex(c) == so.consensus_hex(c)
        assert sg.backends[c].last_consensus_round() == so.backends[c].last_consensus_round()


def test_insert_errors_match_go_strings():
    from babble_amd._lib import HgxError
    h = _hg(3, cap=64)
    fac = hgref.EventFactory("err", 3)
    for i in range(3):
        e = fac.make(i, 0, "", "", [], f"e{i}")
        h.InsertEvent(i, 0, -1, -1, e["ts"], e["hash"], e["s"], [])
    a = fac.make(2, 0, "", "", [b"yo"], "a")
    with pytest.raises(HgxError) as ei:
        h.InsertEvent(2, 0, -1, -1, a["ts"], a["hash"], a["s"], [b"yo"])
    assert ei.value.msg == "CheckSelfParent: Self-parent not last known event by creator"
    with pytest.raises(HgxError) as ei:
        h.InsertEvent(0, 1, 0, -2, a["ts"], a["hash"], a["s"], [])
    assert ei.value.msg == "CheckOtherParent: Other-parent not known"
    with pytest.raises(HgxError) as ei:
        h.InsertEvent(0, 2, 0, -1, a["ts"], a["hash"], a["s"], [])
    assert ei.value.code == 4 and ei.value.msg == "SetEvent: \x02, Skipped Index"
    with pytest.raises(HgxError) as ei:
        h.InsertEvent(7, 0, -1, -1, a["ts"], a["hash"], a["s"], [])
    assert ei.value.msg == "CheckSelfParent: 7, Not Found"


def test_empty_decide_fame_error_like_go():
    from babble_amd._lib import HgxError
    h = _hg(4, cap=16)
    h.DivideRounds()
    with pytest.raises(HgxError) as ei:
        h.DecideFame()
    assert ei.value.msg == "0, Not Found"


FAME_CASES = [(4, 1024, 2, 0, 0.0), (7, 1500, 5, 2, 0.4), (16, 4000, 7, 5, 0.5), (128, 20000, 12, 0, 0.0),
              (200, 20000, 15, 60, 0.0), (256, 30000, 16, 0, 0.3), (512, 24000, 18, 100, 0.2),
              (1024, 16000, 19, 300, 0.0)]


@pytest.mark.parametrize("mode", ["vote", "popc", "mfma"])
@pytest.mark.parametrize("n,E,seed,silent,stale", FAME_CASES)
def test_fame_kernels_agree_with_oracle(mode, n, E, seed, silent, stale):
    """Every DecideFame kernel (per-round popcount k_fame_vote, witness-tiled k_fame_tile with
    the popcount or the int8 MFMA tally; hgx_set_fame_tally picks one) gives the oracle's fame,
    at every n (small n reaches the coin rounds, (j-i) % n == 0)."""
    t = gtrace.gossip(n, E, seed, n_silent=silent, stale_prob=stale, stale_depth=4)
    compare(run_gpu(t, fame=mode), hgref.oracle_run(t), t, hashes=False)


@pytest.mark.parametrize("mode", ["vote", "popc", "mfma"])
@pytest.mark.parametrize("name", ["funky_hashgraph", "consensus_hashgraph"])
def test_fame_kernels_on_fixtures(mode, name):
    """The reference fixtures (funky_hashgraph has a coin round, hashgraph_test.go:1407-1462)
    through each fame kernel."""
    t = hgref.fixture_trace(name)
    compare(run_gpu(t, fame=mode), hgref.oracle_run(t), t)


@pytest.mark.parametrize("mode", ["popc", "mfma"])
def test_fame_tile_batched_graphs(mode):
    """k_fame_tile's (graph, round, witness tile) block mapping over a batched context."""
    G, n, Es = 3, 128, 12000
    traces = [gtrace.gossip(n, Es, 300 + g, n_silent=10 * g, stale_prob=0.15 * g, stale_depth=3) for g in range(G)]
    cat = gtrace.concat_graphs(traces)
    h = _hg(n, cap=cat.E, graphs=G)
    h.set_fame_tally(mode)
    h.insert_trace(cat)
    h.RunConsensus()
    off = 0
    for g, t in enumerate(traces):
        o = hgref.oracle_run(t).results()
        assert list(h.ConsensusEvents(g) - off) == list(o["order"]), g
        assert h.UndecidedRounds(g) == o["undecided"]
        assert h.LastConsensusRound(g) == o["lcr"]
        off += t.E
