"""Checkpoint and Bootstrap (hgx_save / hgx_bootstrap; hashgraph.go:1008-1037, the BadgerStore
replay badger_store.go:345-386) on the GPU:
  * the device writes the same bytes as the host encoder of the same events;
  * Bootstrap from a checkpoint = InsertEvent of the logged events in topological order,
    then ONE DivideRounds / DecideFame / FindOrder: bit-exact with the oracle run that way;
  * a node checkpointed mid-trace (running Core's chunked schedule), bootstrapped into a fresh
    context and continuing the chunked schedule matches the oracle replaying the same history
    (batch over the checkpointed prefix, then the same chunks);
  * a context after Reset (roots) round-trips its roots;
  * bad files are rejected with the reason."""
import numpy as np
import pytest

import hgref
from babble_amd import checkpoint
from babble_amd import trace as gtrace

pytestmark = pytest.mark.gpu


def _hg(n, cap, graphs=1):
    from babble_amd.hashgraph import Hashgraph
    return Hashgraph(n, capacity=cap, n_graphs=graphs)


def _compare(a, b):
    for k in ("round", "witness", "famous", "rr", "cts"):
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k
    assert list(a["order"]) == list(b["order"]), "consensus order"
    for k in ("last_round", "undecided", "lcr", "lcre", "consensus_tx", "pending_loaded"):
        assert a[k] == b[k], k
    assert [(x["rr"], x["ntx"], x["tx_nil"], x["committed"]) for x in a["blocks"]] == [tuple(x[:4]) for x in b["blocks"]]


@pytest.mark.parametrize("n,E,seed", [(4, 1024, 1), (16, 6000, 2), (64, 16000, 3), (256, 30000, 4)])
def test_device_file_equals_host_encoder(tmp_path, n, E, seed):
    t = gtrace.gossip(n, E, seed, stale_prob=0.2, stale_depth=3)
    h = _hg(n, t.E)
    h.insert_trace(t)
    p_dev, p_host = str(tmp_path / "dev.ckpt"), str(tmp_path / "host.ckpt")
    h.save(p_dev)
    checkpoint.write_trace(p_host, t)
    assert open(p_dev, "rb").read() == open(p_host, "rb").read()


@pytest.mark.parametrize("n,E,seed", [(4, 1024, 11), (32, 8000, 12), (256, 30000, 13)])
def test_bootstrap_equals_batch_replay(tmp_path, n, E, seed):
    t = gtrace.gossip(n, E, seed, stale_prob=0.1, stale_depth=2)
    p = str(tmp_path / "t.ckpt")
    checkpoint.write_trace(p, t)
    h = _hg(n, t.E)
    h.Bootstrap(p)
    _compare(h.results(), hgref.oracle_run(t).results())


@pytest.mark.parametrize("n,E,seed,chunk,cut", [(8, 4000, 21, 100, 2000), (64, 16000, 22, 1000, 9000),
                                                (256, 30000, 23, 1000, 17000)])
def test_checkpoint_mid_trace_then_continue(tmp_path, n, E, seed, chunk, cut):
    t = gtrace.gossip(n, E, seed, stale_prob=0.1, stale_depth=2)
    h = _hg(n, t.E)
    for lo in range(0, cut, chunk):
        h.insert_trace(t, lo, min(cut, lo + chunk))
        h.RunConsensus()
    p = str(tmp_path / "mid.ckpt")
    h.save(p)
    h.close()
    h2 = _hg(n, t.E)
    h2.Bootstrap(p)
    for lo in range(cut, E, chunk):
        h2.insert_trace(t, lo, min(E, lo + chunk))
        h2.RunConsensus()
    # the oracle replays the same history: Bootstrap (one batch over the prefix), then the chunks
    o = hgref.Oracle(n)
    o.insert_trace(t, 0, cut)
    rc, msg = o.run_consensus()
    assert not rc, msg
    for lo in range(cut, E, chunk):
        o.insert_trace(t, lo, min(E, lo + chunk))
        rc, msg = o.run_consensus()
        assert not rc, msg
    _compare(h2.results(), o.results())


def test_batched_graphs_round_trip(tmp_path):
    n, G = 16, 4
    traces = [gtrace.gossip(n, 2000 + 300 * g, 30 + g) for g in range(G)]
    t = gtrace.concat_graphs(traces)
    h = _hg(n, t.E, graphs=G)
    h.insert_trace(t)
    h.RunConsensus()
    p = str(tmp_path / "b.ckpt")
    h.save(p)
    h2 = _hg(n, t.E, graphs=G)
    h2.Bootstrap(p)
    for g in range(G):
        assert list(h2.ConsensusEvents(g)) == list(h.ConsensusEvents(g)), g
        assert h2.UndecidedRounds(g) == h.UndecidedRounds(g), g
    r = checkpoint.read(p)
    assert (r["n"], r["graphs"], r["E"]) == (n, G, t.E)


def test_rooted_context_round_trip(tmp_path):
    """A context after Reset (roots from a frame, hashgraph.go:877-995): the file carries the
    roots, Bootstrap reinstalls them and replays the events; the oracle does the same from a
    fresh Hashgraph (Reset with the roots, the frame's events, one consensus run)."""
    n, E = 16, 6000
    t = gtrace.gossip(n, E, 41)
    K = E // 2
    h = _hg(n, E)
    h.insert_trace(t, 0, K)
    h.RunConsensus()
    f = h.GetFrame()
    roots = hgref.frame_root_arrays(f)
    h.Reset(*roots, others=hgref.frame_others_keys(t, f))
    sub, _ = hgref.remap_after_reset(t, f["events"], f)
    h.insert_trace(sub)
    h.RunConsensus()
    p = str(tmp_path / "rooted.ckpt")
    h.save(p)
    r = checkpoint.read(p)
    assert r["roots"] is not None
    assert list(r["roots"][0]) == list(roots[0]) and list(r["roots"][1]) == list(roots[1])
    assert list(r["roots"][2]) == list(roots[2])
    h2 = _hg(n, E)
    h2.Bootstrap(p)
    o = hgref.Oracle(n)
    o.reset(*roots)
    o.insert_trace(sub)
    rc, msg = o.run_consensus()
    assert not rc, msg
    a, b = h2.results(), o.results()
    for k in ("round", "witness", "famous", "rr", "cts"):
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k
    assert list(a["order"]) == list(b["order"])
    assert a["last_round"] == b["last_round"] and a["undecided"] == b["undecided"]
    # what Reset kept (LastConsensusRound, LastCommitedRoundEvents, ConsensusTransactions, the
    # blocks) travels with the file: the bootstrapped node continues the saved one's state
    assert r["kept"] is not None and r["others"] is not None and len(r["others"]) == len(hgref.frame_others_keys(t, f))
    assert h2.LastConsensusRound() == h.LastConsensusRound()
    assert h2.LastCommitedRoundEvents() == h.LastCommitedRoundEvents()
    assert h2.ConsensusTransactions() == h.ConsensusTransactions()
    assert h2.PendingLoadedEvents() == h.PendingLoadedEvents()
    blk = lambda x: [(v["rr"], v["ntx"], v["tx_nil"], v["committed"]) for v in x.Blocks()]
    assert blk(h2) == blk(h) and len(blk(h)) > 0
    assert list(h2.Known()) == list(h.Known())
    # the Root.Others keys came back: a re-save is the same file
    p2 = str(tmp_path / "rooted2.ckpt")
    h2.save(p2)
    assert open(p2, "rb").read() == open(p, "rb").read()
    # a checksum-valid file whose last section is inconsistent (one byte too many) is refused before
    # the context is touched: no roots, no kept state, and the same context then bootstraps the good file
    from babble_amd._lib import HgxError
    raw = open(p, "rb").read()
    body = raw[:-8] + b"\0"
    p3 = str(tmp_path / "rooted_bad.ckpt")
    open(p3, "wb").write(body + checkpoint.fnv1a(body).to_bytes(8, "little"))
    h3 = _hg(n, E)
    with pytest.raises(HgxError, match="size mismatch"):
        h3.Bootstrap(p3)
    assert h3.LastConsensusRound() is None and h3.num_events() == 0 and h3.Blocks() == []
    h3.Bootstrap(p)
    assert list(h3.ConsensusEvents()) == list(h2.ConsensusEvents())


def test_bootstrap_restores_node_state(tmp_path):
    """TestBootstrap (hashgraph_test.go:1351-1404): the bootstrapped Hashgraph has the same
    consensus events, Known, LastConsensusRound, LastCommitedRoundEvents, ConsensusTransactions and
    PendingLoadedEvents; the file also brings back what the BadgerStore keeps for a node to serve
    its peers (badger_store.go:103-125, 309-343, 540): every event id, the participants' keys and
    the caller's per-event payloads."""
    n, E = 16, 6000
    t = gtrace.gossip(n, E, 61, stale_prob=0.1, stale_depth=2)
    keys = hgref.sign_batch(n, [0], np.zeros((1, 32), np.uint8))[0]
    pay = [gtrace.payload(int(t.creator[i]), int(t.tx_seq[i])) if t.ntx[i] else b"" for i in range(E)]
    h = _hg(n, E)
    h.set_participant_keys(keys)
    h.insert_trace(t)
    h.RunConsensus()
    p = str(tmp_path / "node.ckpt")
    h.save_with_payloads(p, pay)
    with pytest.raises(ValueError):
        h.save_with_payloads(str(tmp_path / "short.ckpt"), pay[:-1])   # one payload per event
    r = checkpoint.read(p)
    assert np.array_equal(r["ids"], t.hash) and np.array_equal(r["keys"], keys) and r["payloads"] == pay
    h2 = _hg(n, E)
    h2.Bootstrap(p)
    assert list(h2.ConsensusEvents()) == list(h.ConsensusEvents()) and len(h.ConsensusEvents()) > 0
    assert list(h2.Known()) == list(h.Known())
    assert h2.LastConsensusRound() == h.LastConsensusRound()
    assert h2.LastCommitedRoundEvents() == h.LastCommitedRoundEvents()
    assert h2.ConsensusTransactions() == h.ConsensusTransactions()
    assert h2.PendingLoadedEvents() == h.PendingLoadedEvents()
    for i in (0, 1, E // 2, E - 1):
        assert h2.event_id(i) == t.hash[i].tobytes() == h.event_id(i)
        assert h2.event_payload(i) == pay[i]
    p2 = str(tmp_path / "node2.ckpt")
    h2.save_with_payloads(p2, [h2.event_payload(i) for i in range(E)])
    assert open(p2, "rb").read() == open(p, "rb").read()


def test_compact_insert_has_no_ids(tmp_path):
    """Events inserted from hgx_events32 columns bring only the coin byte: the checkpoint has no
    id section, and the id getter says so."""
    from babble_amd._lib import HgxError
    from babble_amd.hashgraph import compact_columns
    n, E = 8, 2000
    t = gtrace.gossip(n, E, 62)
    h = _hg(n, E)
    h.insert_events32(compact_columns(t))
    h.RunConsensus()
    p = str(tmp_path / "c.ckpt")
    h.save(p)
    r = checkpoint.read(p)
    assert r["ids"] is None and np.array_equal(r["coin"], (t.hash[:, 16] != 0).astype(np.uint8))
    with pytest.raises(HgxError, match="without their ids"):
        h.event_id(0)
    h2 = _hg(n, E)
    h2.Bootstrap(p)
    assert list(h2.ConsensusEvents()) == list(h.ConsensusEvents())


def test_bootstrap_rejections(tmp_path):
    from babble_amd._lib import HgxError
    t = gtrace.gossip(8, 500, 51)
    p = tmp_path / "x.ckpt"
    checkpoint.write_trace(str(p), t)
    with pytest.raises(HgxError, match="participants"):
        _hg(4, 1000).Bootstrap(str(p))          # wrong n
    with pytest.raises(HgxError, match="capacity"):
        _hg(8, 100).Bootstrap(str(p))           # too small
    h = _hg(8, 1000)
    h.insert_trace(t, 0, 10)
    with pytest.raises(HgxError, match="fresh"):
        h.Bootstrap(str(p))                     # not a fresh Hashgraph
    raw = bytearray(p.read_bytes())
    raw[200] ^= 0x40
    p.write_bytes(bytes(raw))
    with pytest.raises(HgxError, match="checksum"):
        _hg(8, 1000).Bootstrap(str(p))
    with pytest.raises(HgxError, match="cannot open"):
        _hg(8, 1000).Bootstrap(str(tmp_path / "missing.ckpt"))
