"""Insert path (device-side validation, hgx_insert.hip), context lifecycle and the Store
views of libhgx, through the C ABI, against the CPU oracle.

InsertEvent's first-failure semantics (hashgraph.go:356-445, common/rolling_index.go:54-68)
are checked batch by batch: the GPU accepts the same prefix as the oracle fed one event at
a time and returns the same Go error string. The Store views (store.go:3-25) are compared
with the oracle's own state, and node/core_test.go's playbooks are replayed the way the
cgo shim drives libhgx (Known -> ParticipantEvents for Diff, wire indices, one batched
insert per sync)."""
import numpy as np
import pytest

import hgref
from babble_amd import trace as gtrace

pytestmark = pytest.mark.gpu

COLS = ("creator", "index", "sp", "op", "ts", "hash", "s", "ntx", "txnil")


def _hg(n, cap=1 << 14, graphs=1):
    from babble_amd.hashgraph import Hashgraph
    return Hashgraph(n, capacity=cap, n_graphs=graphs)


class _Rows:
    """trace rows as columns (editable copies)"""

    def __init__(self, t, sl):
        for k in COLS:
            setattr(self, k, np.array(getattr(t, k)[sl]))
        self.txl = [t.txs(i) for i in range(sl.start, sl.stop)]

    @property
    def E(self):
        return len(self.creator)


def _gpu_insert(h, r, device):
    """(events accepted, Go error string) of one batch"""
    from babble_amd._lib import HgxError
    before = h.num_events()
    try:
        if device:
            from babble_amd.hashgraph import DeviceTrace
            h.insert_device(DeviceTrace(r))
        else:
            h.insert_arrays(*[getattr(r, k) for k in COLS])
        msg = ""
    except HgxError as e:
        msg = e.msg
    return h.num_events() - before, msg


def _oracle_insert(o, r):
    for k in range(r.E):
        rc, msg = o.insert(int(r.creator[k]), int(r.index[k]), int(r.sp[k]), int(r.op[k]), int(r.ts[k]),
                           r.hash[k].tobytes(), r.s[k].tobytes(), r.txl[k])
        if rc:
            return k, msg
    return r.E, ""


def _both(h, o, r, device):
    got, want = _gpu_insert(h, r, device), _oracle_insert(o, r)
    assert got == want, (got, want)
    return got


def _fork(r, t, base):
    k = 37
    sp = int(r.sp[k])
    r.sp[k] = t.sp[sp] if sp >= 0 else 0   # a second child of the self-parent's self-parent


def _unknown_op(r, t, base):
    r.op[53] = -2


def _skipped(r, t, base):
    r.index[12] += 1


def _passed(r, t, base):
    r.index[40] -= 1


def _unknown_creator(r, t, base):
    r.creator[70] = 6


def _future_op(r, t, base):
    r.op[5] = base + 5 + 3   # a later event of the same batch


@pytest.mark.parametrize("device", [False, True])
def test_batch_first_failure_matches_oracle(device):
    """Batches with one rejected event: the same accepted prefix and Go error as the oracle
    fed one event at a time; the remainder then goes in and consensus matches."""
    t = gtrace.gossip(6, 1000, 41, stale_prob=0.2, stale_depth=3)
    h, o = _hg(6, cap=2000), hgref.Oracle(6)
    _both(h, o, _Rows(t, slice(0, 200)), device)
    pos = 200
    for mutate in (_fork, _unknown_op, _skipped, _passed, _unknown_creator, _future_op):
        r = _Rows(t, slice(pos, pos + 100))
        mutate(r, t, pos)
        acc, msg = _both(h, o, r, device)
        assert msg and acc < 100, mutate.__name__
        _both(h, o, _Rows(t, slice(pos + acc, pos + 100)), device)
        pos += 100
    _both(h, o, _Rows(t, slice(pos, t.E)), device)
    h.RunConsensus()
    o.run_consensus()
    a, b = h.results(), o.results()
    for k in ("round", "witness", "famous", "rr", "cts"):
        assert np.array_equal(a[k], b[k]), k
    assert list(a["order"]) == list(b["order"])
    assert a["pending_loaded"] == b["pending_loaded"]


@pytest.mark.parametrize("device", [False, True])
def test_insert_edge_cases(device):
    """empty batch, a chain head with Index -1, a second chain head, capacity"""
    t = gtrace.gossip(4, 64, 3)
    h, o = _hg(4, cap=40), hgref.Oracle(4)
    assert _gpu_insert(h, _Rows(t, slice(0, 0)), device) == (0, "")
    r = _Rows(t, slice(0, 4))
    r.index[2] = -1
    assert _both(h, o, r, device) == (2, "SetEvent: �, Passed Index")
    _both(h, o, _Rows(t, slice(2, 4)), device)
    r = _Rows(t, slice(4, 10))
    r.sp[3] = -1
    acc, msg = _both(h, o, r, device)
    assert msg == "CheckSelfParent: Self-parent not last known event by creator"
    _both(h, o, _Rows(t, slice(4 + acc, 10)), device)
    assert _gpu_insert(h, _Rows(t, slice(10, 64)), device) == (30, "hgx_insert_events: context capacity exceeded")
    assert _gpu_insert(h, _Rows(t, slice(40, 41)), device) == (0, "hgx_insert_events: context capacity exceeded")


def test_other_parent_from_another_graph_rejected():
    n = 4
    cat = gtrace.concat_graphs([gtrace.gossip(n, 100, 5), gtrace.gossip(n, 100, 6)])
    h = _hg(n, cap=cat.E, graphs=2)
    r = _Rows(cat, slice(0, cat.E))
    r.op[150] = 10   # an event of graph 0 as other-parent of a graph-1 event
    assert _gpu_insert(h, r, False) == (150, "CheckOtherParent: Other-parent not known")


def test_device_insert_then_consensus_matches_oracle():
    from babble_amd.hashgraph import DeviceTrace
    t = gtrace.gossip(32, 6000, 8, stale_prob=0.1, stale_depth=3)
    h = _hg(32, cap=t.E)
    dt = DeviceTrace(t)
    for lo in range(0, t.E, 1500):
        h.insert_device(dt, lo, min(t.E, lo + 1500))
    h.RunConsensus()
    a, b = h.results(), hgref.oracle_run(t).results()
    for k in ("round", "witness", "famous", "rr", "cts"):
        assert np.array_equal(a[k], b[k]), k
    assert list(a["order"]) == list(b["order"])
    assert a["pending_loaded"] == b["pending_loaded"] and a["consensus_tx"] == b["consensus_tx"]


def test_clear_and_reinsert():
    """hgx_clear gives a fresh NewHashgraph: a second, different trace in the same context
    matches the oracle (bench.py times clear -> insert -> consensus per step)."""
    h = _hg(16, cap=5000)
    for seed in (61, 62):
        t = gtrace.gossip(16, 4000, seed, n_silent=2)
        h.clear()
        assert h.num_events() == 0 and h.LastRound() == -1
        h.insert_trace(t)
        h.RunConsensus()
        a, b = h.results(), hgref.oracle_run(t).results()
        assert list(a["order"]) == list(b["order"])
        for k in ("round", "rr", "cts", "undecided", "lcr", "pending_loaded"):
            assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k


@pytest.mark.parametrize("n,E,seed", [(8, 6000, 71), (64, 20000, 72)])
def test_round_table_growth_keeps_rows(n, E, seed):
    """Round tables sized for one round grow during DivideRounds (hgx_engine.cpp
    ensure_round_cap): the strongly-see rows of earlier rounds survive every growth."""
    t = gtrace.gossip(n, E, seed, stale_prob=0.2, stale_depth=3)
    h = _hg(n, cap=t.E)
    h.reserve_rounds(1)
    h.insert_trace(t)
    h.RunConsensus()
    a, b = h.results(), hgref.oracle_run(t).results()
    assert b["last_round"] > 20
    for k in ("round", "witness", "famous", "rr", "cts"):
        assert np.array_equal(a[k], b[k]), k
    assert list(a["order"]) == list(b["order"])


def test_round_table_growth_uneven_batched_graphs():
    """A batched context whose events are nearly all in graph 0 (the initial round-table
    guess assumes an even spread over graphs)."""
    n, G = 16, 8
    traces = [gtrace.gossip(n, 16000, 81)] + [gtrace.gossip(n, 64, 82 + g) for g in range(1, G)]
    h = _hg(n, cap=sum(t.E for t in traces), graphs=G)
    h.insert_trace(gtrace.concat_graphs(traces))
    h.RunConsensus()
    off = 0
    for g, t in enumerate(traces):
        o = hgref.oracle_run(t).results()
        assert list(h.ConsensusEvents(g) - off) == list(o["order"]), g
        assert h.UndecidedRounds(g) == o["undecided"] and h.LastConsensusRound(g) == o["lcr"], g
        assert h.LastRound(g) == o["last_round"], g
        off += t.E


def test_primitives_across_batched_graphs():
    """Graph 1 is a copy of graph 0: every primitive agrees within a graph and is false
    (or -1) across graphs."""
    n, E = 4, 200
    t = gtrace.gossip(n, E, 91)
    h = _hg(n, cap=2 * E, graphs=2)
    h.insert_trace(gtrace.concat_graphs([t, t]))
    h.RunConsensus()
    o = hgref.oracle_run(t)
    L = o.L
    rng = np.random.default_rng(3)
    for _ in range(60):
        x, y = (int(v) for v in rng.integers(0, E, 2))
        anc, ss = L.hgo_ancestor(o.h, x, y), L.hgo_strongly_see(o.h, x, y)
        osa = L.hgo_oldest_self_ancestor_to_see(o.h, x, y)
        assert h.Ancestor(x, y) == bool(anc) and h.Ancestor(x + E, y + E) == bool(anc)
        assert h.StronglySee(x, y) == bool(ss) and h.StronglySee(x + E, y + E) == bool(ss)
        assert h.OldestSelfAncestorToSee(x, y) == osa
        assert h.OldestSelfAncestorToSee(x + E, y + E) == (osa + E if osa >= 0 else -1)
        if x != y:
            assert not h.Ancestor(x + E, y) and not h.See(x, y + E)
            assert not h.StronglySee(x + E, y) and h.OldestSelfAncestorToSee(x + E, y) == -1


def test_store_views_match_oracle():
    t = gtrace.gossip(8, 3000, 101, stale_prob=0.3, stale_depth=4)
    h = _hg(8, cap=t.E)
    h.insert_trace(t)
    h.RunConsensus()
    o = hgref.oracle_run(t)
    spi, opc, opi = h.wire_info()
    for x in range(0, t.E, 7):
        assert (spi[x], opc[x], opi[x]) == o.wire(x)
        ev = h.GetEvent(x)
        assert (ev["creator"], ev["index"], ev["self_parent"], ev["other_parent"], ev["timestamp"]) == \
            (t.creator[x], t.index[x], t.sp[x], t.op[x], t.ts[x])
        assert h.ReadWireInfo(int(t.creator[x]), int(spi[x]), int(opc[x]), int(opi[x])) == (t.sp[x], t.op[x])
    known = o.known()
    assert list(h.Known()) == list(known)
    for p in range(8):
        evs = [i for i in range(t.E) if t.creator[i] == p]
        assert h.LastFrom(p) == (evs[-1], False)
        assert h.ParticipantEvents(p, -1) == evs
        assert h.ParticipantEvents(p, 10) == evs[11:]
        assert h.ParticipantEvents(p, int(known[p])) == []
        assert h.ParticipantEvent(p, 5) == evs[5]
        assert h.GetRoot(p) == dict(X=-1, Y=-1, Index=-1, Round=-1)
    for b in h.Blocks():
        assert h.GetBlock(b["rr"]) == b
    g, rr, cts = h.consensus_received()
    res = o.results()
    assert list(g) == list(res["order"])
    assert list(rr) == [int(res["rr"][x]) for x in g] and list(cts) == [int(res["cts"][x]) for x in g]


def test_store_errors_are_go_strings():
    from babble_amd._lib import HgxError
    t = gtrace.gossip(4, 100, 5)
    h = _hg(4, cap=t.E)
    h.insert_trace(t)
    cases = [(lambda: h.ParticipantEvent(1, 1000), "Ϩ, Not Found"),
             (lambda: h.ParticipantEvent(1, -5), "�, Too Late"),
             (lambda: h.ParticipantEvents(1, -3), "\x03, Too Late"),
             (lambda: h.LastFrom(9), "9, Not Found"),
             (lambda: h.GetBlock(12345), "12345, Not Found")]
    for f, msg in cases:
        with pytest.raises(HgxError) as e:
            f()
        assert e.value.msg == msg
    assert _hg(4, cap=8).LastFrom(2) == (-1, True)


def test_core_playbooks_as_the_shim_calls(plays):
    """node/core_test.go's playbooks (TestConsensus, TestConsensusFF) with every Core on its
    own libhgx context, driven the way INTEGRATION.md's shim does: Diff = hgx_known on the
    receiver + hgx_participant_events on the sender (core.go:166-188), the wire indices of
    hgx_wire_info resolved with hgx_read_wire_info (hashgraph.go:569-614) or inside the batch,
    the unknown events plus the new head inserted in ONE hgx_insert_events call (Core.Sync,
    core.go:190-230), then RunConsensus. Must equal the oracle-backed Core simulation."""
    for fx in ("core_consensus", "core_ff"):
        p = plays[fx]
        n = p["n"]
        fac = hgref.EventFactory(fx, n)
        so = hgref.CoreSim(fx, n, lambda m: hgref.Oracle(m))
        hexes = {}                             # event hex -> wire event (shared by all cores)
        cores = [dict(h=_hg(n, cap=4096), hexes=[], pool=[], head="", seq=0) for _ in range(n)]

        def make(c, index, sp_hex, op_hex, txs):
            e = fac.make(c, index, sp_hex, op_hex, txs, f"ev{len(hexes)}")
            hexes[e["hex"]] = e
            return e

        def insert(core, evs, parents):
            cols = {k: [] for k in COLS}
            for e, (sp, op) in zip(evs, parents):
                for k, v in (("creator", e["creator"]), ("index", e["index"]), ("sp", sp), ("op", op),
                             ("ts", e["ts"]), ("ntx", len(e["txs"] or [])), ("txnil", 1 if e["txs"] is None else 0)):
                    cols[k].append(v)
                cols["hash"].append(np.frombuffer(e["hash"], np.uint8))
                cols["s"].append(np.frombuffer(e["s"], np.uint8))
            core["h"].insert_arrays(*[np.stack(cols[k]) if k in ("hash", "s") else cols[k] for k in COLS])
            core["hexes"].extend(e["hex"] for e in evs)

        for i in range(n):   # Core.Init: genesis, nil transactions (core.go:79-85)
            e = make(i, 0, "", "", None)
            insert(cores[i], [e], [(-1, -1)])
            cores[i]["head"] = e["hex"]
        for frm, to, pl in p["playbook"]:
            src, dst = cores[frm], cores[to]
            known = dst["h"].Known()
            lids = sorted(g for q in range(n) for g in src["h"].ParticipantEvents(q, int(known[q])))
            spi, opc, opi = src["h"].wire_info()
            E0 = dst["h"].num_events()
            pending = {}                      # (creator, index) -> gid of this batch on dst
            batch, parents = [], []
            for lid in lids:                  # ToWire on the sender, ReadWireInfo on the receiver
                e = hexes[src["hexes"][lid]]
                sp, op = -1, -1
                if spi[lid] >= 0:
                    sp = pending.get((e["creator"], int(spi[lid])))
                    if sp is None:
                        sp = dst["h"].ReadWireInfo(e["creator"], int(spi[lid]), -1, -1)[0]
                if opi[lid] >= 0:
                    op = pending.get((int(opc[lid]), int(opi[lid])))
                    if op is None:
                        op = dst["h"].ReadWireInfo(e["creator"], -1, int(opc[lid]), int(opi[lid]))[1]
                pending[(e["creator"], e["index"])] = E0 + len(batch)
                batch.append(e)
                parents.append((sp, op))
            dst["pool"].extend(x.encode() for x in pl)
            if batch or dst["pool"]:          # the new head (core.go:215-227)
                other = batch[-1]["hex"] if batch else ""
                ne = make(to, dst["seq"] + 1, dst["head"], other, list(dst["pool"]))
                head_gid = dst["hexes"].index(dst["head"])
                parents.append((head_gid, E0 + len(batch) - 1 if batch else -1))
                batch.append(ne)
                dst["head"], dst["seq"], dst["pool"] = ne["hex"], dst["seq"] + 1, []
            insert(dst, batch, parents)
            dst["h"].RunConsensus()
            so.sync_and_run(frm, to, [x.encode() for x in pl])
        for c in range(n):
            got = [cores[c]["hexes"][int(x)] for x in cores[c]["h"].ConsensusEvents()]
            assert got == so.consensus_hex(c), (fx, c)
            assert cores[c]["h"].LastConsensusRound() == so.backends[c].last_consensus_round()


def test_commit_callback_like_commit_ch():
    """hgx_set_commit_callback: commitCh sends (hashgraph.go:848-854) — every block with
    transactions, in SetBlock order, over a chunked run; the callback reads the block's events."""
    t = gtrace.gossip(8, 4000, 91, stale_prob=0.1, stale_depth=2)
    h = _hg(8, cap=t.E)
    got = []

    def on_block(g, b, rr, first, nev, ntx):
        order = h.ConsensusEvents(g)
        txs = [t.tx_payload(int(x)) for x in order[first:first + nev]]
        got.append((b, rr, ntx, sum(len(x) for x in txs)))

    h.set_commit_callback(on_block)
    for lo in range(0, t.E, 500):
        h.insert_trace(t, lo, min(t.E, lo + 500))
        h.RunConsensus()
    blocks = h.Blocks()
    want = [(i, b["rr"], b["ntx"], b["ntx"]) for i, b in enumerate(blocks) if b["ntx"] > 0]
    assert got == want and len(got) > 3
    h.set_commit_callback(None)


def test_commit_callback_sees_final_state_and_raises():
    """The callback runs after FindOrder has updated the graph state (ConsensusTransactions,
    PendingLoadedEvents read inside it equal the values after the call), and an exception it
    raises surfaces from the RunConsensus call instead of being dropped by ctypes."""
    t = gtrace.gossip(8, 3000, 92, stale_prob=0.1, stale_depth=2)
    h = _hg(8, cap=t.E)
    seen = []
    h.set_commit_callback(lambda *a: seen.append((h.ConsensusTransactions(), h.PendingLoadedEvents())))
    h.insert_trace(t)
    h.RunConsensus()
    assert seen and all(s == (h.ConsensusTransactions(), h.PendingLoadedEvents()) for s in seen)

    class Boom(Exception):
        pass

    def bad(*a):
        raise Boom("consumer failed")

    h2 = _hg(8, cap=t.E)
    h2.set_commit_callback(bad)
    h2.insert_trace(t)
    with pytest.raises(Boom):
        h2.RunConsensus()
    assert len(h2.ConsensusEvents()) > 0   # the call itself completed
    h2.set_commit_callback(None)


def test_core_playbooks_through_wire_events(plays):
    """node/core_test.go's playbooks with Core.Sync fed as the network delivers it: the sender's
    WireEvents (hgx_wire_info = SetWireInfo) inserted by the receiver with hgx_insert_wire_events
    (ReadWireInfo + InsertEvent per event, one call per sync), then the new head and RunConsensus.
    Must equal the oracle-backed Core simulation."""
    for fx in ("core_consensus", "core_ff"):
        p = plays[fx]
        n = p["n"]
        fac = hgref.EventFactory(fx, n)
        so = hgref.CoreSim(fx, n, lambda m: hgref.Oracle(m))
        hexes = {}
        cores = [dict(h=_hg(n, cap=4096), hexes=[], pool=[], head="", seq=0) for _ in range(n)]

        def make(c, index, sp_hex, op_hex, txs):
            e = fac.make(c, index, sp_hex, op_hex, txs, f"ev{len(hexes)}")
            hexes[e["hex"]] = e
            return e

        def insert_local(core, e, sp, op):
            core["h"].insert_arrays([e["creator"]], [e["index"]], [sp], [op], [e["ts"]],
                                    np.frombuffer(e["hash"], np.uint8).reshape(1, 32),
                                    np.frombuffer(e["s"], np.uint8).reshape(1, 32), [len(e["txs"] or [])],
                                    [1 if e["txs"] is None else 0])
            core["hexes"].append(e["hex"])

        for i in range(n):
            e = make(i, 0, "", "", None)
            insert_local(cores[i], e, -1, -1)
            cores[i]["head"] = e["hex"]
        for frm, to, pl in p["playbook"]:
            src, dst = cores[frm], cores[to]
            known = dst["h"].Known()
            lids = sorted(g for q in range(n) for g in src["h"].ParticipantEvents(q, int(known[q])))
            spi, opc, opi = src["h"].wire_info()
            if lids:
                es = [hexes[src["hexes"][g]] for g in lids]
                dst["h"].insert_wire([e["creator"] for e in es], [e["index"] for e in es], [int(spi[g]) for g in lids],
                                     [int(opc[g]) for g in lids], [int(opi[g]) for g in lids], [e["ts"] for e in es],
                                     np.stack([np.frombuffer(e["hash"], np.uint8) for e in es]),
                                     np.stack([np.frombuffer(e["s"], np.uint8) for e in es]),
                                     [len(e["txs"] or []) for e in es], [1 if e["txs"] is None else 0 for e in es])
                dst["hexes"].extend(e["hex"] for e in es)
            dst["pool"].extend(x.encode() for x in pl)
            if lids or dst["pool"]:
                other = hexes[src["hexes"][lids[-1]]]["hex"] if lids else ""
                ne = make(to, dst["seq"] + 1, dst["head"], other, list(dst["pool"]))
                insert_local(dst, ne, dst["hexes"].index(dst["head"]),
                             dst["hexes"].index(other) if other else -1)
                dst["head"], dst["seq"], dst["pool"] = ne["hex"], dst["seq"] + 1, []
            dst["h"].RunConsensus()
            so.sync_and_run(frm, to, [x.encode() for x in pl])
        for c in range(n):
            got = [cores[c]["hexes"][int(x)] for x in cores[c]["h"].ConsensusEvents()]
            assert got == so.consensus_hex(c), (fx, c)


def test_wire_events_errors_like_read_wire_info():
    """ReadWireInfo errors stop Core.Sync after the events before them (hashgraph.go:586-598)."""
    from babble_amd._lib import HgxError
    n = 3
    h = _hg(n, cap=64)
    fac = hgref.EventFactory("wire", n)
    evs = [fac.make(i, 0, "", "", [], f"g{i}") for i in range(n)]

    def cols(rows):
        return ([r[0] for r in rows], [r[1] for r in rows], [r[2] for r in rows], [r[3] for r in rows],
                [r[4] for r in rows], [evs[0]["ts"]] * len(rows),
                np.stack([np.frombuffer(evs[i % n]["hash"], np.uint8) for i in range(len(rows))]),
                np.stack([np.frombuffer(evs[i % n]["s"], np.uint8) for i in range(len(rows))]),
                [0] * len(rows), [0] * len(rows))
    # (creator, index, sp index, op creator, op index): the genesis events, then 1's next event
    # naming 0's event 0 (in the batch), then one naming an index 1 does not have
    rows = [(0, 0, -1, -1, -1), (1, 0, -1, -1, -1), (1, 1, 0, 0, 0), (2, 0, -1, -1, -1), (2, 1, 0, 1, 7)]
    with pytest.raises(HgxError) as ei:
        h.insert_wire(*cols(rows))
    assert ei.value.msg == "\x07, Not Found" and ei.value.inserted == 4
    assert h.num_events() == 4
    with pytest.raises(HgxError) as ei:   # a creator id the participants map does not have
        h.insert_wire(*cols([(9, 0, -1, -1, -1)]))
    assert ei.value.code == 300
