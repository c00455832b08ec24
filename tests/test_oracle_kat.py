"""Pins the CPU oracle against every known-answer assertion of the reference's own
tests (hashgraph/hashgraph_test.go, node/core_test.go), restated in tests/golden/kat.json.
CPU only."""
import numpy as np
import pytest

import hgref
from hgref import MAXI32, Oracle, fixture_trace, oracle_run


def _batch(name):
    t = fixture_trace(name)
    o = Oracle(t.n)
    o.insert_trace(t)
    return t, o, t.name_to_gid()


def _g(ix, nm):
    return ix[nm] if nm else -1


@pytest.mark.parametrize("key,expect", [("ancestor_true", 1), ("ancestor_false", 0)])
def test_ancestor(kat, key, expect):
    t, o, ix = _batch(kat[key]["fixture"])
    for x, y in kat[key]["pairs"]:
        assert o.L.hgo_ancestor(o.h, _g(ix, x), _g(ix, y)) == expect, (x, y)


@pytest.mark.parametrize("key,expect", [("self_ancestor_true", 1), ("self_ancestor_false", 0)])
def test_self_ancestor(kat, key, expect):
    t, o, ix = _batch(kat[key]["fixture"])
    for x, y in kat[key]["pairs"]:
        assert o.L.hgo_self_ancestor(o.h, _g(ix, x), _g(ix, y)) == expect, (x, y)


def test_see(kat):
    t, o, ix = _batch(kat["see_true"]["fixture"])
    for x, y in kat["see_true"]["pairs"]:
        assert o.L.hgo_see(o.h, ix[x], ix[y]) == 1


def test_insert_event_coordinates(kat):
    k = kat["insert_event"]
    t, o, ix = _batch(k["fixture"])
    for nm, ex in k["events"].items():
        la, fd = o.coords(ix[nm])
        assert list(la) == [c[0] for c in ex["la"]], nm
        assert list(fd) == [c[0] for c in ex["fd"]], nm
        # the coordinate hash must name the event at (participant, index)
        for p, (idx, ename) in enumerate(ex["fd"]):
            if ename:
                assert t.creator[ix[ename]] == p and t.index[ix[ename]] == idx
        assert list(o.wire(ix[nm])) == ex["wire"], nm
    assert o.L.hgo_pending_loaded_events(o.h) == k["pending_loaded_events"]


@pytest.mark.parametrize("key,expect", [("strongly_see_true", 1), ("strongly_see_false", 0)])
def test_strongly_see(kat, key, expect):
    t, o, ix = _batch(kat[key]["fixture"])
    for x, y in kat[key]["pairs"]:
        assert o.L.hgo_strongly_see(o.h, ix[x], ix[y]) == expect, (x, y)


def test_parent_round_witness_round(kat):
    t, o, ix = _batch("round_hashgraph")
    o.divide_rounds()
    for nm, (r, root) in kat["parent_round"]["expect"].items():
        assert o.parent_round(ix[nm]) == (r, root), nm
    for nm in kat["witness"]["true"]:
        assert o.L.hgo_witness(o.h, ix[nm]) == 1, nm
    for nm in kat["witness"]["false"]:
        assert o.L.hgo_witness(o.h, ix[nm]) == 0, nm
    for nm in kat["round_inc"]["true"]:
        assert o.L.hgo_round_inc(o.h, ix[nm]) == 1, nm
    for nm in kat["round_inc"]["false"]:
        assert o.L.hgo_round_inc(o.h, ix[nm]) == 0, nm
    for nm, r in kat["round"]["expect"].items():
        assert o.L.hgo_round(o.h, ix[nm]) == r, nm
    for a, b, d in kat["round_diff"]["expect"]:
        assert o.L.hgo_round(o.h, ix[a]) - o.L.hgo_round(o.h, ix[b]) == d


def test_divide_rounds(kat):
    k = kat["divide_rounds"]
    t, o, ix = _batch(k["fixture"])
    o.divide_rounds()
    assert o.L.hgo_last_round(o.h) == k["last_round"]
    for r, names in k["round_witnesses"].items():
        assert sorted(o.round_witnesses(int(r))) == sorted(ix[nm] for nm in names)
    # UndecidedRounds duplicate-0 quirk
    assert o.undecided_rounds() == [0, 0, 1]


def test_decide_fame(kat):
    k = kat["decide_fame"]
    t, o, ix = _batch(k["fixture"])
    o.divide_rounds()
    assert o.decide_fame()[0] == 0
    for nm, r in k["rounds"].items():
        assert o.L.hgo_round(o.h, ix[nm]) == r
    for nm in k["famous_true"]:
        assert o.L.hgo_famous(o.h, ix[nm]) == 1


def test_oldest_self_ancestor_to_see(kat):
    t, o, ix = _batch("consensus_hashgraph")
    for x, y, a in kat["oldest_self_ancestor_to_see"]["expect"]:
        assert o.L.hgo_oldest_self_ancestor_to_see(o.h, ix[x], ix[y]) == _g(ix, a), (x, y)


def test_decide_round_received(kat):
    k = kat["decide_round_received"]
    t, o, ix = _batch(k["fixture"])
    o.divide_rounds()
    o.decide_fame()
    assert o.decide_round_received()[0] == 0
    for nm, g in ix.items():
        if nm.startswith(k["prefix"]):
            assert o.L.hgo_round_received(o.h, g) == k["round_received"], nm


def test_find_order_and_blocks(kat):
    k = kat["find_order"]
    t, o, ix = _batch(k["fixture"])
    assert o.run_consensus()[0] == 0
    ce = list(o.consensus_events())
    assert len(ce) == k["consensus_len"]
    assert o.L.hgo_pending_loaded_events(o.h) == k["pending_loaded_events"]
    assert t.names[ce[0]] == k["first"]
    assert t.names[ce[6]] == k["index6"]
    kb = kat["blocks"]
    blocks = {b["rr"]: b for b in o.blocks()}
    assert blocks[kb["block_rr"]]["txs"] == [x.encode() for x in kb["txs"]]


def test_known(kat):
    t, o, ix = _batch("consensus_hashgraph")
    assert {str(i): int(v) for i, v in enumerate(o.known())} == kat["known"]["expect"]


def test_funky_fame_and_blocks(kat):
    t, o, ix = _batch("funky_hashgraph")
    o.divide_rounds()
    assert o.L.hgo_last_round(o.h) == kat["funky_fame"]["last_round"]
    assert o.decide_fame()[0] == 0
    assert o.undecided_rounds() == kat["funky_fame"]["undecided_rounds"]
    assert o.find_order()[0] == 0
    counts = {str(b["rr"]): b["ntx"] for b in o.blocks()}
    for rr, c in kat["funky_blocks"]["block_tx_counts"].items():
        assert counts[rr] == c
    # the diagram comment (hashgraph_test.go:1407-1462): w00 decided famous after the coin round
    assert o.L.hgo_famous(o.h, ix["w00"]) == 1


def test_fork_rejected():
    fac = hgref.EventFactory("fork", 3)
    o = Oracle(3)
    ev = []
    for i in range(3):
        e = fac.make(i, 0, "", "", [], f"e{i}")
        assert o.insert(i, 0, -1, -1, e["ts"], e["hash"], e["s"], [])[0] == 0
        ev.append(e)
    a = fac.make(2, 0, "", "", [b"yo"], "a")
    rc, msg = o.insert(2, 0, -1, -1, a["ts"], a["hash"], a["s"], [b"yo"])
    assert rc != 0 and msg.startswith("CheckSelfParent")
    e01 = fac.make(0, 1, ev[0]["hex"], a["hex"], [], "e01")
    rc, msg = o.insert(0, 1, 0, hgref_unknown(), e01["ts"], e01["hash"], e01["s"], [])
    assert rc != 0 and msg == "CheckOtherParent: Other-parent not known"
    e20 = fac.make(2, 1, ev[2]["hex"], e01["hex"], [], "e20")
    rc, msg = o.insert(2, 1, 2, hgref_unknown(), e20["ts"], e20["hash"], e20["s"], [])
    assert rc != 0 and msg == "CheckOtherParent: Other-parent not known"


def hgref_unknown():
    return -2


def test_index_rules():
    fac = hgref.EventFactory("idx", 2)
    o = Oracle(2)
    e0 = fac.make(0, 0, "", "", [], "e0")
    assert o.insert(0, 0, -1, -1, e0["ts"], e0["hash"], e0["s"], [])[0] == 0
    e2 = fac.make(0, 2, e0["hex"], "", [], "e2")
    rc, msg = o.insert(0, 2, 0, -1, e2["ts"], e2["hash"], e2["s"], [])
    assert rc == 4 and msg == "SetEvent: \x02, Skipped Index"
    rc, msg = o.insert(0, 0, 0, -1, e2["ts"], e2["hash"], e2["s"], [])
    assert rc == 3 and msg.endswith("Passed Index")


def _core_backend(n):
    return Oracle(n)


def test_core_consensus(plays, kat):
    fx = plays["core_consensus"]
    sim = hgref.CoreSim("core_consensus", fx["n"], _core_backend)
    for frm, to, pl in fx["playbook"]:
        sim.sync_and_run(frm, to, [x.encode() for x in pl])
    c0 = sim.consensus_hex(0)
    assert len(c0) == kat["core_consensus"]["core0_consensus_len"]
    for c in (1, 2):
        cc = sim.consensus_hex(c)
        assert cc[:len(c0)] == c0[:len(cc)]


def test_core_ff(plays, kat):
    fx = plays["core_ff"]
    k = kat["core_ff"]
    sim = hgref.CoreSim("core_ff", fx["n"], _core_backend)
    for frm, to, pl in fx["playbook"]:
        sim.sync_and_run(frm, to, [x.encode() for x in pl])
    assert sim.backends[0].last_consensus_round() == k["core0_last_consensus_round"]
    assert sim.backends[1].last_consensus_round() == k["core1_last_consensus_round"]
    assert len(sim.consensus_hex(0)) == k["core0_consensus_len"]
    c1 = sim.consensus_hex(1)
    assert len(c1) == k["core1_consensus_len"]
    for c in (2, 3):
        cc = sim.consensus_hex(c)
        for i, e in enumerate(c1):
            assert cc[i] == e


def test_rfc3339nano_and_block_json():
    L = hgref.oracle_lib()
    import ctypes as C
    buf = C.create_string_buffer(64)
    n = L.goenc_rfc3339nano(1_500_000_000_000_000_000, buf)
    assert buf.raw[:n] == b"2017-07-14T02:40:00Z"
    n = L.goenc_rfc3339nano(1_500_000_000_123_400_000, buf)
    assert buf.raw[:n] == b"2017-07-14T02:40:00.1234Z"
    # docs/design.rst:102-115 example block body
    js = hgref.go_block_json(24, [b"Node1 Tx1", b"Node1 Tx2"], False)
    assert js == b'{"RoundReceived":24,"Transactions":["Tm9kZTEgVHgx","Tm9kZTEgVHgy"]}\n'
    assert hgref.go_block_json(3, [], True) == b'{"RoundReceived":3,"Transactions":null}\n'
    assert hgref.go_block_json(3, [], False) == b'{"RoundReceived":3,"Transactions":[]}\n'


def test_sha256_matches_hashlib():
    import ctypes as C
    L = hgref.oracle_lib()
    rng = np.random.default_rng(0)
    for ln in (0, 1, 55, 56, 63, 64, 65, 119, 120, 1000):
        data = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
        out = C.create_string_buffer(32)
        L.goenc_sha256(C.create_string_buffer(data, max(ln, 1)), ln, out)
        assert out.raw == hgref.sha256(data)


def test_chunked_equals_batch_on_fixture():
    """without late witnesses, batch and chunked schedules agree."""
    t = fixture_trace("funky_hashgraph")
    a = oracle_run(t).results()
    b = oracle_run(t, chunk=7).results()
    assert list(a["order"]) == list(b["order"])
