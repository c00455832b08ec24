"""The oracle's Reset / GetFrame / Root.Others (hashgraph.go:877-995, root.go) pinned by the
reference's own tests on the consensus fixture (hashgraph_test.go:1144-1349): TestGetFrame's
roots and events, TestReset's re-insertion with explicit roots (Known after it), and
TestResetFromFrame (Known, then LastConsensusRound == 1 after consensus). CPU only."""
import numpy as np

import hgref


def _fixture():
    t = hgref.fixture_trace("consensus_hashgraph")
    idx = {nm: i for i, nm in enumerate(t.names)}
    return t, idx


def test_get_frame():   # hashgraph_test.go:1216-1300
    t, idx = _fixture()
    o = hgref.oracle_run(t)
    f = o.get_frame()
    exp = {0: (idx["e02"], idx["f1b"], 1, 0), 1: (idx["e10"], idx["e02"], 1, 0), 2: (idx["e21b"], idx["f1b"], 2, 0)}
    for p in range(3):
        assert f["roots"][p] == exp[p], p
    assert f["others"] == {}
    skip = {0: 1, 1: 1, 2: 2}
    want = sorted(g for g in range(t.E) if t.index[g] > skip[int(t.creator[g])])
    assert f["events"] == want


def test_reset_with_explicit_roots():   # hashgraph_test.go:1144-1214
    t, idx = _fixture()
    o = hgref.oracle_run(t)
    frame = {"roots": [(idx["f02b"], idx["g1"], 4, 2), (idx["f10"], idx["f02b"], 4, 2), (idx["f21"], idx["g1"], 4, 2)],
             "others": {idx["o02"]: idx["f21"]}}
    assert o.reset(*hgref.frame_root_arrays(frame)) == 0
    evs = ["g1", "g0", "g2", "g10", "g21", "o02", "g02", "h1", "h0", "h2"]
    sub, _ = hgref.remap_after_reset(t, [idx[e] for e in evs], frame)
    assert (sub.sp >= -1).all() and (sub.op != hgref.UNKNOWN).all()
    o.insert_trace(sub)
    assert list(o.known()) == [8, 7, 7]


def test_reset_from_frame():   # hashgraph_test.go:1302-1349
    t, idx = _fixture()
    o = hgref.oracle_run(t)
    f = o.get_frame()
    assert o.reset(*hgref.frame_root_arrays(f)) == 0
    sub, _ = hgref.remap_after_reset(t, f["events"], f)
    o.insert_trace(sub)
    assert list(o.known()) == [8, 7, 7]
    o.run_consensus()
    assert o.last_consensus_round() == 1
