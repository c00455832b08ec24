"""Reset / GetFrame / Root.Others on the GPU path (hgx_reset, hgx_get_frame; hashgraph.go:877-995)
against the oracle: the reference's fixture scenarios (hashgraph_test.go:1144-1349), then gossip
traces that fast-forward from a frame (run to a point, GetFrame, Reset, re-insert the frame and
keep inserting) — rounds start at the roots' rounds, the first events sit on Root.X / Root.Y,
the later ones reach other-parents through Root.Others; every output must stay bit-exact."""
import numpy as np
import pytest

import hgref
from babble_amd import trace as gtrace
from test_gpu_parity import compare

pytestmark = pytest.mark.gpu


def _hg(n, cap):
    from babble_amd.hashgraph import Hashgraph
    return Hashgraph(n, capacity=cap)


def test_fixture_frame_and_reset_from_frame():
    t = hgref.fixture_trace("consensus_hashgraph")
    o = hgref.oracle_run(t)
    h = _hg(t.n, 256)
    h.insert_trace(t)
    h.RunConsensus()
    f = h.GetFrame()
    assert f == o.get_frame()
    h.Reset(*hgref.frame_root_arrays(f), others=hgref.frame_others_keys(t, f))
    o.reset(*hgref.frame_root_arrays(f))
    sub, _ = hgref.remap_after_reset(t, f["events"], f)
    h.insert_trace(sub)
    o.insert_trace(sub)
    assert list(h.Known()) == [8, 7, 7] == list(o.known())
    h.RunConsensus()
    o.run_consensus()
    assert h.LastConsensusRound() == 1
    compare(h, o, sub, hashes=False)


def test_fixture_reset_with_explicit_roots():
    t = hgref.fixture_trace("consensus_hashgraph")
    idx = {nm: i for i, nm in enumerate(t.names)}
    h = _hg(t.n, 256)
    h.insert_trace(t)
    h.RunConsensus()
    frame = {"roots": [(idx["f02b"], idx["g1"], 4, 2), (idx["f10"], idx["f02b"], 4, 2), (idx["f21"], idx["g1"], 4, 2)],
             "others": {idx["o02"]: idx["f21"]}}
    h.Reset(*hgref.frame_root_arrays(frame), others=hgref.frame_others_keys(t, frame))
    sub, _ = hgref.remap_after_reset(t, [idx[e] for e in ("g1", "g0", "g2", "g10", "g21", "o02", "g02", "h1", "h0",
                                                            "h2")], frame)
    h.insert_trace(sub)
    assert list(h.Known()) == [8, 7, 7]
    root = h.GetRoot(0)
    assert (root["X"], root["Y"], root["Index"], root["Round"]) == (-1, hgref.ROOT_Y, 4, 2)


def test_reset_errors():
    from babble_amd._lib import HgxError
    t = hgref.fixture_trace("consensus_hashgraph")
    idx = {nm: i for i, nm in enumerate(t.names)}
    h = _hg(t.n, 256)
    frame = {"roots": [(idx["f02b"], idx["g1"], 4, 2), (idx["f10"], idx["f02b"], 4, 2), (idx["f21"], idx["g1"], 4, 2)],
             "others": {}}
    h.Reset(*hgref.frame_root_arrays(frame))
    sub, _ = hgref.remap_after_reset(t, [idx["g1"], idx["g0"], idx["g2"], idx["g10"], idx["g21"], idx["o02"]], frame)
    with pytest.raises(HgxError) as ei:   # o02's other-parent is outside the store, no Others entry
        h.insert_trace(sub)
    assert ei.value.msg == "CheckOtherParent: Other-parent not known"


def test_root_other_needs_an_others_key():
    """HGX_ROOT_OTHER is accepted only for an event whose id is a key of the roots' Others maps
    (hashgraph.go:437-440): the same insert fails at o02 without the key, and at a later event
    that claims a Root.Others parent it does not have."""
    from babble_amd._lib import HgxError
    t = hgref.fixture_trace("consensus_hashgraph")
    idx = {nm: i for i, nm in enumerate(t.names)}
    frame = {"roots": [(idx["f02b"], idx["g1"], 4, 2), (idx["f10"], idx["f02b"], 4, 2), (idx["f21"], idx["g1"], 4, 2)],
             "others": {idx["o02"]: idx["f21"]}}
    order = [idx[e] for e in ("g1", "g0", "g2", "g10", "g21", "o02", "g02", "h1", "h0", "h2")]
    sub, _ = hgref.remap_after_reset(t, order, frame)
    k_o02 = order.index(idx["o02"])
    assert sub.op[k_o02] == hgref.ROOT_OTHER
    h = _hg(t.n, 256)
    h.Reset(*hgref.frame_root_arrays(frame))          # no Others keys
    with pytest.raises(HgxError) as ei:
        h.insert_trace(sub)
    assert ei.value.msg == "CheckOtherParent: Other-parent not known" and h.num_events() == k_o02
    # a bogus claim: g02 (whose other-parent is in the store) sent with ROOT_OTHER
    k_g02 = order.index(idx["g02"])
    sub.op = sub.op.copy()
    sub.op[k_g02] = hgref.ROOT_OTHER
    h2 = _hg(t.n, 256)
    h2.Reset(*hgref.frame_root_arrays(frame), others=hgref.frame_others_keys(t, frame))
    with pytest.raises(HgxError) as ei:
        h2.insert_trace(sub)
    assert ei.value.msg == "CheckOtherParent: Other-parent not known" and h2.num_events() == k_g02


@pytest.mark.parametrize("n,E,seed,chunks", [(4, 1500, 71, 3), (16, 6000, 72, 4), (64, 20000, 73, 2),
                                             (256, 40000, 74, 2), (512, 40000, 75, 2)])
def test_gossip_fast_forward_from_frame(n, E, seed, chunks):
    t = gtrace.gossip(n, E, seed)
    K = E // 2
    o = hgref.Oracle(n)
    h = _hg(n, E)
    for lo in range(0, K, K // 2):   # two syncs before the frame
        hi = min(K, lo + K // 2)
        o.insert_trace(t, lo, hi)
        o.run_consensus()
        h.insert_trace(t, lo, hi)
        h.RunConsensus()
    f = o.get_frame()
    assert h.GetFrame() == f
    o.reset(*hgref.frame_root_arrays(f))
    h.Reset(*hgref.frame_root_arrays(f), others=hgref.frame_others_keys(t, f))
    sub, new = hgref.remap_after_reset(t, f["events"], f)
    o.insert_trace(sub)
    h.insert_trace(sub)
    o.run_consensus()
    h.RunConsensus()
    rest = list(range(K, E))
    step = (len(rest) + chunks - 1) // chunks
    parts = [sub]
    for k in range(0, len(rest), step):
        part, new = hgref.remap_after_reset(t, rest[k:k + step], f, new)
        assert (part.sp != hgref.UNKNOWN).all() and (part.op != hgref.UNKNOWN).all()
        o.insert_trace(part)
        h.insert_trace(part)
        o.run_consensus()
        h.RunConsensus()
        parts.append(part)
    r = o.results()
    assert r["last_round"] > max(x[3] for x in f["roots"]) + 2 and len(r["order"]) > 0
    compare(h, o, parts[0], hashes=False)
