"""InsertEvent with Event.Verify on the device (hgx_set_participant_keys +
hgx_insert_events_verified[_device]; hashgraph.go:356-363, event.go:142-152).

Signatures come from libcrypto (oracle/p256_ref sign, derived keys) over per-event body
digests, and the trace's S column is the signature's S, so the consensus order (whose tie
break is S, consensus_sorter.go) runs on real signatures. Checked:
  * a whole signed trace is accepted and its consensus is bit-exact with the oracle;
  * the batch stops at the first bad signature with Go's "Invalid signature", and the
    signature's failure comes before the parent checks of the same event;
  * a creator key that is not a P-256 point panics like the reference (nil key);
  * the device-resident variant, and the "keys not set" error."""
import hashlib

import numpy as np
import pytest

import hgref
from babble_amd import trace as gtrace

pytestmark = pytest.mark.gpu


def _signed(n, E, seed):
    t = gtrace.gossip(n, E, seed, stale_prob=0.1, stale_depth=2)
    dig = np.stack([np.frombuffer(hashlib.sha256(b"body %d %d" % (seed, i)).digest(), np.uint8) for i in range(t.E)])
    keys, r, s = hgref.sign_batch(n, t.creator, dig)
    t.s = s.copy()   # the trace's S is the signature's S
    return t, keys, dig, r


def _hg(n, cap):
    from babble_amd.hashgraph import Hashgraph
    return Hashgraph(n, capacity=cap)


@pytest.mark.parametrize("n,E,seed", [(4, 1500, 1), (16, 6000, 2), (64, 12000, 3)])
def test_signed_trace_accepted_and_bit_exact(n, E, seed):
    t, keys, dig, r = _signed(n, E, seed)
    h = _hg(n, t.E)
    h.set_participant_keys(keys)
    assert h.insert_verified(t, dig, r) == t.E
    h.RunConsensus()
    a, b = h.results(), hgref.oracle_run(t).results()
    for k in ("round", "witness", "famous", "rr", "cts"):
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k
    assert list(a["order"]) == list(b["order"])


def test_first_bad_signature_stops_the_batch():
    from babble_amd._lib import HgxError
    t, keys, dig, r = _signed(8, 3000, 4)
    for k0, field in ((1700, "r"), (2500, "digest"), (10, "s")):
        h = _hg(8, t.E)
        h.set_participant_keys(keys)
        rr, dd, ss = r.copy(), dig.copy(), t.s.copy()
        {"r": rr, "digest": dd, "s": ss}[field][k0, 7] ^= 0x10
        t2 = gtrace.GossipTrace(**{**t.__dict__, "s": ss})
        with pytest.raises(HgxError) as ei:
            h.insert_verified(t2, dd, rr)
        assert ei.value.msg == "Invalid signature" and ei.value.code == 104
        assert ei.value.inserted == k0 and h.num_events() == k0
        # the accepted prefix continues normally once the caller resends the good event
        assert h.insert_verified(t, dig, r, k0, t.E) == t.E - k0


def test_signature_failure_comes_before_parent_checks():
    """Event k0 has both a bad signature and an unknown other-parent, a later event a bad
    parent only: the error is "Invalid signature" at k0 (Verify runs first in InsertEvent)."""
    from babble_amd._lib import HgxError
    t, keys, dig, r = _signed(8, 2000, 5)
    k0 = 900
    op = t.op.copy()
    op[k0] = -2          # HGX_UNKNOWN_PARENT
    op[k0 + 50] = -2
    rr = r.copy()
    rr[k0, 0] ^= 1
    t2 = gtrace.GossipTrace(**{**t.__dict__, "op": op})
    h = _hg(8, t.E)
    h.set_participant_keys(keys)
    with pytest.raises(HgxError) as ei:
        h.insert_verified(t2, dig, rr)
    assert ei.value.msg == "Invalid signature" and ei.value.inserted == k0
    # good signature, bad parent: the parent check's error
    h2 = _hg(8, t.E)
    h2.set_participant_keys(keys)
    with pytest.raises(HgxError) as ei:
        h2.insert_verified(t2, dig, r)
    assert ei.value.msg == "CheckOtherParent: Other-parent not known" and ei.value.inserted == k0


def test_key_not_on_curve_panics_like_the_reference():
    from babble_amd._lib import HgxError
    t, keys, dig, r = _signed(4, 800, 6)
    bad = keys.copy()
    bad[2, 64] ^= 1          # participant 2's Body.Creator is not a curve point
    h = _hg(4, t.E)
    h.set_participant_keys(bad)
    first2 = int(np.nonzero(t.creator == 2)[0][0])
    with pytest.raises(HgxError) as ei:
        h.insert_verified(t, dig, r)
    assert ei.value.code == 300 and "nil pointer dereference" in ei.value.msg
    assert ei.value.inserted == first2


def test_device_resident_variant_and_keys_required():
    from babble_amd._lib import HgxError
    from babble_amd.hashgraph import DeviceBuffer, DeviceTrace
    t, keys, dig, r = _signed(16, 5000, 7)
    h = _hg(16, t.E)
    with pytest.raises(HgxError, match="participant keys not set"):
        h.insert_verified(t, dig, r)
    h.set_participant_keys(keys)
    dt, dd, dr = DeviceTrace(t), DeviceBuffer(dig), DeviceBuffer(r)
    assert h.insert_verified_device(dt, dd.addr, dr.addr, 0, 2500) == 2500
    assert h.insert_verified_device(dt, dd.addr, dr.addr, 2500, t.E) == t.E - 2500
    h.RunConsensus()
    b = hgref.oracle_run(t).results()
    assert list(h.ConsensusEvents()) == list(b["order"])
