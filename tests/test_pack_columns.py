"""hgx_pack_events32 (include/hgx.h), the host helper that builds hgx_events_packed's 10-byte
structure columns: decoding them as the device does (k_unpack_packed + k_unpack_exc,
babble_amd/csrc/hgx_insert.hip) gives back the hgx_events32 columns exactly. Host only."""
import numpy as np
import pytest

from babble_amd import trace as gtrace


def _decode(pk, base):
    m = len(pk["creator16"])
    g = base + np.arange(m, dtype=np.int64)

    def par(b):
        b = b.astype(np.int64)
        return np.where(b == 0, -1, np.where(b == 0xFFFF, -2, g - b)).astype(np.int32)

    sp, op = par(pk["sp_back"]), par(pk["op_back"])
    sp[pk["exc_pos"]] = pk["exc_sp"]
    op[pk["exc_pos"]] = pk["exc_op"]
    return pk["creator16"].astype(np.int32), sp, op


@pytest.mark.parametrize("base", [0, 12345, 70000])
def test_pack_round_trip(base):
    from babble_amd.hashgraph import compact_columns, pack_columns
    cols = compact_columns(gtrace.gossip(16, 5000, 3, stale_prob=0.2, stale_depth=3))
    cols["sp"] = np.where(cols["sp"] >= 0, cols["sp"] + base, cols["sp"]).astype(np.int32)
    cols["op"] = np.where(cols["op"] >= 0, cols["op"] + base, cols["op"]).astype(np.int32)
    # the forms the distance cannot hold: unknown, Root.Y, far back, forward
    cols["op"][100], cols["op"][200], cols["sp"][300] = -2, -3, base + 4000
    cols["op"][4999] = max(0, base + 4999 - 70000) if base else -2
    pk = pack_columns(cols, base)
    cr, sp, op = _decode(pk, base)
    assert np.array_equal(cr, cols["creator"]) and np.array_equal(sp, cols["sp"]) and np.array_equal(op, cols["op"])
    assert {100, 200, 300} <= set(pk["exc_pos"].tolist())
    assert pk["creator16"].dtype == np.uint16 and pk["sp_back"].dtype == np.uint16


def test_pack_refusals():
    from babble_amd import _lib
    from babble_amd.hashgraph import compact_columns, pack_columns
    cols = compact_columns(gtrace.gossip(4, 300, 4))
    cols["creator"][7] = 70000
    with pytest.raises(_lib.HgxError) as ei:
        pack_columns(cols, 0)
    assert "creator outside" in ei.value.msg
    cols = compact_columns(gtrace.gossip(4, 300, 4))
    cols["op"][:] = -2   # every event escaped: the list grows until it fits
    pk = pack_columns(cols, 0)
    assert len(pk["exc_pos"]) == 300
