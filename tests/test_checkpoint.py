"""Checkpoint file format (include/hgx.h "persistence", babble_amd/checkpoint.py) on the host:
the FNV-1a checksum's published known answers, a write/read round trip of a gossip trace,
and the rejections (corrupted byte, truncation, wrong magic). The device writer and
hgx_bootstrap are checked against the same bytes in tests/test_gpu_checkpoint.py."""
import numpy as np
import pytest

from babble_amd import checkpoint
from babble_amd import trace as gtrace


def test_fnv1a_known_answers():
    # FNV-1a 64 test vectors (Fowler/Noll/Vo reference: "" and "a", "foobar")
    assert checkpoint.fnv1a(b"") == 0xCBF29CE484222325
    assert checkpoint.fnv1a(b"a") == 0xAF63DC4C8601EC8C
    assert checkpoint.fnv1a(b"foobar") == 0x85944171F73967E8


def test_trace_round_trip(tmp_path):
    t = gtrace.gossip(8, 3000, 5, stale_prob=0.2, stale_depth=3)
    p = str(tmp_path / "t.ckpt")
    checkpoint.write_trace(p, t)
    r = checkpoint.read(p)
    assert (r["n"], r["graphs"], r["E"], r["roots"]) == (8, 1, t.E, None)
    assert np.array_equal(r["creator"], t.creator)
    assert np.array_equal(r["index"], t.index) and np.array_equal(r["self_parent"], t.sp)
    assert np.array_equal(r["other_parent"], t.op) and np.array_equal(r["timestamp_ns"], t.ts)
    assert np.array_equal(r["sig_s"], t.s) and np.array_equal(r["coin"], (t.hash[:, 16] != 0).astype(np.uint8))
    assert np.array_equal(r["ntx"], t.ntx) and np.array_equal(r["tx_nil"], t.txnil.astype(np.uint8))
    # header layout: magic, version 1, n, graphs, flags, E (little-endian)
    raw = open(p, "rb").read()
    assert raw[:8] == b"HGXCKPT1" and raw[8:12] == (1).to_bytes(4, "little")
    assert len(raw) == 32 + t.E * (4 + 8 * 4 + 32 + 1 + 4 + 1) + 8


def test_rooted_header(tmp_path):
    t = gtrace.gossip(4, 100, 6)
    data = checkpoint.encode(4, 1, t.creator, t.index, t.sp, t.op, t.ts, t.s, t.hash[:, 16], t.ntx, t.txnil,
                             roots=([3, -1, 7, 2], [1, -1, 2, 0], [1, 0, 1, 0]))
    p = tmp_path / "r.ckpt"
    p.write_bytes(data)
    r = checkpoint.read(str(p))
    ri, rr, ry = r["roots"]
    assert list(ri) == [3, -1, 7, 2] and list(rr) == [1, -1, 2, 0] and list(ry) == [1, 0, 1, 0]
    assert np.array_equal(r["creator"], t.creator)


@pytest.mark.parametrize("how", ["flip", "truncate", "magic"])
def test_rejections(tmp_path, how):
    t = gtrace.gossip(4, 200, 7)
    p = tmp_path / "b.ckpt"
    checkpoint.write_trace(str(p), t)
    raw = bytearray(p.read_bytes())
    if how == "flip":
        raw[100] ^= 1
    elif how == "truncate":
        raw = raw[:-20]
    else:
        raw[0:8] = b"NOTACKPT"
        raw[-8:] = checkpoint.fnv1a(bytes(raw[:-8])).to_bytes(8, "little")
    p.write_bytes(bytes(raw))
    with pytest.raises(ValueError):
        checkpoint.read(str(p))
