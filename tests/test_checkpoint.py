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
    assert np.array_equal(r["ids"], t.hash) and r["keys"] is None and r["payloads"] is None
    # header layout: magic, version 2, n, graphs, flags (2 = event ids), E (little-endian)
    raw = open(p, "rb").read()
    assert raw[:8] == b"HGXCKPT1" and raw[8:12] == (2).to_bytes(4, "little")
    assert raw[20:24] == (2).to_bytes(4, "little")
    assert len(raw) == 32 + t.E * (4 + 8 * 4 + 32 + 1 + 4 + 1 + 32) + 8


def test_optional_sections_round_trip(tmp_path):
    """Rooted state (roots, Root.Others keys, what Reset kept), keys and payloads."""
    t = gtrace.gossip(4, 300, 9)
    keys = np.arange(4 * 65, dtype=np.uint8).reshape(4, 65)
    pay = [b"tx%d" % i * (i % 3) for i in range(t.E)]
    others = np.arange(2 * 32, dtype=np.uint8).reshape(2, 32)
    kept = [dict(has_lcr=True, lcr=7, lcre=12, consensus_tx=99, blocks=[(3, 10, 5, 0, 1), (4, 2, 0, 1, 0)])]
    data = checkpoint.encode(4, 1, t.creator, t.index, t.sp, t.op, t.ts, t.s, t.hash[:, 16], t.ntx, t.txnil,
                             roots=([3, -1, 7, 2], [1, -1, 2, 0], [1, 0, 1, 0]), others=others, kept=kept,
                             ids=t.hash, keys=keys, payloads=pay)
    p = tmp_path / "o.ckpt"
    p.write_bytes(data)
    r = checkpoint.read(str(p))
    assert r["flags"] == 1 | 2 | 4 | 8
    assert np.array_equal(r["others"], others) and r["kept"] == kept
    assert np.array_equal(r["ids"], t.hash) and np.array_equal(r["keys"], keys) and r["payloads"] == pay


def test_version1_file_still_reads(tmp_path):
    t = gtrace.gossip(4, 100, 10)
    body = b"".join([b"HGXCKPT1", (1).to_bytes(4, "little"), np.array([4, 1, 0], "<i4").tobytes(),
                     np.array([t.E], "<i8").tobytes(), np.asarray(t.creator, "<i4").tobytes(),
                     np.asarray(t.index, "<i8").tobytes(), np.asarray(t.sp, "<i8").tobytes(),
                     np.asarray(t.op, "<i8").tobytes(), np.asarray(t.ts, "<i8").tobytes(), t.s.tobytes(),
                     (t.hash[:, 16] != 0).astype(np.uint8).tobytes(), np.asarray(t.ntx, "<i4").tobytes(),
                     t.txnil.astype(np.uint8).tobytes()])
    p = tmp_path / "v1.ckpt"
    p.write_bytes(body + np.array([checkpoint.fnv1a(body)], "<u8").tobytes())
    r = checkpoint.read(str(p))
    assert r["version"] == 1 and r["ids"] is None and np.array_equal(r["creator"], t.creator)


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


@pytest.mark.parametrize("bad", ["decrease", "nonzero_start"])
def test_payload_offsets_rejected(tmp_path, bad):
    """Payload offsets that do not start at 0 or decrease: libhgx's hgx_bootstrap rejects the file
    ("payload offsets decrease"), and so does the host reader."""
    t = gtrace.gossip(4, 50, 12)
    pay = [b"p%d" % i for i in range(t.E)]
    data = bytearray(checkpoint.encode(4, 1, t.creator, t.index, t.sp, t.op, t.ts, t.s, t.hash[:, 16], t.ntx,
                                       t.txnil, payloads=pay))
    # the offsets section is the last E + 1 int64 before the blob and the checksum
    blob = sum(len(x) for x in pay)
    at = len(data) - 8 - blob - 8 * (t.E + 1)
    off = np.frombuffer(bytes(data[at:at + 8 * (t.E + 1)]), "<i8").copy()
    assert off[0] == 0 and off[-1] == blob
    if bad == "decrease":
        off[5], off[6] = off[6], off[5]
    else:
        off[0] = 1
    data[at:at + 8 * (t.E + 1)] = off.tobytes()
    data[-8:] = checkpoint.fnv1a(bytes(data[:-8])).to_bytes(8, "little")
    p = tmp_path / "p.ckpt"
    p.write_bytes(bytes(data))
    with pytest.raises(ValueError):
        checkpoint.read(str(p))
