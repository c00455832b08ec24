"""Checkpoint files of the resident event DAG (include/hgx.h, "persistence").

The reference persists its DAG in the BadgerStore as an event log keyed by topological index
(badger_store.go:103-125, 309-343) and Hashgraph.Bootstrap replays that log through
InsertEvent before running consensus once (hashgraph.go:1008-1037, dbTopologicalEvents
badger_store.go:345-386). Here the log is one binary structure-of-arrays file; libhgx writes
it (hgx_save) and replays it (hgx_bootstrap). This module reads and writes the same format on
the host, so a synthetic trace can be written as a checkpoint and bootstrapped, and a file
written by the device can be inspected. Little-endian layout:

    "HGXCKPT1" | u32 version | i32 n | i32 graphs | i32 flags (1 = rooted) | i64 E
    | rooted: i32 root_index[C] | i32 root_round[C] | u8 root_y_is_event[C] (zero pad to 4)
    | i32 creator[E] | i64 index[E] | i64 self_parent[E] | i64 other_parent[E]
    | i64 timestamp_ns[E] | u8 sig_s[E][32] | u8 coin[E] | i32 ntx[E] | u8 tx_nil[E]
    | u64 FNV-1a over every preceding byte
"""
from __future__ import annotations

from typing import Optional

import numpy as np

MAGIC = b"HGXCKPT1"
VERSION = 1


def fnv1a(data: bytes) -> int:
    """64-bit FNV-1a of the bytes (the file's checksum), computed by libhgx (hgx_checksum; a
    host function, no device needed)."""
    from . import _lib
    L = _lib.lib()
    b = np.frombuffer(data, np.uint8)
    return int(L.hgx_checksum(_lib.ptr(b), b.size))


def encode(n: int, graphs: int, creator, index, sp, op, ts, sig_s, coin, ntx, tx_nil,
           roots: Optional[tuple] = None) -> bytes:
    """The file bytes for E events (gid order). roots = (root_index, root_round, root_y_is_event)
    of a context after a Reset, else None."""
    E = len(creator)
    C = n * graphs
    parts = [MAGIC, np.array([VERSION], "<u4").tobytes(),
             np.array([n, graphs, 1 if roots is not None else 0], "<i4").tobytes(), np.array([E], "<i8").tobytes()]
    if roots is not None:
        ri, rr, ry = roots
        y = np.zeros((C + 3) & ~3, np.uint8)
        y[:C] = np.asarray(ry, np.uint8)
        parts += [np.asarray(ri, "<i4").tobytes(), np.asarray(rr, "<i4").tobytes(), y.tobytes()]
    parts += [np.asarray(creator, "<i4").tobytes(), np.asarray(index, "<i8").tobytes(),
              np.asarray(sp, "<i8").tobytes(), np.asarray(op, "<i8").tobytes(), np.asarray(ts, "<i8").tobytes(),
              np.ascontiguousarray(np.asarray(sig_s, np.uint8).reshape(E, 32)).tobytes(),
              (np.asarray(coin) != 0).astype(np.uint8).tobytes(), np.asarray(ntx, "<i4").tobytes(),
              (np.asarray(tx_nil) != 0).astype(np.uint8).tobytes()]
    body = b"".join(parts)
    return body + np.array([fnv1a(body)], "<u8").tobytes()


def write_trace(path: str, t, graphs: int = 1) -> None:
    """A synthetic trace (babble_amd.trace.GossipTrace; n = participants per graph) as a checkpoint:
    the coin is the event hash's byte 16 (middleBit, hashgraph.go:1039-1048)."""
    data = encode(t.n, graphs, t.creator, t.index, t.sp, t.op, t.ts, t.s, t.hash[:, 16] != 0, t.ntx, t.txnil)
    with open(path, "wb") as f:
        f.write(data)


def read(path: str) -> dict:
    """Parse and verify a checkpoint file (ValueError on a bad magic, version, size or checksum)."""
    with open(path, "rb") as f:
        buf = f.read()
    if len(buf) < 40:
        raise ValueError("truncated file")
    if fnv1a(buf[:-8]) != int(np.frombuffer(buf[-8:], "<u8")[0]):
        raise ValueError("checksum mismatch")
    if buf[:8] != MAGIC:
        raise ValueError("not a checkpoint file")
    version = int(np.frombuffer(buf, "<u4", 1, 8)[0])
    if version != VERSION:
        raise ValueError(f"unsupported version {version}")
    n, graphs, flags = (int(x) for x in np.frombuffer(buf, "<i4", 3, 12))
    E = int(np.frombuffer(buf, "<i8", 1, 24)[0])
    C = n * graphs
    pos = 32
    out = {"n": n, "graphs": graphs, "E": E, "roots": None}

    def take(dtype, count, shape=None):
        nonlocal pos
        a = np.frombuffer(buf, dtype, count, pos)
        pos += a.nbytes
        return a.reshape(shape) if shape else a

    if flags & 1:
        ri, rr = take("<i4", C), take("<i4", C)
        y = take(np.uint8, (C + 3) & ~3)[:C]
        out["roots"] = (ri, rr, y)
    for name, dt, cnt, shp in (("creator", "<i4", E, None), ("index", "<i8", E, None), ("self_parent", "<i8", E, None),
                               ("other_parent", "<i8", E, None), ("timestamp_ns", "<i8", E, None),
                               ("sig_s", np.uint8, 32 * E, (E, 32)), ("coin", np.uint8, E, None),
                               ("ntx", "<i4", E, None), ("tx_nil", np.uint8, E, None)):
        out[name] = take(dt, cnt, shp)
    if pos != len(buf) - 8:
        raise ValueError("size mismatch")
    return out
