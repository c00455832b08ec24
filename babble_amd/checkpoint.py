"""Checkpoint files of the resident event DAG (include/hgx.h, "persistence").

The reference persists its DAG in the BadgerStore: events keyed by topological index with their
bodies and signatures, the participants, the roots and the blocks (badger_store.go:103-125,
309-343, 540); Hashgraph.Bootstrap replays the events through InsertEvent before running
consensus once (hashgraph.go:1008-1037, dbTopologicalEvents badger_store.go:345-386). Here the log
is one binary structure-of-arrays file; libhgx writes it (hgx_save / hgx_save_ex) and replays it
(hgx_bootstrap). This module reads and writes the same format on the host, so a synthetic trace
can be written as a checkpoint and bootstrapped, and a file written by the device can be
inspected. Little-endian layout (version 2; version 1 = no optional sections and flags <= 1):

    "HGXCKPT1" | u32 version | i32 n | i32 graphs | i32 flags | i64 E
        flags: 1 rooted, 2 event ids, 4 participant keys, 8 payloads
    | rooted: i32 root_index[C] | i32 root_round[C] | u8 root_y_is_event[C] (zero pad to 4)
        | i64 n_others | u8 others[n_others][32]
        | per graph: i32 has_lcr, i32 lcr, i32 lcre, i32 0, i64 consensus_tx, i64 n_blocks,
          n_blocks x (i32 rr, i32 events, i64 transactions, i32 nil, i32 committed)
    | i32 creator[E] | i64 index[E] | i64 self_parent[E] | i64 other_parent[E]
    | i64 timestamp_ns[E] | u8 sig_s[E][32] | u8 coin[E] | i32 ntx[E] | u8 tx_nil[E]
    | ids u8[E][32] | keys u8[C][65] | payloads: i64 off[E+1], u8 bytes[off[E]]
    | u64 FNV-1a over every preceding byte
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np

MAGIC = b"HGXCKPT1"
VERSION = 2
ROOTED, IDS, KEYS, PAYLOADS = 1, 2, 4, 8


def fnv1a(data: bytes) -> int:
    """64-bit FNV-1a of the bytes (the file's checksum), computed by libhgx (hgx_checksum; a
    host function, no device needed)."""
    from . import _lib
    L = _lib.lib()
    b = np.frombuffer(data, np.uint8)
    return int(L.hgx_checksum(_lib.ptr(b), b.size))


def encode(n: int, graphs: int, creator, index, sp, op, ts, sig_s, coin, ntx, tx_nil,
           roots: Optional[tuple] = None, others=None, kept: Optional[Sequence[dict]] = None,
           ids=None, keys=None, payloads: Optional[Sequence[bytes]] = None) -> bytes:
    """The file bytes for E events (gid order). roots = (root_index, root_round, root_y_is_event)
    of a context after a Reset (with its Root.Others keys and, per graph, what Reset kept:
    dict(has_lcr, lcr, lcre, consensus_tx, blocks=[(rr, events, transactions, nil, committed)]));
    ids = the events' 32-byte ids, keys = the participants' 65-byte keys, payloads = per-event bytes."""
    E = len(creator)
    C = n * graphs
    flags = (ROOTED if roots is not None else 0) | (IDS if ids is not None else 0) | \
        (KEYS if keys is not None else 0) | (PAYLOADS if payloads is not None else 0)
    parts = [MAGIC, np.array([VERSION], "<u4").tobytes(),
             np.array([n, graphs, flags], "<i4").tobytes(), np.array([E], "<i8").tobytes()]
    if roots is not None:
        ri, rr, ry = roots
        y = np.zeros((C + 3) & ~3, np.uint8)
        y[:C] = np.asarray(ry, np.uint8)
        ok = np.zeros((0, 32), np.uint8) if others is None else np.asarray(others, np.uint8).reshape(-1, 32)
        parts += [np.asarray(ri, "<i4").tobytes(), np.asarray(rr, "<i4").tobytes(), y.tobytes(),
                  np.array([ok.shape[0]], "<i8").tobytes(), ok.tobytes()]
        for g in range(graphs):
            k = (kept or [{}] * graphs)[g]
            blocks = k.get("blocks", [])
            parts += [np.array([1 if k.get("has_lcr") else 0, k.get("lcr", 0), k.get("lcre", 0), 0], "<i4").tobytes(),
                      np.array([k.get("consensus_tx", 0), len(blocks)], "<i8").tobytes()]
            for rr_, nev, ntx_, nil_, com in blocks:
                parts += [np.array([rr_, nev], "<i4").tobytes(), np.array([ntx_], "<i8").tobytes(),
                          np.array([nil_, com], "<i4").tobytes()]
    parts += [np.asarray(creator, "<i4").tobytes(), np.asarray(index, "<i8").tobytes(),
              np.asarray(sp, "<i8").tobytes(), np.asarray(op, "<i8").tobytes(), np.asarray(ts, "<i8").tobytes(),
              np.ascontiguousarray(np.asarray(sig_s, np.uint8).reshape(E, 32)).tobytes(),
              (np.asarray(coin) != 0).astype(np.uint8).tobytes(), np.asarray(ntx, "<i4").tobytes(),
              (np.asarray(tx_nil) != 0).astype(np.uint8).tobytes()]
    if ids is not None:
        parts.append(np.ascontiguousarray(np.asarray(ids, np.uint8).reshape(E, 32)).tobytes())
    if keys is not None:
        parts.append(np.ascontiguousarray(np.asarray(keys, np.uint8).reshape(C, 65)).tobytes())
    if payloads is not None:
        off = np.zeros(E + 1, "<i8")
        off[1:] = np.cumsum([len(b) for b in payloads]) if E else []
        parts += [off.tobytes(), b"".join(payloads)]
    body = b"".join(parts)
    return body + np.array([fnv1a(body)], "<u8").tobytes()


def write_trace(path: str, t, graphs: int = 1, with_ids: bool = True) -> None:
    """A synthetic trace (babble_amd.trace.GossipTrace; n = participants per graph) as a checkpoint
    (with its event ids unless with_ids=False): the coin is the id's byte 16 (middleBit,
    hashgraph.go:1039-1048)."""
    data = encode(t.n, graphs, t.creator, t.index, t.sp, t.op, t.ts, t.s, t.hash[:, 16] != 0, t.ntx, t.txnil,
                  ids=t.hash if with_ids else None)
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
    if version not in (1, 2):
        raise ValueError(f"unsupported version {version}")
    n, graphs, flags = (int(x) for x in np.frombuffer(buf, "<i4", 3, 12))
    if version == 1 and flags & ~ROOTED:
        raise ValueError("unsupported flags")
    E = int(np.frombuffer(buf, "<i8", 1, 24)[0])
    C = n * graphs
    pos = 32
    end = len(buf) - 8
    out = {"n": n, "graphs": graphs, "E": E, "version": version, "flags": flags, "roots": None, "others": None,
           "kept": None, "ids": None, "keys": None, "payloads": None}

    def take(dtype, count, shape=None):
        nonlocal pos
        a = np.frombuffer(buf, dtype, count, pos)
        pos += a.nbytes
        if pos > end:
            raise ValueError("truncated file")
        return a.reshape(shape) if shape else a

    try:
        if flags & ROOTED:
            ri, rr = take("<i4", C), take("<i4", C)
            y = take(np.uint8, (C + 3) & ~3)[:C]
            out["roots"] = (ri, rr, y)
            if version >= 2:
                no = int(take("<i8", 1)[0])
                out["others"] = take(np.uint8, 32 * no, (no, 32))
                kept = []
                for _ in range(graphs):
                    h4 = take("<i4", 4)
                    c2 = take("<i8", 2)
                    blocks = []
                    for _ in range(int(c2[1])):
                        a = take("<i4", 2)
                        t = take("<i8", 1)
                        b = take("<i4", 2)
                        blocks.append((int(a[0]), int(a[1]), int(t[0]), int(b[0]), int(b[1])))
                    kept.append(dict(has_lcr=bool(h4[0]), lcr=int(h4[1]), lcre=int(h4[2]),
                                     consensus_tx=int(c2[0]), blocks=blocks))
                out["kept"] = kept
        for name, dt, cnt, shp in (("creator", "<i4", E, None), ("index", "<i8", E, None),
                                   ("self_parent", "<i8", E, None), ("other_parent", "<i8", E, None),
                                   ("timestamp_ns", "<i8", E, None), ("sig_s", np.uint8, 32 * E, (E, 32)),
                                   ("coin", np.uint8, E, None), ("ntx", "<i4", E, None), ("tx_nil", np.uint8, E, None)):
            out[name] = take(dt, cnt, shp)
        if flags & IDS:
            out["ids"] = take(np.uint8, 32 * E, (E, 32))
        if flags & KEYS:
            out["keys"] = take(np.uint8, 65 * C, (C, 65))
        if flags & PAYLOADS:
            off = take("<i8", E + 1)
            if E >= 0 and (off[0] != 0 or np.any(np.diff(off) < 0)):
                raise ValueError("payload offsets decrease")   # (libhgx rejects the same file)
            blob = take(np.uint8, int(off[-1]) if E >= 0 else 0).tobytes()
            out["payloads"] = [blob[off[i]:off[i + 1]] for i in range(E)]
    except ValueError:
        raise
    except Exception as e:  # numpy out-of-range reads
        raise ValueError("truncated file") from e
    if pos != end:
        raise ValueError("size mismatch")
    return out
