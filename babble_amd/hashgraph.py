"""Python mirror of the reference's hashgraph.Hashgraph API over libhgx's C ABI.

Reference: datatypevoid/babble v0.2.0 hashgraph/hashgraph.go. Method names follow
the Go API (InsertEvent, DivideRounds, DecideFame, FindOrder, Round, Witness,
StronglySee, ...) with the same argument meaning and the same error strings
(raised as babble_amd._lib.HgxError). Events are addressed by dense ids (gid, in
insertion order) -- the cgo shim described in INTEGRATION.md maps Go hex ids to
these. All computation happens in the HIP kernels of libhgx.so; this module only
marshals arrays.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import HgxError, hgx_error, hgx_events, ptr

UNKNOWN_PARENT = -2


def compact_columns(t) -> dict:
    """hgx_events32 columns of a trace (include/hgx.h): int32 Index and parents, the coin byte
    (middleBit: byte 16 of the event id is not 0, hashgraph.go:1039-1048) instead of the id, and
    len(Transactions) with -1 for nil. What a caller builds instead of the wide columns."""
    ntx = np.where(np.asarray(t.txnil) != 0, -1, np.asarray(t.ntx)).astype(np.int32)
    return dict(creator=np.ascontiguousarray(t.creator, np.int32), index=np.ascontiguousarray(t.index, np.int32),
                sp=np.ascontiguousarray(t.sp, np.int32), op=np.ascontiguousarray(t.op, np.int32),
                ts=np.ascontiguousarray(t.ts, np.int64),
                coin=np.ascontiguousarray(np.asarray(t.hash)[:, 16] != 0, np.uint8),
                s=np.ascontiguousarray(t.s, np.uint8), ntx=ntx)


class HostBuffer:
    """One page-locked host allocation (hgx_host_alloc), freed with the object. `.array` is a numpy
    view over it; the caller keeps the HostBuffer alive while the view is in use."""

    def __init__(self, shape, dtype):
        dt = np.dtype(dtype)
        nbytes = max(1, int(np.prod(shape)) * dt.itemsize)
        self._L = _lib.lib()
        self.p = self._L.hgx_host_alloc(nbytes)
        if not self.p:
            raise MemoryError(f"hgx_host_alloc({nbytes}) failed")
        raw = (C.c_uint8 * nbytes).from_address(self.p)
        self.array = np.frombuffer(raw, dtype=np.uint8)[:int(np.prod(shape)) * dt.itemsize].view(dt).reshape(shape)

    def __del__(self):
        p, self.p = getattr(self, "p", None), None
        if p:
            self.array = None
            self._L.hgx_host_free(p)


def pinned_columns(cols: dict) -> dict:
    """The same columns copied into page-locked host memory (hgx_host_alloc), as a caller that keeps
    its sync buffers there hands them over. The returned dict holds the buffers under "_buffers"."""
    out, bufs = {}, []
    for k, v in cols.items():
        if isinstance(v, np.ndarray):
            b = HostBuffer(v.shape, v.dtype)
            b.array[...] = v
            bufs.append(b)
            out[k] = b.array
        else:
            out[k] = v
    out["_buffers"] = bufs
    return out


def pack_columns(cols: dict, base: int) -> dict:
    """hgx_events_packed columns (include/hgx.h) of compact_columns() whose first event gets gid
    `base` (hgx_num_events of the context it goes into): creator as u16, each parent as its
    distance back (0 = "", 0xFFFF = the exception list), built by libhgx's hgx_pack_events32. The
    payload columns are shared with `cols`."""
    L = _lib.lib()
    m = len(cols["creator"])
    _, ev = _events32_of(cols, 0, m)
    out = dict(creator16=np.empty(m, np.uint16), sp_back=np.empty(m, np.uint16), op_back=np.empty(m, np.uint16))
    cap = max(16, m // 64)
    while True:
        x = dict(exc_pos=np.empty(cap, np.int64), exc_sp=np.empty(cap, np.int32), exc_op=np.empty(cap, np.int32))
        n_exc = C.c_int64(0)
        err = hgx_error()
        rc = L.hgx_pack_events32(C.byref(ev), m, base, ptr(out["creator16"]), ptr(out["sp_back"]),
                                 ptr(out["op_back"]), ptr(x["exc_pos"]), ptr(x["exc_sp"]), ptr(x["exc_op"]), cap,
                                 C.byref(n_exc), C.byref(err))
        if rc == 0:
            break
        if n_exc.value <= cap:
            _lib.check(rc, err)
        cap = n_exc.value
    k = n_exc.value
    out.update({nm: np.ascontiguousarray(v[:k]) for nm, v in x.items()})
    out.update(index=cols["index"], ts=cols["ts"], coin=cols["coin"], s=cols["s"], ntx=cols["ntx"])
    return out


def _events32_of(cols: dict, lo: int, hi: int):
    a = {k: v[lo:hi] for k, v in cols.items()}
    return a, _lib.hgx_events32(*[ptr(a[k]) for k in ("creator", "index", "sp", "op", "ts", "coin", "s", "ntx")])


class Hashgraph:
    """One context = NewHashgraph(participants, NewInmemStore(participants, cap)) (hashgraph.go:39-66).

    n_graphs > 1 makes a batched context of independent hashgraphs (graph g owns
    participant ids g*n .. g*n+n-1); per-graph getters take `graph`.
    """

    def __init__(self, n_participants: int, capacity: int = 1 << 16, device: int = 0, n_graphs: int = 1,
                 shard_devices: Optional[Sequence[int]] = None):
        """shard_devices: one graph whose round recurrence is chain-sharded over these devices
        (hgx_create_sharded; shard 0 on shard_devices[0], ordinals may repeat)."""
        self.L = _lib.lib()
        self.n = n_participants
        self.G = n_graphs
        err = hgx_error()
        if shard_devices is not None:
            if n_graphs != 1:
                raise ValueError("a chain-sharded context holds one graph")
            devs = np.ascontiguousarray(list(shard_devices), np.int32)
            self.ctx = self.L.hgx_create_sharded(n_participants, capacity, len(devs), ptr(devs), C.byref(err))
        else:
            self.ctx = self.L.hgx_create_batch(n_graphs, n_participants, capacity, device, C.byref(err))
        if not self.ctx:
            raise HgxError(err.code, err.msg.decode(errors="replace"))
        self.capacity = capacity

    def close(self):
        if getattr(self, "ctx", None):
            self.L.hgx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ inserts
    def insert_arrays(self, creator, index, sp, op, ts, hash32, s32, ntx, txnil) -> int:
        """Bulk InsertEvent(e, true) in order; raises HgxError on the first rejected event."""
        a = dict(creator=np.ascontiguousarray(creator, np.int32), index=np.ascontiguousarray(index, np.int64),
                 sp=np.ascontiguousarray(sp, np.int64), op=np.ascontiguousarray(op, np.int64),
                 ts=np.ascontiguousarray(ts, np.int64), h=np.ascontiguousarray(hash32, np.uint8),
                 s=np.ascontiguousarray(s32, np.uint8), ntx=np.ascontiguousarray(ntx, np.int32),
                 nil=np.ascontiguousarray(txnil, np.int32))
        cnt = int(a["creator"].shape[0])
        ev = hgx_events(ptr(a["creator"]), ptr(a["index"]), ptr(a["sp"]), ptr(a["op"]), ptr(a["ts"]),
                        ptr(a["h"]), ptr(a["s"]), ptr(a["ntx"]), ptr(a["nil"]))
        err = hgx_error()
        n_ins = C.c_int64(0)
        rc = self.L.hgx_insert_events(self.ctx, C.byref(ev), cnt, C.byref(n_ins), C.byref(err))
        _lib.check(rc, err)
        return n_ins.value

    def set_participant_keys(self, keys65):
        """Participants' public keys (C x 65 bytes, participant id order) for Event.Verify."""
        k = np.ascontiguousarray(keys65, np.uint8).reshape(-1, 65)
        self._call(lambda ctx, e: self.L.hgx_set_participant_keys(ctx, ptr(k), e))

    def insert_verified(self, t, digest32, r32, lo: int = 0, hi: Optional[int] = None) -> int:
        """InsertEvent with Event.Verify (hgx_insert_events_verified): events [lo, hi) of a trace,
        their body digests and signature R (S = the trace's S column). Raises HgxError on the first
        rejected event, with .inserted = events inserted before it."""
        hi = t.E if hi is None else hi
        sl = slice(lo, hi)
        a = dict(creator=np.ascontiguousarray(t.creator[sl], np.int32), index=np.ascontiguousarray(t.index[sl], np.int64),
                 sp=np.ascontiguousarray(t.sp[sl], np.int64), op=np.ascontiguousarray(t.op[sl], np.int64),
                 ts=np.ascontiguousarray(t.ts[sl], np.int64), h=np.ascontiguousarray(t.hash[sl], np.uint8),
                 s=np.ascontiguousarray(t.s[sl], np.uint8), ntx=np.ascontiguousarray(t.ntx[sl], np.int32),
                 nil=np.ascontiguousarray(t.txnil[sl], np.int32),
                 d=np.ascontiguousarray(np.asarray(digest32)[sl], np.uint8),
                 r=np.ascontiguousarray(np.asarray(r32)[sl], np.uint8))
        ev = hgx_events(ptr(a["creator"]), ptr(a["index"]), ptr(a["sp"]), ptr(a["op"]), ptr(a["ts"]),
                        ptr(a["h"]), ptr(a["s"]), ptr(a["ntx"]), ptr(a["nil"]))
        err = hgx_error()
        n_ins = C.c_int64(0)
        rc = self.L.hgx_insert_events_verified(self.ctx, C.byref(ev), ptr(a["d"]), ptr(a["r"]), hi - lo,
                                               C.byref(n_ins), C.byref(err))
        if rc:
            e = HgxError(int(err.code or rc), err.msg.decode(errors="replace"))
            e.inserted = n_ins.value
            raise e
        return n_ins.value

    def insert_verified_device(self, dt: "DeviceTrace", d_digest, d_r, lo: int = 0, hi: Optional[int] = None) -> int:
        """The same with every column resident in HBM (d_digest / d_r: device addresses of 32-byte rows)."""
        hi = dt.E if hi is None else hi
        ev = dt.events(lo, hi)
        err = hgx_error()
        n_ins = C.c_int64(0)
        rc = self.L.hgx_insert_events_verified_device(self.ctx, C.byref(ev), C.c_void_p(int(d_digest) + 32 * lo),
                                                      C.c_void_p(int(d_r) + 32 * lo), hi - lo, C.byref(n_ins),
                                                      C.byref(err))
        if rc:
            e = HgxError(int(err.code or rc), err.msg.decode(errors="replace"))
            e.inserted = n_ins.value
            raise e
        return n_ins.value

    def insert_wire(self, creator_id, index, sp_index, op_creator, op_index, ts, hash32, s32, ntx, txnil) -> int:
        """Core.Sync's loop over WireEvents (hgx_insert_wire_events): ReadWireInfo + InsertEvent(e, false)
        per event; on the first error raises HgxError with .inserted = events inserted before it."""
        a = [np.ascontiguousarray(creator_id, np.int32), np.ascontiguousarray(index, np.int64),
             np.ascontiguousarray(sp_index, np.int64), np.ascontiguousarray(op_creator, np.int32),
             np.ascontiguousarray(op_index, np.int64), np.ascontiguousarray(ts, np.int64),
             np.ascontiguousarray(hash32, np.uint8), np.ascontiguousarray(s32, np.uint8),
             np.ascontiguousarray(ntx, np.int32), np.ascontiguousarray(txnil, np.int32)]
        ev = _lib.hgx_wire_events(*[ptr(x) for x in a])
        err = hgx_error()
        n_ins = C.c_int64(0)
        rc = self.L.hgx_insert_wire_events(self.ctx, C.byref(ev), int(a[0].shape[0]), C.byref(n_ins), C.byref(err))
        if rc:
            e = HgxError(rc, err.msg.decode(errors="replace"))
            e.inserted = n_ins.value
            raise e
        return n_ins.value

    def insert_device(self, dt: "DeviceTrace", lo: int = 0, hi: Optional[int] = None) -> int:
        """Bulk InsertEvent of a trace already resident in HBM (hgx_insert_events_device)."""
        hi = dt.E if hi is None else hi
        ev = dt.events(lo, hi)
        err = hgx_error()
        n_ins = C.c_int64(0)
        rc = self.L.hgx_insert_events_device(self.ctx, C.byref(ev), hi - lo, C.byref(n_ins), C.byref(err))
        _lib.check(rc, err)
        return n_ins.value

    def clear(self):
        """Forget every event: a fresh NewHashgraph (device allocations kept)."""
        rc = self.L.hgx_clear(self.ctx)
        if rc:
            raise HgxError(rc, "hgx_clear failed")

    def insert_trace(self, t, lo: int = 0, hi: Optional[int] = None) -> int:
        hi = t.E if hi is None else hi
        sl = slice(lo, hi)
        return self.insert_arrays(t.creator[sl], t.index[sl], t.sp[sl], t.op[sl], t.ts[sl], t.hash[sl], t.s[sl],
                                  t.ntx[sl], t.txnil[sl])

    def insert_and_run(self, t, lo: int = 0, hi: Optional[int] = None) -> int:
        """Bootstrap / Core.Sync + RunConsensus in one call (hgx_insert_and_run): events [lo, hi) of a
        trace inserted, then DivideRounds / DecideFame / FindOrder, the payload columns copied to HBM
        while DivideRounds runs. Raises HgxError like insert_trace (.inserted = the accepted prefix)."""
        hi = t.E if hi is None else hi
        sl = slice(lo, hi)
        a = dict(creator=np.ascontiguousarray(t.creator[sl], np.int32), index=np.ascontiguousarray(t.index[sl], np.int64),
                 sp=np.ascontiguousarray(t.sp[sl], np.int64), op=np.ascontiguousarray(t.op[sl], np.int64),
                 ts=np.ascontiguousarray(t.ts[sl], np.int64), h=np.ascontiguousarray(t.hash[sl], np.uint8),
                 s=np.ascontiguousarray(t.s[sl], np.uint8), ntx=np.ascontiguousarray(t.ntx[sl], np.int32),
                 nil=np.ascontiguousarray(t.txnil[sl], np.int32))
        ev = hgx_events(ptr(a["creator"]), ptr(a["index"]), ptr(a["sp"]), ptr(a["op"]), ptr(a["ts"]),
                        ptr(a["h"]), ptr(a["s"]), ptr(a["ntx"]), ptr(a["nil"]))
        err = hgx_error()
        n_ins = C.c_int64(0)
        self._cb_error = None
        rc = self.L.hgx_insert_and_run(self.ctx, C.byref(ev), hi - lo, C.byref(n_ins), C.byref(err))
        if rc:
            e = HgxError(int(err.code or rc), err.msg.decode(errors="replace"))
            e.inserted = n_ins.value
            raise e
        cb_err, self._cb_error = getattr(self, "_cb_error", None), None
        if cb_err is not None:
            raise cb_err
        return n_ins.value

    def _events32(self, cols: dict, lo: int, hi: int):
        return _events32_of(cols, lo, hi)

    def insert_events32(self, cols: dict, lo: int = 0, hi: Optional[int] = None) -> int:
        """InsertEvent from the compact columns of compact_columns() (hgx_insert_events32)."""
        hi = len(cols["creator"]) if hi is None else hi
        a, ev = self._events32(cols, lo, hi)
        err = hgx_error()
        n_ins = C.c_int64(0)
        rc = self.L.hgx_insert_events32(self.ctx, C.byref(ev), hi - lo, C.byref(n_ins), C.byref(err))
        if rc:
            e = HgxError(int(err.code or rc), err.msg.decode(errors="replace"))
            e.inserted = n_ins.value
            raise e
        return n_ins.value

    def insert_and_run32(self, cols: dict, lo: int = 0, hi: Optional[int] = None) -> int:
        """insert_and_run from the compact columns (hgx_insert_and_run32: 61 bytes per event)."""
        hi = len(cols["creator"]) if hi is None else hi
        a, ev = self._events32(cols, lo, hi)
        err = hgx_error()
        n_ins = C.c_int64(0)
        self._cb_error = None
        rc = self.L.hgx_insert_and_run32(self.ctx, C.byref(ev), hi - lo, C.byref(n_ins), C.byref(err))
        if rc:
            e = HgxError(int(err.code or rc), err.msg.decode(errors="replace"))
            e.inserted = n_ins.value
            raise e
        cb_err, self._cb_error = getattr(self, "_cb_error", None), None
        if cb_err is not None:
            raise cb_err
        return n_ins.value

    def _packed_call(self, fn, pk: dict) -> int:
        m = len(pk["creator16"])
        ev = _lib.hgx_events_packed(ptr(pk["creator16"]), ptr(pk["index"]), ptr(pk["sp_back"]), ptr(pk["op_back"]),
                                    len(pk["exc_pos"]), ptr(pk["exc_pos"]), ptr(pk["exc_sp"]), ptr(pk["exc_op"]),
                                    ptr(pk["ts"]), ptr(pk["coin"]), ptr(pk["s"]), ptr(pk["ntx"]))
        err = hgx_error()
        n_ins = C.c_int64(0)
        self._cb_error = None
        rc = fn(self.ctx, C.byref(ev), m, C.byref(n_ins), C.byref(err))
        if rc:
            e = HgxError(int(err.code or rc), err.msg.decode(errors="replace"))
            e.inserted = n_ins.value
            raise e
        cb_err, self._cb_error = getattr(self, "_cb_error", None), None
        if cb_err is not None:
            raise cb_err
        return n_ins.value

    def insert_events_packed(self, pk: dict) -> int:
        """InsertEvent from pack_columns() output (hgx_insert_events_packed); its base must be
        num_events() now."""
        return self._packed_call(self.L.hgx_insert_events_packed, pk)

    def insert_and_run_packed(self, pk: dict) -> int:
        """insert_and_run from pack_columns() output (hgx_insert_and_run_packed: 10-byte structure
        columns + the 45-byte compact payload)."""
        return self._packed_call(self.L.hgx_insert_and_run_packed, pk)

    def InsertEvent(self, creator: int, index: int, self_parent: int, other_parent: int, timestamp_ns: int,
                    hash32: bytes, s32: bytes, transactions: Optional[Sequence[bytes]]):
        """InsertEvent(event, true) (hashgraph.go:356-401): raises HgxError with the Go error string."""
        txs = [] if transactions is None else list(transactions)
        self.insert_arrays([creator], [index], [self_parent], [other_parent], [timestamp_ns],
                           np.frombuffer(hash32, np.uint8).reshape(1, 32), np.frombuffer(s32, np.uint8).reshape(1, 32),
                           [len(txs)], [1 if transactions is None else 0])

    # ------------------------------------------------------------------ the consensus calls
    def _call(self, fn):
        err = hgx_error()
        self._cb_error = None
        rc = fn(self.ctx, C.byref(err))
        _lib.check(rc, err)
        cb_err, self._cb_error = getattr(self, "_cb_error", None), None
        if cb_err is not None:   # a commit callback raised inside the call: re-raised here
            raise cb_err

    def DivideRounds(self):
        self._call(self.L.hgx_divide_rounds)

    def DecideFame(self):
        self._call(self.L.hgx_decide_fame)

    def FindOrder(self):
        self._call(self.L.hgx_find_order)

    def RunConsensus(self):
        """node/core.go:277-303"""
        self._call(self.L.hgx_run_consensus)

    def save(self, path: str):
        """Checkpoint of the resident events (hgx_save; the BadgerStore's topological event log,
        badger_store.go:309-343). Format: include/hgx.h, babble_amd/checkpoint.py."""
        self._call(lambda ctx, e: self.L.hgx_save(ctx, os.fsencode(path), e))

    def save_with_payloads(self, path: str, payloads: Sequence[bytes]):
        """Checkpoint with the caller's per-event bytes (hgx_save_ex), one entry per event
        (ValueError otherwise: hgx_save_ex reads E + 1 offsets and that many blob bytes)."""
        if len(payloads) != self.num_events():
            raise ValueError(f"save_with_payloads: {len(payloads)} payloads for {self.num_events()} events")
        off = np.zeros(len(payloads) + 1, np.int64)
        off[1:] = np.cumsum([len(b) for b in payloads]) if len(payloads) else []
        blob = np.frombuffer(b"".join(payloads) or b"\0", np.uint8).copy()
        self._call(lambda ctx, e: self.L.hgx_save_ex(ctx, os.fsencode(path), ptr(off), ptr(blob), e))

    def event_id(self, gid: int) -> bytes:
        """Event.Hash of an inserted event (hgx_get_event_id)."""
        out = np.zeros(32, np.uint8)
        self._call(lambda ctx, e: self.L.hgx_get_event_id(ctx, gid, ptr(out), e))
        return out.tobytes()

    def event_payload(self, gid: int) -> bytes:
        """The payload a bootstrapped checkpoint stored for the event (hgx_get_event_payload)."""
        ln = C.c_int64(0)
        self._call(lambda ctx, e: self.L.hgx_get_event_payload(ctx, gid, None, 0, C.byref(ln), e))
        out = np.zeros(max(1, ln.value), np.uint8)
        self._call(lambda ctx, e: self.L.hgx_get_event_payload(ctx, gid, ptr(out), ln.value, C.byref(ln), e))
        return out[:ln.value].tobytes()

    def Bootstrap(self, path: str):
        """Hashgraph.Bootstrap (hashgraph.go:1008-1037) from a checkpoint file: replay the events
        in topological order, then DivideRounds / DecideFame / FindOrder once (hgx_bootstrap)."""
        self._call(lambda ctx, e: self.L.hgx_bootstrap(ctx, os.fsencode(path), e))

    def set_commit_callback(self, fn):
        """commitCh (hashgraph.go:848-854): fn(graph, block, rr, first, n_events, n_tx) for every new
        block with transactions, at the end of FindOrder (after the counters are updated); None
        removes it. An exception raised by fn is kept (later blocks are still delivered) and
        re-raised when the FindOrder / RunConsensus call returns."""
        if fn is None:
            self._commit_cb = None
            rc = self.L.hgx_set_commit_callback(self.ctx, None, None)
        else:
            def tramp(_user, g, b, rr, first, nev, ntx):
                try:
                    fn(int(g), int(b), int(rr), int(first), int(nev), int(ntx))
                except BaseException as ex:   # ctypes would print and drop it
                    if getattr(self, "_cb_error", None) is None:
                        self._cb_error = ex
            self._commit_cb = _lib.COMMIT_FN(tramp)   # kept alive while registered
            rc = self.L.hgx_set_commit_callback(self.ctx, C.cast(self._commit_cb, C.c_void_p), None)
        if rc:
            raise HgxError(rc, "hgx_set_commit_callback failed")

    # ------------------------------------------------------------------ Reset / GetFrame
    ROOT_Y, ROOT_OTHER = -3, -4   # other-parent codes after a Reset (hgx.h)

    def Reset(self, root_index, root_round, root_y_is_event, others=None):
        """Hashgraph.Reset(roots) (hashgraph.go:877-895): per participant Root.Index, Root.Round and
        whether Root.Y names an event; `others` = the 32-byte ids of the events the roots' Others
        maps hold (hgx_set_root_others). Then insert with self-parent -1 = Root.X and other-parent
        ROOT_Y / ROOT_OTHER for parents outside the store."""
        a = [np.ascontiguousarray(x, np.int32) for x in (root_index, root_round, root_y_is_event)]
        err = hgx_error()
        rc = self.L.hgx_reset(self.ctx, *[ptr(x) for x in a], C.byref(err))
        _lib.check(rc, err)
        if others is not None and len(others):
            k = np.ascontiguousarray(others, np.uint8).reshape(-1, 32)
            self._call(lambda ctx, e: self.L.hgx_set_root_others(ctx, ptr(k), k.shape[0], e))

    def GetFrame(self):
        """Hashgraph.GetFrame (hashgraph.go:897-995): roots (x, y, index, round per participant),
        events (gids, topological order), others {event: other-parent}."""
        C_ = self.n * self.G
        ne, no = C.c_int64(), C.c_int64()
        rx, ry = np.zeros(C_, np.int64), np.zeros(C_, np.int64)
        ri, rr = np.zeros(C_, np.int32), np.zeros(C_, np.int32)
        err = hgx_error()
        cap = self.num_events() + 1
        ev = np.zeros(cap, np.int64)
        oe, op = np.zeros(cap, np.int64), np.zeros(cap, np.int64)
        rc = self.L.hgx_get_frame(self.ctx, ptr(ev), cap, C.byref(ne), ptr(rx), ptr(ry), ptr(ri), ptr(rr), ptr(oe),
                                  ptr(op), cap, C.byref(no), C.byref(err))
        _lib.check(rc, err)
        return dict(roots=[(int(rx[p]), int(ry[p]), int(ri[p]), int(rr[p])) for p in range(C_)],
                    events=[int(x) for x in ev[:ne.value]],
                    others={int(oe[k]): int(op[k]) for k in range(no.value)})

    # ------------------------------------------------------------------ row-sharded graph
    def set_shard(self, rank: int, world: int):
        """One graph row-sharded over `world` ranks (hgx_set_shard)."""
        if self.L.hgx_set_shard(self.ctx, rank, world) != 0:
            raise ValueError("invalid shard")
        self.shard = (rank, world)

    def FindOrderSharded(self, all_gather):
        """FindOrder of a row-sharded graph: begin, exchange of the shards' consensus timestamps,
        end. all_gather(local: np.ndarray[int64], counts: list[int]) -> list of every rank's
        array (torch.distributed over gloo, or over RCCL with device buffers)."""
        rank, world = self.shard
        self._call(self.L.hgx_find_order_begin)
        counts = [int(self.L.hgx_shard_values(self.ctx, r)) for r in range(world)]
        mine = np.zeros(counts[rank], np.int64)
        if counts[rank] and self.L.hgx_shard_export(self.ctx, ptr(mine), 0) != 0:
            raise HgxError(200, "hgx_shard_export failed")
        parts = all_gather(mine, counts)
        for r in range(world):
            if r != rank and counts[r]:
                a = np.ascontiguousarray(parts[r], np.int64)
                if self.L.hgx_shard_import(self.ctx, r, ptr(a), 0) != 0:
                    raise HgxError(200, "hgx_shard_import failed")
        self._call(self.L.hgx_find_order_end)

    def RunConsensusSharded(self, all_gather):
        self.DivideRounds()
        self.DecideFame()
        self.FindOrderSharded(all_gather)

    def reset_consensus(self):
        """Fresh consensus state over the same resident events (Bootstrap replay)."""
        rc = self.L.hgx_reset_consensus(self.ctx)
        if rc:
            raise HgxError(rc, "hgx_reset_consensus failed")

    # ------------------------------------------------------------------ state (hashgraph.go:15-37)
    def UndecidedRounds(self, graph: int = 0) -> List[int]:
        k = self.L.hgx_undecided_rounds(self.ctx, graph, None, 0)
        buf = np.zeros(max(k, 1), np.int32)
        self.L.hgx_undecided_rounds(self.ctx, graph, ptr(buf), k)
        return [int(v) for v in buf[:k]]

    def LastConsensusRound(self, graph: int = 0) -> Optional[int]:
        has = C.c_int32(0)
        v = self.L.hgx_last_consensus_round(self.ctx, graph, C.byref(has))
        return int(v) if has.value else None

    def LastCommitedRoundEvents(self, graph: int = 0) -> int:
        return int(self.L.hgx_last_commited_round_events(self.ctx, graph))

    def ConsensusTransactions(self, graph: int = 0) -> int:
        return int(self.L.hgx_consensus_transactions(self.ctx, graph))

    def PendingLoadedEvents(self, graph: int = 0) -> int:
        return int(self.L.hgx_pending_loaded_events(self.ctx, graph))

    def SuperMajority(self) -> int:
        return int(self.L.hgx_super_majority(self.ctx))

    # ------------------------------------------------------------------ Store views
    def LastRound(self, graph: int = 0) -> int:
        return int(self.L.hgx_last_round(self.ctx, graph))

    def RoundEvents(self, r: int, graph: int = 0) -> int:
        return int(self.L.hgx_round_event_count(self.ctx, graph, r))

    def RoundWitnesses(self, r: int, graph: int = 0) -> List[int]:
        buf = np.zeros(self.n, np.int64)
        k = self.L.hgx_round_witnesses(self.ctx, graph, r, ptr(buf), self.n)
        return [int(v) for v in buf[:k]]

    def Known(self, graph: int = 0) -> np.ndarray:
        out = np.zeros(self.n, np.int32)
        self.L.hgx_known(self.ctx, graph, ptr(out))
        return out

    def ConsensusEvents(self, graph: int = 0) -> np.ndarray:
        k = int(self.L.hgx_consensus_events_count(self.ctx, graph))
        out = np.zeros(max(k, 1), np.int64)
        if k:
            rc = self.L.hgx_consensus_events(self.ctx, graph, 0, k, ptr(out))
            if rc:
                raise HgxError(rc, "hgx_consensus_events failed")
        return out[:k]

    def GetBlock(self, rr: int, graph: int = 0) -> dict:
        """Store.GetBlock(rr): the block with that RoundReceived (HgxError "<rr>, Not Found")."""
        b, err = C.c_int64(), hgx_error()
        _lib.check(self.L.hgx_get_block(self.ctx, graph, rr, C.byref(b), C.byref(err)), err)
        return self.Blocks(graph)[b.value]

    def consensus_received(self, graph: int = 0, first: int = 0, count: Optional[int] = None):
        """(gids, round received, consensus timestamps) along the graph's consensus order."""
        k = int(self.L.hgx_consensus_events_count(self.ctx, graph))
        count = k - first if count is None else count
        g = np.zeros(max(count, 1), np.int64)
        rr = np.zeros(max(count, 1), np.int32)
        ts = np.zeros(max(count, 1), np.int64)
        if count:
            rc = self.L.hgx_consensus_received(self.ctx, graph, first, count, ptr(g), ptr(rr), ptr(ts))
            if rc:
                raise HgxError(rc, "hgx_consensus_received failed")
        return g[:count], rr[:count], ts[:count]

    # ------------------------------------------------------------------ Store: events by participant
    def LastFrom(self, participant: int):
        """(gid of the last event or -1, isRoot) (inmem_store.go:85-102)."""
        gid, root, err = C.c_int64(), C.c_int32(), hgx_error()
        _lib.check(self.L.hgx_last_from(self.ctx, participant, C.byref(gid), C.byref(root), C.byref(err)), err)
        return gid.value, bool(root.value)

    def ParticipantEvents(self, participant: int, skip: int) -> List[int]:
        cnt, err = C.c_int64(), hgx_error()
        _lib.check(self.L.hgx_participant_events(self.ctx, participant, skip, None, 0, C.byref(cnt), C.byref(err)),
                   err)
        out = np.zeros(max(cnt.value, 1), np.int64)
        _lib.check(self.L.hgx_participant_events(self.ctx, participant, skip, ptr(out), cnt.value, C.byref(cnt),
                                                 C.byref(err)), err)
        return [int(v) for v in out[:cnt.value]]

    def ParticipantEvent(self, participant: int, index: int) -> int:
        gid, err = C.c_int64(), hgx_error()
        _lib.check(self.L.hgx_participant_event(self.ctx, participant, index, C.byref(gid), C.byref(err)), err)
        return gid.value

    def GetRoot(self, participant: int) -> dict:
        x, y, idx, rnd, err = C.c_int64(), C.c_int64(), C.c_int32(), C.c_int32(), hgx_error()
        _lib.check(self.L.hgx_get_root(self.ctx, participant, C.byref(x), C.byref(y), C.byref(idx), C.byref(rnd),
                                       C.byref(err)), err)
        return dict(X=x.value, Y=y.value, Index=idx.value, Round=rnd.value)

    def GetEvent(self, gid: int) -> dict:
        cr, ix, sp, op, ts, nt, nil, err = (C.c_int32(), C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64(),
                                            C.c_int32(), C.c_int32(), hgx_error())
        _lib.check(self.L.hgx_get_event(self.ctx, gid, C.byref(cr), C.byref(ix), C.byref(sp), C.byref(op),
                                        C.byref(ts), C.byref(nt), C.byref(nil), C.byref(err)), err)
        return dict(creator=cr.value, index=ix.value, self_parent=sp.value, other_parent=op.value,
                    timestamp=ts.value, ntx=nt.value, tx_nil=bool(nil.value))

    def wire_info(self, first: int = 0, count: Optional[int] = None):
        """SetWireInfo of events [first, first+count): (self-parent index, other-parent creator, other-parent index)."""
        count = self.num_events() - first if count is None else count
        a, b, c = (np.zeros(max(count, 1), np.int32) for _ in range(3))
        if count:
            rc = self.L.hgx_wire_info(self.ctx, first, count, ptr(a), ptr(b), ptr(c))
            if rc:
                raise HgxError(rc, "hgx_wire_info failed")
        return a[:count], b[:count], c[:count]

    def ReadWireInfo(self, creator: int, sp_index: int, op_creator: int, op_index: int):
        sp, op, err = C.c_int64(), C.c_int64(), hgx_error()
        _lib.check(self.L.hgx_read_wire_info(self.ctx, creator, sp_index, op_creator, op_index, C.byref(sp),
                                             C.byref(op), C.byref(err)), err)
        return sp.value, op.value

    def Blocks(self, graph: int = 0) -> List[dict]:
        res = []
        for b in range(int(self.L.hgx_num_blocks(self.ctx, graph))):
            rr, nev, nil, com = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int32()
            first, ntx = C.c_int64(), C.c_int64()
            self.L.hgx_block_info(self.ctx, graph, b, C.byref(rr), C.byref(first), C.byref(nev), C.byref(ntx),
                                  C.byref(nil), C.byref(com))
            res.append(dict(rr=rr.value, first=first.value, n_events=nev.value, ntx=ntx.value,
                            tx_nil=bool(nil.value), committed=bool(com.value)))
        return res

    # ------------------------------------------------------------------ primitives
    def Ancestor(self, x: int, y: int) -> bool:
        return bool(self.L.hgx_ancestor(self.ctx, x, y))

    def SelfAncestor(self, x: int, y: int) -> bool:
        return bool(self.L.hgx_self_ancestor(self.ctx, x, y))

    def See(self, x: int, y: int) -> bool:
        return bool(self.L.hgx_see(self.ctx, x, y))

    def StronglySee(self, x: int, y: int) -> bool:
        return bool(self.L.hgx_strongly_see(self.ctx, x, y))

    def OldestSelfAncestorToSee(self, x: int, y: int) -> int:
        return int(self.L.hgx_oldest_self_ancestor_to_see(self.ctx, x, y))

    def Round(self, x: int) -> int:
        return int(self.L.hgx_round(self.ctx, x))

    def Witness(self, x: int) -> bool:
        return bool(self.L.hgx_witness(self.ctx, x))

    def coords(self, x: int):
        la = np.zeros(self.n, np.int32)
        fd = np.zeros(self.n, np.int32)
        rc = self.L.hgx_get_coords(self.ctx, x, ptr(la), ptr(fd))
        if rc:
            raise HgxError(rc, "hgx_get_coords failed")
        return la, fd

    # ------------------------------------------------------------------ bulk results
    def num_events(self) -> int:
        return int(self.L.hgx_num_events(self.ctx))

    def rounds(self):
        E = self.num_events()
        rnd = np.zeros(max(E, 1), np.int32)
        wit = np.zeros(max(E, 1), np.int8)
        fam = np.zeros(max(E, 1), np.int8)
        if E:
            rc = self.L.hgx_get_rounds(self.ctx, 0, E, ptr(rnd), ptr(wit), ptr(fam))
            if rc:
                raise HgxError(rc, "hgx_get_rounds failed")
        return rnd[:E], wit[:E], fam[:E]

    def received(self):
        E = self.num_events()
        rr = np.zeros(max(E, 1), np.int32)
        cts = np.zeros(max(E, 1), np.int64)
        if E:
            rc = self.L.hgx_get_received(self.ctx, 0, E, ptr(rr), ptr(cts))
            if rc:
                raise HgxError(rc, "hgx_get_received failed")
        return rr[:E], cts[:E]

    def results(self, graph: int = 0) -> dict:
        """Same shape as tests' oracle results() for parity comparison (single-graph contexts)."""
        rnd, wit, fam = self.rounds()
        rr, cts = self.received()
        return dict(round=rnd, witness=wit, famous=fam, rr=rr, cts=np.where(rr >= 0, cts, 0),
                    order=self.ConsensusEvents(graph), last_round=self.LastRound(graph),
                    undecided=self.UndecidedRounds(graph), lcr=self.LastConsensusRound(graph),
                    lcre=self.LastCommitedRoundEvents(graph), consensus_tx=self.ConsensusTransactions(graph),
                    pending_loaded=self.PendingLoadedEvents(graph), blocks=self.Blocks(graph))

    def phase_times(self):
        out = np.zeros(22, np.float64)
        self.L.hgx_phase_times(self.ctx, ptr(out), 22)
        return dict(coords_ms=out[0], rounds_ms=out[1], fame_ms=out[2], order_ms=out[3],
                    la_sweeps=int(out[4]), rounds=int(out[5]), compact=int(out[6]),
                    la_rows=int(out[7]), rebuild=int(out[8]), r_lo=int(out[9]),
                    la_wave=int(out[10]), la_wave_fallbacks=int(out[11]), la_wave_segs=int(out[12]),
                    round_p_runs=int(out[13]), round_p_fallbacks=int(out[14]), round_p_ovf=int(out[15]),
                    round_p_fail_round=int(out[16]), round_p_fail_chain=int(out[17]),
                    round_g_runs=int(out[18]), la_small=int(out[19]), la_verify=int(out[20]),
                    sort_seg=int(out[21]))

    def set_fame_tally(self, mode):
        """DecideFame tally: "popc" (default), "vote" (per-round kernel) or "mfma" (int8 MFMA)."""
        m = {"popc": 0, "vote": 1, "mfma": 2}[mode] if isinstance(mode, str) else int(mode)
        if self.L.hgx_set_fame_tally(self.ctx, m) != 0:
            raise ValueError(f"invalid fame tally {mode}")

    def set_la_kernel(self, mode):
        """DivideRounds lastAncestors: "wave" (default, one dataflow pass; a small graph's whole
        graph in LDS), "ring" (the dataflow pass without the small-graph form) or "sweep"
        (Gauss-Seidel); "wave+verify" runs the verify sweep after every time-segmented pass (by default
        only when the segments' exactness check fails)."""
        m = {"wave": 0, "sweep": 1, "ring": 1025, "wave+verify": 1026}[mode] if isinstance(mode, str) else int(mode)
        if self.L.hgx_set_la_kernel(self.ctx, m) != 0:
            raise ValueError(f"invalid lastAncestors kernel {mode}")

    def set_round_kernel(self, mode):
        """DivideRounds rounds: "auto" (default: the persistent recurrence on calls that lay the DAG
        out anew, where it applies, else per-round "candidate" launches; the whole-graph
        recurrence on every call for n <= 16), "persistent" (the persistent recurrence on every
        call where it applies), "graph" (one workgroup per graph of n <= 16 on every call),
        "block" (block binary search per round), "candidate" (one launch per round, one lane
        per candidate) or "auto-steps" ("auto" without the big-n persistent recurrence: n > 256
        runs the "candidate" steps)."""
        m = ({"auto": 0, "block": 1, "candidate": 2, "persistent": 3, "graph": 4, "auto-steps": 5}[mode]
             if isinstance(mode, str) else int(mode))
        if self.L.hgx_set_round_kernel(self.ctx, m) != 0:
            raise ValueError(f"invalid round kernel {mode}")

    def set_sort_kernel(self, mode):
        """FindOrder's sort: "auto" (default: buckets by (graph, roundReceived), each sorted in LDS,
        where every bucket holds <= 8 192 events) or "radix" (LSD radix passes over the whole list)."""
        m = {"auto": 0, "radix": 1}[mode] if isinstance(mode, str) else int(mode)
        if self.L.hgx_set_sort_kernel(self.ctx, m) != 0:
            raise ValueError(f"invalid sort kernel {mode}")

    def set_round_shards(self, shards: int):
        """hgx_create_sharded's chain-sharded recurrence with every shard on this context's device
        (hgx_set_round_shards): on an empty context; W shards on one device need
        GPU_MAX_HW_QUEUES >= W + 2."""
        if self.L.hgx_set_round_shards(self.ctx, int(shards)) != 0:
            raise ValueError(f"invalid shard count {shards} (an empty context, 1..8 shards, "
                             f"GPU_MAX_HW_QUEUES >= shards + 2 for shards sharing a device)")

    def set_shard_remote(self, on: bool = True):
        """Test switch (hgx_set_shard_remote): the shards' window stores take the cross-device
        (system-scope) path even where the shards share a device."""
        if self.L.hgx_set_shard_remote(self.ctx, 1 if on else 0) != 0:
            raise ValueError("hgx_set_shard_remote: not a chain-sharded context")

    def set_cts_kernel(self, mode):
        """FindOrder consensus timestamps: "auto" = "tile" (default: one tile of 8 positions per
        block) or "pipe" (resident blocks with several tiles' loads in flight, hgx_cts.hip)."""
        m = {"auto": 0, "tile": 1, "pipe": 2}[mode] if isinstance(mode, str) else int(mode)
        if self.L.hgx_set_cts_kernel(self.ctx, m) != 0:
            raise ValueError(f"invalid timestamp kernel {mode}")

    def set_incremental(self, on: bool):
        """DivideRounds schedule: incremental (default) or full recompute on every call."""
        if self.L.hgx_set_incremental(self.ctx, 1 if on else 0) != 0:
            raise ValueError("invalid schedule")

    def reserve_rounds(self, rounds: int):
        """Size the per-round tables (before the first DivideRounds; small values exercise growth)."""
        if self.L.hgx_reserve_rounds(self.ctx, int(rounds)) != 0:
            raise ValueError("hgx_reserve_rounds failed")

    def set_coord_storage(self, mode):
        """0 = auto (uint16 coordinates when every Index fits), 1 = always int32."""
        if self.L.hgx_set_coord_storage(self.ctx, int(mode)) != 0:
            raise ValueError(f"invalid coordinate storage mode {mode}")

    def kernel_stats(self):
        res = {}
        for k in range(10):
            name = C.create_string_buffer(32)
            ms, launches, nbytes = C.c_double(), C.c_int64(), C.c_double()
            if self.L.hgx_kernel_stats(self.ctx, k, name, 32, C.byref(ms), C.byref(launches), C.byref(nbytes)):
                break
            res[name.value.decode()] = dict(ms=ms.value, launches=launches.value, bytes=nbytes.value)
        return res

    KERNELS = ("layout", "la_sweep", "fd_build", "round_gather", "round_search", "fame", "threshold",
               "round_received", "cts_median", "order_sort")

    def set_kernel_timing(self, which=True):
        """True = time every kernel launch with HIP events; a kernel name = only that one; False = off."""
        if which is True:
            mask = -1
        elif not which:
            mask = 0
        else:
            mask = 1 << self.KERNELS.index(which)
        self.L.hgx_set_kernel_timing(self.ctx, mask)

    def reset_stats(self):
        self.L.hgx_reset_stats(self.ctx)


class DeviceBuffer:
    """A host array copied to a buffer from hgx_device_alloc (libhgx's own HIP runtime)."""

    def __init__(self, a: np.ndarray, device: int = 0):
        self.L = _lib.lib()
        self.device = device
        a = np.ascontiguousarray(a)
        self.nbytes = a.nbytes
        self.p = C.c_void_p()
        if self.L.hgx_device_alloc(device, max(1, a.nbytes), C.byref(self.p)) != 0:
            raise HgxError(200, "hgx_device_alloc failed")
        if a.nbytes and self.L.hgx_device_copy(device, self.p, ptr(a), a.nbytes, 1) != 0:
            self.close()
            raise HgxError(200, "hgx_device_copy failed")

    @property
    def addr(self) -> int:
        return int(self.p.value or 0)

    def close(self):
        if getattr(self, "p", None) is not None and self.p.value:
            self.L.hgx_device_free(self.device, self.p)
            self.p = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceTrace:
    """A trace's hgx_events columns resident in HBM (buffers from hgx_device_alloc on the
    context's device). Feeds Hashgraph.insert_device."""

    def __init__(self, t, device: int = 0):
        self.L = _lib.lib()
        self.device = device
        self.E = int(t.creator.shape[0])
        self.bufs = {}
        for name, src, dt in (("creator", t.creator, np.int32), ("index", t.index, np.int64),
                              ("sp", t.sp, np.int64), ("op", t.op, np.int64), ("ts", t.ts, np.int64),
                              ("hash", t.hash, np.uint8), ("s", t.s, np.uint8), ("ntx", t.ntx, np.int32),
                              ("nil", t.txnil, np.int32)):
            a = np.ascontiguousarray(src, dtype=dt)
            p = C.c_void_p()
            if self.L.hgx_device_alloc(device, a.nbytes, C.byref(p)) != 0:
                self.close()
                raise HgxError(200, "hgx_device_alloc failed")
            self.bufs[name] = (p, a.itemsize * (32 if name in ("hash", "s") else 1))
            if a.nbytes and self.L.hgx_device_copy(device, p, ptr(a), a.nbytes, 1) != 0:
                self.close()
                raise HgxError(200, "hgx_device_copy failed")

    def close(self):
        for p, _ in getattr(self, "bufs", {}).values():
            self.L.hgx_device_free(self.device, p)
        self.bufs = {}

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def events(self, lo: int, hi: int) -> hgx_events:
        def p(name):
            base, per = self.bufs[name]
            return C.c_void_p((base.value or 0) + lo * per)

        return hgx_events(p("creator"), p("index"), p("sp"), p("op"), p("ts"), p("hash"), p("s"), p("ntx"), p("nil"))


def block_hash(rr: int, txs: List[bytes], tx_nil: bool) -> bytes:
    """SHA256(json.Encoder(Block)) (hashgraph/block.go:44-53), computed by libhgx."""
    L = _lib.lib()
    ntx = len(txs)
    bufs = [C.create_string_buffer(t, max(len(t), 1)) for t in txs]
    ptrs = (C.c_void_p * max(ntx, 1))(*[C.cast(b, C.c_void_p) for b in bufs])
    lens = (C.c_int64 * max(ntx, 1))(*[len(t) for t in txs])
    out = C.create_string_buffer(32)
    rc = L.hgx_block_hash(rr, ntx, ptrs, lens, 1 if tx_nil else 0, out)
    if rc:
        raise HgxError(rc, "hgx_block_hash failed")
    return out.raw


def sha256_batch(data: np.ndarray, offsets: np.ndarray, device: int = 0) -> np.ndarray:
    """crypto.SHA256 (crypto/utils.go:11-16) of every message data[offsets[i]:offsets[i+1]]
    in one device launch (hgx_sha256_batch). Returns a (count, 32) uint8 array.
    Raises HgxError (code HGX_ERR_DEVICE) without a gfx950 GPU: there is no CPU path."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    count = max(len(offsets) - 1, 0)
    out = np.zeros((count, 32), dtype=np.uint8)
    err = hgx_error()
    rc = _lib.lib().hgx_sha256_batch(device, ptr(data) if data.size else None, ptr(offsets) if count else None,
                                     count, ptr(out) if count else None, C.byref(err))
    _lib.check(rc, err)
    return out


def event_ids(bodies: Sequence[bytes], device: int = 0) -> List[bytes]:
    """Event.Hash for a batch of json.Encoder(Event) encodings (hashgraph/event.go:171-180),
    hashed on the GPU; Hex() is "0x%X" of each (event.go:183-188)."""
    lens = np.fromiter((len(b) for b in bodies), dtype=np.int64, count=len(bodies))
    offsets = np.zeros(len(bodies) + 1, dtype=np.int64)
    np.cumsum(lens, out=offsets[1:])
    data = np.frombuffer(b"".join(bodies), dtype=np.uint8)
    return [bytes(r) for r in sha256_batch(data, offsets, device)]


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def sha256_bench_messages(n: int, min_len: int, max_len: int, seed: int) -> List[bytes]:
    """The first n synthetic messages hgx_sha256_bench hashes (include/hgx.h), rebuilt on the host."""
    i = np.arange(n, dtype=np.uint64)
    lens = min_len + (_splitmix64(~np.uint64(seed) + i) % np.uint64(max_len - min_len + 1)).astype(np.int64)
    total = int(lens.sum())
    words = _splitmix64(np.uint64(seed) + np.arange((total + 7) // 8, dtype=np.uint64))
    blob = words.astype("<u8").tobytes()
    out, o = [], 0
    for ln in lens:
        out.append(blob[o:o + int(ln)])
        o += int(ln)
    return out


def sha256_bench(count: int, min_len: int, max_len: int, seed: int = 5, warmup: int = 1, iters: int = 3,
                 n_sample: int = 64, device: int = 0) -> dict:
    """Device-resident SHA-256 throughput (hgx_sha256_bench) + digests of the first n_sample messages."""
    ms, tot, nb = C.c_double(), C.c_int64(), C.c_int64()
    sample = np.zeros((n_sample, 32), dtype=np.uint8)
    rc = _lib.lib().hgx_sha256_bench(device, count, min_len, max_len, seed, warmup, iters, C.byref(ms),
                                     C.byref(tot), C.byref(nb), n_sample, ptr(sample))
    if rc:
        raise HgxError(rc, "hgx_sha256_bench failed")
    return {"ms_per_launch": ms.value, "bytes": tot.value, "blocks": nb.value, "sample": sample}


def _p256_cols(keys65, key_idx, digest, r, s):
    k = np.ascontiguousarray(keys65, np.uint8).reshape(-1, 65)
    cols = [np.ascontiguousarray(key_idx, np.int32)] + [np.ascontiguousarray(x, np.uint8).reshape(-1, 32)
                                                         for x in (digest, r, s)]
    m = cols[0].shape[0]
    assert all(c.shape[0] == m for c in cols[1:])
    return k, cols, m


def p256_verify(keys65, key_idx, digest, r, s, device: int = 0) -> np.ndarray:
    """Event.Verify for a batch (hgx_p256_verify_batch): 1 valid, 0 invalid, 2 key not a P-256 point."""
    k, cols, m = _p256_cols(keys65, key_idx, digest, r, s)
    out = np.zeros(m, np.uint8)
    err = hgx_error()
    rc = _lib.lib().hgx_p256_verify_batch(device, ptr(k), k.shape[0], *[ptr(c) for c in cols], m, ptr(out),
                                          C.byref(err))
    _lib.check(rc, err)
    return out


def p256_verify_bench(keys65, key_idx, digest, r, s, warmup: int = 1, iters: int = 3, device: int = 0) -> dict:
    """Device-resident verify throughput (hgx_p256_verify_bench): ms per (tables + verify) launch."""
    k, cols, m = _p256_cols(keys65, key_idx, digest, r, s)
    out = np.zeros(m, np.uint8)
    ms = C.c_double()
    rc = _lib.lib().hgx_p256_verify_bench(device, ptr(k), k.shape[0], *[ptr(c) for c in cols], m, warmup, iters,
                                          ptr(out), C.byref(ms))
    if rc:
        raise HgxError(rc, "hgx_p256_verify_bench failed")
    return {"ms_per_launch": ms.value, "out": out}
