"""Test infrastructure: ctypes binding of the CPU oracle (oracle/liboracle_hg.so) plus
trace construction for the reference's fixtures and the Core gossip simulation.

Nothing here is product code.  The oracle restates the reference consensus path
(datatypevoid/babble hashgraph/hashgraph.go); the fixtures restate the play tables
of hashgraph/hashgraph_test.go and node/core_test.go (tests/golden/plays.json).
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
import os
import subprocess
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle_hg.so")
GOLDEN = os.path.join(ROOT, "tests", "golden")

T0_NS = 1_500_000_000_000_000_000  # 2017-07-14T02:40:00Z, synthetic creation clock
MAXI32 = 2147483647

_lib = None


def oracle_lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(ORACLE_SO):
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
    L = C.CDLL(ORACLE_SO)
    i32, i64, p = C.c_int, C.c_int64, C.c_void_p
    L.hgo_new.restype = p
    L.hgo_new.argtypes = [i32]
    L.hgo_free.argtypes = [p]
    L.hgo_insert.restype = i32
    L.hgo_insert.argtypes = [p, i32, i64, i64, i64, i64, p, p, i32, i32, p, p, C.c_char_p, i32]
    L.hgo_insert_batch.restype = i64
    L.hgo_insert_batch.argtypes = [p, i64] + [p] * 11 + [C.POINTER(C.c_int), C.c_char_p, i32]
    for nm in ("hgo_divide_rounds",):
        getattr(L, nm).argtypes = [p]
        getattr(L, nm).restype = i32
    for nm in ("hgo_decide_fame", "hgo_decide_round_received", "hgo_find_order"):
        getattr(L, nm).argtypes = [p, C.c_char_p, i32]
        getattr(L, nm).restype = i32
    for nm in ("hgo_ancestor", "hgo_self_ancestor", "hgo_see", "hgo_strongly_see"):
        getattr(L, nm).argtypes = [p, i64, i64]
        getattr(L, nm).restype = i32
    L.hgo_oldest_self_ancestor_to_see.argtypes = [p, i64, i64]
    L.hgo_oldest_self_ancestor_to_see.restype = i64
    L.hgo_parent_round.argtypes = [p, i64, C.POINTER(C.c_int)]
    L.hgo_parent_round.restype = i32
    for nm in ("hgo_round_inc", "hgo_round", "hgo_witness", "hgo_famous", "hgo_round_received"):
        getattr(L, nm).argtypes = [p, i64]
        getattr(L, nm).restype = i32
    L.hgo_consensus_timestamp.argtypes = [p, i64]
    L.hgo_consensus_timestamp.restype = i64
    for nm in ("hgo_num_events", "hgo_consensus_transactions", "hgo_pending_loaded_events", "hgo_num_blocks"):
        getattr(L, nm).argtypes = [p]
        getattr(L, nm).restype = i64
    for nm in ("hgo_super_majority", "hgo_last_round", "hgo_last_commited_round_events"):
        getattr(L, nm).argtypes = [p]
        getattr(L, nm).restype = i32
    L.hgo_round_event_count.argtypes = [p, i32]
    L.hgo_round_event_count.restype = i32
    L.hgo_round_witnesses.argtypes = [p, i32, p, i32]
    L.hgo_round_witnesses.restype = i32
    L.hgo_coords.argtypes = [p, i64, p, p]
    L.hgo_wire_info.argtypes = [p, i64, p, p, p]
    L.hgo_undecided_rounds.argtypes = [p, p, i32]
    L.hgo_undecided_rounds.restype = i32
    L.hgo_last_consensus_round.argtypes = [p, C.POINTER(C.c_int)]
    L.hgo_last_consensus_round.restype = i32
    L.hgo_consensus_events.argtypes = [p, p, i64]
    L.hgo_consensus_events.restype = i64
    L.hgo_known.argtypes = [p, p]
    L.hgo_reset.argtypes = [p, p, p, p]
    L.hgo_reset.restype = i32
    L.hgo_get_frame.argtypes = [p, p, i64, p, p, p, p, p, p, p, i64, p]
    L.hgo_get_frame.restype = i32
    L.hgo_block.argtypes = [p, i64, p, p, p, p, p]
    L.hgo_block_tx.argtypes = [p, i64, i32, p, i64]
    L.hgo_block_tx.restype = i64
    # Go encoders
    L.goenc_sha256.argtypes = [p, C.c_size_t, p]
    L.goenc_event_json_bound.argtypes = [i32, p, C.c_size_t]
    L.goenc_event_json_bound.restype = C.c_size_t
    L.goenc_event_json.argtypes = [i32, p, p, i32, C.c_char_p, C.c_char_p, p, C.c_size_t, i64, i64, p, p, p]
    L.goenc_event_json.restype = C.c_size_t
    L.goenc_block_json_bound.argtypes = [i32, p]
    L.goenc_block_json_bound.restype = C.c_size_t
    L.goenc_block_json.argtypes = [i64, i32, p, p, i32, p]
    L.goenc_block_json.restype = C.c_size_t
    L.goenc_rfc3339nano.argtypes = [i64, p]
    L.goenc_rfc3339nano.restype = C.c_size_t
    _lib = L
    return L


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


# ----------------------------------------------------------------------------- Go encoders

def go_event_json(txs: Optional[List[bytes]], sp_hex: str, op_hex: str, creator: bytes,
                  ts_ns: int, index: int, r: bytes, s: bytes) -> bytes:
    L = oracle_lib()
    txs_l = txs or []
    ntx = len(txs_l)
    bufs = [C.create_string_buffer(t, len(t)) if len(t) else C.create_string_buffer(1) for t in txs_l]
    ptrs = (C.c_void_p * max(ntx, 1))(*[C.cast(b, C.c_void_p) for b in bufs])
    lens = (C.c_size_t * max(ntx, 1))(*[len(t) for t in txs_l])
    cbuf = C.create_string_buffer(creator, len(creator))
    bound = L.goenc_event_json_bound(ntx, lens, len(creator))
    out = C.create_string_buffer(bound)
    rb = C.create_string_buffer(r, 32)
    sb = C.create_string_buffer(s, 32)
    n = L.goenc_event_json(ntx, ptrs, lens, 1 if txs is None else 0, sp_hex.encode(), op_hex.encode(),
                           cbuf, len(creator), ts_ns, index, rb, sb, out)
    return out.raw[:n]


def go_block_json(rr: int, txs: List[bytes], tx_nil: bool) -> bytes:
    L = oracle_lib()
    ntx = len(txs)
    bufs = [C.create_string_buffer(t, len(t)) if len(t) else C.create_string_buffer(1) for t in txs]
    ptrs = (C.c_void_p * max(ntx, 1))(*[C.cast(b, C.c_void_p) for b in bufs])
    lens = (C.c_size_t * max(ntx, 1))(*[len(t) for t in txs])
    out = C.create_string_buffer(L.goenc_block_json_bound(ntx, lens))
    n = L.goenc_block_json(rr, ntx, ptrs, lens, 1 if tx_nil else 0, out)
    return out.raw[:n]


def sha256(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()


# ----------------------------------------------------------------------------- traces

@dataclass
class Trace:
    """Structure-of-arrays event trace in insertion (topological) order."""
    n: int
    creator: np.ndarray       # int32 [E]
    index: np.ndarray         # int64 [E]
    sp: np.ndarray            # int64 [E] gid or -1
    op: np.ndarray            # int64 [E] gid or -1
    ts: np.ndarray            # int64 [E] unix ns
    hash: np.ndarray          # uint8 [E,32]
    s: np.ndarray             # uint8 [E,32] big-endian signature S
    ntx: np.ndarray           # int32 [E]
    txnil: np.ndarray         # int32 [E]
    txs: List[List[bytes]] = field(default_factory=list)  # payloads per event
    names: List[str] = field(default_factory=list)

    @property
    def E(self) -> int:
        return int(self.creator.shape[0])

    def name_to_gid(self) -> Dict[str, int]:
        return {nm: i for i, nm in enumerate(self.names)}


def fixture_key(fixture: str, p: int) -> bytes:
    return b"\x04" + sha256(f"{fixture}/key/{p}/x".encode()) + sha256(f"{fixture}/key/{p}/y".encode())


def _sig(tag: str):
    r = sha256(("R/" + tag).encode())
    s = sha256(("S/" + tag).encode())
    return r, s


class EventFactory:
    """Builds Go-identical event ids (SHA256 of json.Encoder(Event) output)."""

    def __init__(self, fixture: str, n: int):
        self.fixture = fixture
        self.n = n
        self.keys = [fixture_key(fixture, p) for p in range(n)]
        self.clock = 0

    def make(self, creator: int, index: int, sp_hex: str, op_hex: str, txs: Optional[List[bytes]], tag: str):
        ts = T0_NS + self.clock * 1000
        self.clock += 1
        r, s = _sig(f"{self.fixture}/{tag}")
        js = go_event_json(txs, sp_hex, op_hex, self.keys[creator], ts, index, r, s)
        h = sha256(js)
        return dict(creator=creator, index=index, ts=ts, txs=txs, r=r, s=s, hash=h,
                    hex="0x" + h.hex().upper(), json=js, tag=tag)


def load_plays() -> dict:
    with open(os.path.join(GOLDEN, "plays.json")) as f:
        return json.load(f)


def load_kat() -> dict:
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        return json.load(f)


def _payload(p):
    if p is None:
        return None
    return [x.encode() for x in p]


def fixture_trace(name: str) -> Trace:
    """Trace of a hashgraph_test.go fixture, events in the test's orderedEvents order."""
    fx = load_plays()[name]
    n = fx["n"]
    fac = EventFactory(name, n)
    evs, idx = [], {}
    for p, (nm, pl) in enumerate(fx["genesis"]):
        e = fac.make(p, 0, "", "", _payload(pl), nm)
        e["sp"], e["op"], e["name"] = -1, -1, nm
        idx[nm] = len(evs)
        evs.append(e)
    for to, index, spn, opn, nm, pl in fx["plays"]:
        sp = idx[spn] if spn else -1
        op = idx[opn] if opn else -1
        e = fac.make(to, index, evs[sp]["hex"] if sp >= 0 else "", evs[op]["hex"] if op >= 0 else "",
                     _payload(pl), nm)
        e["sp"], e["op"], e["name"] = sp, op, nm
        idx[nm] = len(evs)
        evs.append(e)
    return trace_from_events(n, evs)


def trace_from_events(n: int, evs: List[dict]) -> Trace:
    E = len(evs)
    t = Trace(
        n=n,
        creator=np.array([e["creator"] for e in evs], dtype=np.int32),
        index=np.array([e["index"] for e in evs], dtype=np.int64),
        sp=np.array([e["sp"] for e in evs], dtype=np.int64),
        op=np.array([e["op"] for e in evs], dtype=np.int64),
        ts=np.array([e["ts"] for e in evs], dtype=np.int64),
        hash=np.frombuffer(b"".join(e["hash"] for e in evs), dtype=np.uint8).reshape(E, 32).copy()
        if E else np.zeros((0, 32), np.uint8),
        s=np.frombuffer(b"".join(e["s"] for e in evs), dtype=np.uint8).reshape(E, 32).copy()
        if E else np.zeros((0, 32), np.uint8),
        ntx=np.array([len(e["txs"] or []) for e in evs], dtype=np.int32),
        txnil=np.array([1 if e["txs"] is None else 0 for e in evs], dtype=np.int32),
        txs=[list(e["txs"] or []) for e in evs],
        names=[e.get("name", e.get("tag", str(i))) for i, e in enumerate(evs)],
    )
    return t


# ----------------------------------------------------------------------------- oracle driver

class Oracle:
    """Thin wrapper over one oracle Hashgraph instance (gids = insertion order)."""

    def __init__(self, n: int):
        self.L = oracle_lib()
        self.h = self.L.hgo_new(n)
        self.n = n

    def __del__(self):
        try:
            if self.h:
                self.L.hgo_free(self.h)
                self.h = None
        except Exception:
            pass

    def insert(self, creator, index, sp, op, ts, hash32: bytes, s32: bytes, txs: Optional[List[bytes]]):
        err = C.create_string_buffer(256)
        txl = txs or []
        blob = b"".join(txl)
        lens = np.array([len(x) for x in txl] or [0], dtype=np.int32)
        bb = C.create_string_buffer(blob, max(len(blob), 1))
        hb = C.create_string_buffer(hash32, 32)
        sb = C.create_string_buffer(s32, 32)
        rc = self.L.hgo_insert(self.h, int(creator), int(index), int(sp), int(op), int(ts), hb, sb,
                               len(txl), 1 if txs is None else 0, bb, _ptr(lens), err, 256)
        return rc, err.value.decode(errors="replace")

    def insert_trace(self, t: Trace, lo: int = 0, hi: Optional[int] = None):
        hi = t.E if hi is None else hi
        if hasattr(t, "tx_seq"):   # generated gossip trace: one C call for the batch
            return self.insert_gossip(t, lo, hi)
        for i in range(lo, hi):
            txs = t.txs(i) if callable(getattr(t, "txs", None)) else (None if t.txnil[i] else t.txs[i])
            rc, msg = self.insert(t.creator[i], t.index[i], t.sp[i], t.op[i], t.ts[i], t.hash[i].tobytes(),
                                  t.s[i].tobytes(), txs)
            if rc:
                raise RuntimeError(f"oracle insert {i}: {msg}")

    def insert_gossip(self, t, lo: int, hi: int):
        """Batch insert of a generated trace (payloads rebuilt from tx_seq) via hgo_insert_batch."""
        sl = slice(lo, hi)
        cols = [np.ascontiguousarray(t.creator[sl], np.int32), np.ascontiguousarray(t.index[sl], np.int64),
                np.ascontiguousarray(t.sp[sl], np.int64), np.ascontiguousarray(t.op[sl], np.int64),
                np.ascontiguousarray(t.ts[sl], np.int64), np.ascontiguousarray(t.hash[sl], np.uint8),
                np.ascontiguousarray(t.s[sl], np.uint8), np.ascontiguousarray(t.ntx[sl], np.int32),
                np.ascontiguousarray(t.txnil[sl], np.int32)]
        has = np.nonzero(cols[7] > 0)[0]
        assert int(cols[7].max(initial=0)) <= 1, "generated traces carry at most one payload per event"
        pls = [gossip_payload(int(cols[0][k]), int(t.tx_seq[lo + k])) for k in has]
        blob = b"".join(pls)
        lens = np.array([len(x) for x in pls] or [0], np.int32)
        bb = C.create_string_buffer(blob, max(len(blob), 1))
        err = C.create_string_buffer(256)
        rc = C.c_int(0)
        m = self.L.hgo_insert_batch(self.h, hi - lo, *[_ptr(c) for c in cols], bb, _ptr(lens), C.byref(rc), err, 256)
        if rc.value:
            raise RuntimeError(f"oracle insert {lo + m}: {err.value.decode(errors='replace')}")

    def divide_rounds(self):
        return self.L.hgo_divide_rounds(self.h)

    def _call_err(self, fn):
        err = C.create_string_buffer(256)
        rc = fn(self.h, err, 256)
        return rc, err.value.decode(errors="replace")

    def decide_fame(self):
        return self._call_err(self.L.hgo_decide_fame)

    def decide_round_received(self):
        return self._call_err(self.L.hgo_decide_round_received)

    def find_order(self):
        return self._call_err(self.L.hgo_find_order)

    def run_consensus(self):
        self.divide_rounds()
        rc, msg = self.decide_fame()
        if rc:
            return rc, msg
        return self.find_order()

    # getters
    def E(self):
        return int(self.L.hgo_num_events(self.h))

    def coords(self, x):
        la = np.zeros(self.n, np.int32)
        fd = np.zeros(self.n, np.int32)
        self.L.hgo_coords(self.h, x, _ptr(la), _ptr(fd))
        return la, fd

    def wire(self, x):
        a, b, c = C.c_int32(), C.c_int32(), C.c_int32()
        self.L.hgo_wire_info(self.h, x, C.byref(a), C.byref(b), C.byref(c))
        return a.value, b.value, c.value

    def parent_round(self, x):
        r = C.c_int()
        v = self.L.hgo_parent_round(self.h, x, C.byref(r))
        return v, bool(r.value)

    def undecided_rounds(self):
        buf = np.zeros(1 << 16, np.int32)
        k = self.L.hgo_undecided_rounds(self.h, _ptr(buf), buf.size)
        return [int(v) for v in buf[:min(k, buf.size)]]

    def last_consensus_round(self):
        has = C.c_int()
        v = self.L.hgo_last_consensus_round(self.h, C.byref(has))
        return v if has.value else None

    def consensus_events(self):
        k = self.L.hgo_consensus_events(self.h, None, 0)
        out = np.zeros(max(k, 1), np.int64)
        self.L.hgo_consensus_events(self.h, _ptr(out), k)
        return out[:k]

    def round_witnesses(self, r):
        buf = np.zeros(1 << 14, np.int64)
        k = self.L.hgo_round_witnesses(self.h, r, _ptr(buf), buf.size)
        return [int(v) for v in buf[:k]]

    def known(self):
        out = np.zeros(self.n, np.int32)
        self.L.hgo_known(self.h, _ptr(out))
        return out

    def reset(self, root_index, root_round, root_y_is_event):
        """Hashgraph.Reset(roots) (hashgraph.go:877-895)."""
        a = [np.ascontiguousarray(root_index, np.int32), np.ascontiguousarray(root_round, np.int32),
             np.ascontiguousarray(root_y_is_event, np.uint8)]
        return self.L.hgo_reset(self.h, *[_ptr(x) for x in a])

    def get_frame(self):
        """Hashgraph.GetFrame (hashgraph.go:897-995), the encodings of include/hgx.h hgx_get_frame."""
        n, E = self.n, self.E()
        ev, oe, op = np.zeros(E + 1, np.int64), np.zeros(E + 1, np.int64), np.zeros(E + 1, np.int64)
        rx, ry = np.zeros(n, np.int64), np.zeros(n, np.int64)
        ri, rr = np.zeros(n, np.int32), np.zeros(n, np.int32)
        ne, no = C.c_int64(), C.c_int64()
        rc = self.L.hgo_get_frame(self.h, _ptr(ev), E + 1, C.byref(ne), _ptr(rx), _ptr(ry), _ptr(ri), _ptr(rr),
                                  _ptr(oe), _ptr(op), E + 1, C.byref(no))
        if rc:
            raise RuntimeError(f"hgo_get_frame: {rc}")
        return dict(roots=[(int(rx[p]), int(ry[p]), int(ri[p]), int(rr[p])) for p in range(n)],
                    events=[int(x) for x in ev[:ne.value]],
                    others={int(oe[k]): int(op[k]) for k in range(no.value)})

    def blocks(self):
        res = []
        for b in range(self.L.hgo_num_blocks(self.h)):
            rr, ntx, nil, com = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int32()
            hb = C.create_string_buffer(32)
            self.L.hgo_block(self.h, b, C.byref(rr), C.byref(ntx), C.byref(nil), C.byref(com), hb)
            txs = []
            for t in range(ntx.value):
                ln = self.L.hgo_block_tx(self.h, b, t, None, 0)
                buf = C.create_string_buffer(max(ln, 1))
                self.L.hgo_block_tx(self.h, b, t, buf, ln)
                txs.append(buf.raw[:ln])
            res.append(dict(rr=rr.value, ntx=ntx.value, tx_nil=bool(nil.value), committed=bool(com.value),
                            hash=hb.raw, txs=txs))
        return res

    def results(self) -> dict:
        """Per-event and global consensus state in a comparable form."""
        L, h = self.L, self.h
        E = self.E()
        rnd = np.array([L.hgo_round(h, x) for x in range(E)], np.int32)
        wit = np.array([L.hgo_witness(h, x) for x in range(E)], np.int8)
        fam = np.array([L.hgo_famous(h, x) for x in range(E)], np.int8)
        rr = np.array([L.hgo_round_received(h, x) for x in range(E)], np.int32)
        cts = np.array([L.hgo_consensus_timestamp(h, x) if rr[x] >= 0 else 0 for x in range(E)], np.int64)
        return dict(round=rnd, witness=wit, famous=fam, rr=rr, cts=cts,
                    order=self.consensus_events(), last_round=int(L.hgo_last_round(h)),
                    undecided=self.undecided_rounds(), lcr=self.last_consensus_round(),
                    lcre=int(L.hgo_last_commited_round_events(h)),
                    consensus_tx=int(L.hgo_consensus_transactions(h)),
                    pending_loaded=int(L.hgo_pending_loaded_events(h)),
                    blocks=[(b["rr"], b["ntx"], b["tx_nil"], b["committed"], b["hash"]) for b in self.blocks()])


def gossip_payload(creator: int, seq: int) -> bytes:
    """hgx_trace_tx_payload's bytes (include/hgx.h): "p%03d tx %08d"""
    return b"p%03d tx %08d" % (creator, seq)


def sign_batch(n_keys: int, key_idx, digests):
    """ECDSA P-256 signatures from libcrypto (oracle/p256_ref sign: derived keys, random nonces)
    for digests[i] under key key_idx[i]. Returns (public keys [n_keys, 65], r [m, 32], s [m, 32])."""
    import subprocess
    import tempfile
    exe = os.path.join(ROOT, "oracle", "p256_ref")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    key_idx = np.asarray(key_idx, np.uint32)
    digests = np.ascontiguousarray(digests, np.uint8).reshape(-1, 32)
    m = len(key_idx)
    rec = np.zeros(m, dtype=[("k", "<u4"), ("d", "u1", 32)])
    rec["k"], rec["d"] = key_idx, digests
    with tempfile.TemporaryDirectory() as td:
        fi, fo = os.path.join(td, "in"), os.path.join(td, "out")
        rec.tofile(fi)
        subprocess.check_call([exe, "sign", str(n_keys), fi, fo])
        out = np.fromfile(fo, np.uint8)
    keys = out[:65 * n_keys].reshape(n_keys, 65)
    rs = out[65 * n_keys:].reshape(m, 64)
    return keys, np.ascontiguousarray(rs[:, :32]), np.ascontiguousarray(rs[:, 32:])


def oracle_run(t: Trace, chunk: Optional[int] = None) -> Oracle:
    """Insert a trace and run consensus: batch (Bootstrap-style, hashgraph.go:1008-1037)
    or every `chunk` inserted events (Core.RunConsensus after each sync)."""
    o = Oracle(t.n)
    if chunk is None:
        o.insert_trace(t)
        rc, msg = o.run_consensus()
    else:
        rc, msg = 0, ""
        for lo in range(0, t.E, chunk):
            o.insert_trace(t, lo, min(t.E, lo + chunk))
            rc, msg = o.run_consensus()
            if rc:
                break
    if rc:
        raise RuntimeError(f"oracle consensus failed: {msg}")
    return o


# ----------------------------------------------------------------------------- Core simulation

class CoreSim:
    """Deterministic gossip among n Cores, each with its own Hashgraph backend
    (node/core_test.go:514-537 synchronizeCores/syncAndRunConsensus; node/core.go:79-230).

    backend_factory(n) must return an object with insert(creator, index, sp, op, ts, hash, s, txs)
    -> (rc, msg), run_consensus(), consensus_events() (local gids), last_consensus_round(), known().
    """

    def __init__(self, fixture: str, n: int, backend_factory):
        self.n = n
        self.fac = EventFactory(fixture, n)
        self.events: List[dict] = []          # global events
        self.by_hex: Dict[str, int] = {}
        self.backends = [backend_factory(n) for _ in range(n)]
        self.local: List[List[int]] = [[] for _ in range(n)]       # core -> [global id in insertion order]
        self.l2g: List[Dict[int, int]] = [dict() for _ in range(n)]
        self.g2l: List[Dict[int, int]] = [dict() for _ in range(n)]
        self.head = [-1] * n
        self.seq = [0] * n
        self.pool: List[List[bytes]] = [[] for _ in range(n)]
        for i in range(n):                     # Core.Init: genesis with nil txs (core.go:79-85)
            g = self._create(i, 0, -1, -1, None)
            self._insert(i, g)

    def _create(self, creator, index, sp_g, op_g, txs):
        sp_hex = self.events[sp_g]["hex"] if sp_g >= 0 else ""
        op_hex = self.events[op_g]["hex"] if op_g >= 0 else ""
        e = self.fac.make(creator, index, sp_hex, op_hex, txs, f"ev{len(self.events)}")
        e["sp_g"], e["op_g"] = sp_g, op_g
        g = len(self.events)
        self.events.append(e)
        self.by_hex[e["hex"]] = g
        return g

    def _insert(self, core, g):
        e = self.events[g]
        sp = self.g2l[core][e["sp_g"]] if e["sp_g"] >= 0 else -1
        op = self.g2l[core].get(e["op_g"], -2) if e["op_g"] >= 0 else -1
        rc, msg = self.backends[core].insert(e["creator"], e["index"], sp, op, e["ts"], e["hash"], e["s"], e["txs"])
        if rc:
            raise RuntimeError(f"core {core} insert: {msg}")
        lid = len(self.local[core])
        self.local[core].append(g)
        self.l2g[core][lid] = g
        self.g2l[core][g] = lid
        if e["creator"] == core:
            self.head[core] = g
            self.seq[core] = e["index"]

    def sync(self, frm, to, payload: List[bytes]):
        known = self.backends[to].known()
        unknown = []                            # Core.Diff (core.go:166-188)
        for g in self.local[frm]:
            e = self.events[g]
            if e["index"] > known[e["creator"]]:
                unknown.append(g)               # from's local order == topological order
        self.pool[to].extend(payload)           # AddTransactions
        other_head = -1
        for k, g in enumerate(unknown):         # Core.Sync (core.go:190-230)
            self._insert(to, g)
            if k == len(unknown) - 1:
                other_head = g
        if unknown or self.pool[to]:
            g = self._create(to, self.seq[to] + 1, self.head[to], other_head, list(self.pool[to]))
            self._insert(to, g)
            self.pool[to] = []

    def sync_and_run(self, frm, to, payload):
        self.sync(frm, to, payload)
        rc, msg = self.backends[to].run_consensus()
        if rc:
            raise RuntimeError(f"core {to} consensus: {msg}")

    def consensus_hex(self, core) -> List[str]:
        return [self.events[self.l2g[core][int(x)]]["hex"] for x in self.backends[core].consensus_events()]


# ----------------------------------------------------------------------------- Reset / frames
ROOT_Y, ROOT_OTHER, UNKNOWN = -3, -4, -2


def frame_root_arrays(frame):
    """hgx_reset / hgo_reset arguments from a frame's roots."""
    idx = [r[2] for r in frame["roots"]]
    rnd = [r[3] for r in frame["roots"]]
    yev = [0 if r[1] == -1 else 1 for r in frame["roots"]]
    return idx, rnd, yev


def frame_others_keys(t, frame):
    """The ids (32-byte hashes) of the events the frame's Root.Others maps hold (source gids of
    trace t), for hgx_set_root_others."""
    keys = sorted(frame["others"])
    return np.asarray(t.hash, np.uint8).reshape(-1, 32)[np.asarray(keys, np.int64)] if keys else \
        np.zeros((0, 32), np.uint8)


def remap_after_reset(t, order, frame, new=None):
    """The source events `order` (source gids, topological) as a trace to insert into a
    hashgraph reset with `frame`'s roots, parents resolved like InsertEvent does
    (hashgraph.go:404-445): a parent already re-inserted -> its new gid; a self-parent equal to
    the creator's Root.X -> -1; an other-parent equal to Root.Y -> ROOT_Y, or to the event's
    Root.Others entry -> ROOT_OTHER; anything else -> UNKNOWN. `new` (source gid -> new gid)
    carries over between calls. Returns (trace, new)."""
    new = {} if new is None else new
    base = len(new)
    sp_new, op_new = [], []
    for k, src in enumerate(order):
        c = int(t.creator[src])
        rx, ry = frame["roots"][c][0], frame["roots"][c][1]
        sp, op = int(t.sp[src]), int(t.op[src])
        sp_new.append(new[sp] if sp in new else (-1 if sp == rx else UNKNOWN))
        if op == -1:
            op_new.append(-1)
        elif op in new:
            op_new.append(new[op])
        elif op == ry:
            op_new.append(ROOT_Y)
        elif frame["others"].get(src) == op:
            op_new.append(ROOT_OTHER)
        else:
            op_new.append(UNKNOWN)
        new[src] = base + k
    sel = np.asarray(order, np.int64)
    cols = dict(creator=t.creator[sel], index=t.index[sel], sp=np.array(sp_new, np.int64),
                op=np.array(op_new, np.int64), ts=t.ts[sel], hash=t.hash[sel], s=t.s[sel], ntx=t.ntx[sel],
                txnil=t.txnil[sel])
    if hasattr(t, "tx_seq"):
        sub = type(t)(t.n, tx_seq=t.tx_seq[sel], **cols)
    else:
        sub = Trace(n=t.n, txs=[t.txs[int(x)] for x in sel],
                    names=[t.names[int(x)] for x in sel] if t.names else [], **cols)
    return sub, new
