"""C-ABI checks that need no GPU: the library loads, exports every entry point
include/hgx.h declares, and refuses to run without an MI355X (no CPU fallback).
Also the product-side Go block encoder against the oracle's independent one."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import hgref
from babble_amd import _lib

HDR = os.path.join(hgref.ROOT, "include", "hgx.h")


def declared():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hgx_[a-z0-9_]+)\s*\(", src)))


def test_exports_every_declared_symbol():
    L = _lib.lib()
    names = declared()
    assert len(names) >= 40
    missing = [nm for nm in names if not hasattr(L, nm)]
    assert not missing, missing


def test_abi_version():
    assert _lib.lib().hgx_abi_version() == 6


def test_create_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    err = _lib.hgx_error()
    ctx = _lib.lib().hgx_create(4, 16, 0, C.byref(err))
    assert not ctx
    assert err.code == 200 and b"hgx_create" in err.msg


def test_block_hash_product_vs_oracle_encoder():
    from babble_amd.hashgraph import block_hash
    cases = [(1, [b"e21"], False), (3, [], True), (3, [], False), (7, [b"", b"x" * 100, b"abc"], False),
             (123456, [bytes(range(256))] * 5, False)]
    for rr, txs, nil in cases:
        assert block_hash(rr, txs, nil) == hgref.sha256(hgref.go_block_json(rr, txs, nil))


def test_trace_generator_deterministic():
    from babble_amd import trace
    a = trace.gossip(8, 500, 42, n_silent=2, stale_prob=0.3, stale_depth=3)
    b = trace.gossip(8, 500, 42, n_silent=2, stale_prob=0.3, stale_depth=3)
    for f in ("creator", "index", "sp", "op", "ts", "hash", "s", "ntx", "txnil"):
        assert np.array_equal(getattr(a, f), getattr(b, f))
    assert (a.creator < 6).all()                      # silent peers never create
    assert a.creator[:6].tolist() == list(range(6))   # genesis first
    # self-parent chain is consecutive per creator
    for c in range(6):
        idx = np.where(a.creator == c)[0]
        assert a.index[idx].tolist() == list(range(len(idx)))
        assert a.sp[idx[1:]].tolist() == idx[:-1].tolist()
    assert trace.payload(3, 17) == b"p003 tx 00000017"


def test_sha256_batch_validates_then_fails_loudly_without_gpu():
    import torch
    from babble_amd.hashgraph import sha256_batch
    with pytest.raises(_lib.HgxError) as ei:
        sha256_batch(np.zeros(4, np.uint8), np.array([0, 3, 2], np.int64))
    assert ei.value.code == 102 and "non-decreasing" in str(ei.value)
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_lib.HgxError) as ei:
        sha256_batch(np.zeros(4, np.uint8), np.array([0, 2, 4], np.int64))
    assert "no CPU fallback" in str(ei.value)
