"""Parity of the batched device SHA-256 (hgx_sha256_batch) with the
CPU digest the reference's crypto.SHA256 computes (crypto/utils.go:11-16).

The checker is hashlib (FIPS 180-4 SHA-256, the same function Go's crypto/sha256
implements) plus the FIPS known answers; event bodies come from the oracle's Go-JSON
encoder (oracle/goenc.c, the Event.Marshal restatement of hashgraph/event.go:155-162),
so the ids match the fixture events' ids (hashgraph/event.go:171-188). Bit-exact."""
import hashlib

import numpy as np
import pytest

import hgref

pytestmark = pytest.mark.gpu


def _pack(msgs):
    lens = np.array([len(m) for m in msgs], dtype=np.int64)
    off = np.zeros(len(msgs) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    return np.frombuffer(b"".join(msgs), dtype=np.uint8).copy(), off


def _check(msgs):
    from babble_amd.hashgraph import sha256_batch
    data, off = _pack(msgs)
    got = sha256_batch(data, off)
    want = np.frombuffer(b"".join(hashlib.sha256(m).digest() for m in msgs), dtype=np.uint8).reshape(-1, 32)
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, [(int(i), len(msgs[i])) for i in bad[:10]]


def test_fips_known_answers():
    from babble_amd.hashgraph import sha256_batch
    msgs = [b"", b"abc", b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq"]
    want = ["e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855",
            "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad",
            "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"]
    data, off = _pack(msgs)
    got = sha256_batch(data, off)
    assert [bytes(r).hex() for r in got] == want


def test_padding_boundaries_and_unaligned_starts():
    rng = np.random.default_rng(7)
    lens = list(range(0, 260)) + [447, 448, 503, 504, 511, 512, 513, 1000, 4095, 4096, 4097]
    msgs = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]
    _check(msgs)
    _check(msgs[::-1])           # every start alignment with every length class


def test_fixture_event_ids(plays):
    """Event ids of every reference fixture event (hashgraph_test.go plays) hashed on the GPU."""
    from babble_amd.hashgraph import event_ids
    checked = 0
    for name, fx in plays.items():
        if not isinstance(fx, dict) or "plays" not in fx:
            continue
        checked += 1
        fac = hgref.EventFactory(name, fx["n"])
        evs, hexes = [], {}
        for p, (nm, pl) in enumerate(fx["genesis"]):
            e = fac.make(p, 0, "", "", hgref._payload(pl), nm)
            hexes[nm] = e["hex"]
            evs.append(e)
        for to, index, spn, opn, nm, pl in fx["plays"]:
            e = fac.make(to, index, hexes[spn] if spn else "", hexes[opn] if opn else "", hgref._payload(pl), nm)
            hexes[nm] = e["hex"]
            evs.append(e)
        ids = event_ids([e["json"] for e in evs])
        assert ids == [e["hash"] for e in evs], name
        assert ["0x" + i.hex().upper() for i in ids] == [e["hex"] for e in evs]
    assert checked >= 4


def test_block_json_digests_match_block_hash():
    from babble_amd.hashgraph import block_hash, event_ids
    cases = [(1, [b"e21"], False), (3, [], True), (7, [b"", b"x" * 100, b"abc"], False),
             (123456, [bytes(range(256))] * 5, False)]
    bodies = [hgref.go_block_json(rr, txs, nil) for rr, txs, nil in cases]
    assert event_ids(bodies) == [block_hash(rr, txs, nil) for rr, txs, nil in cases]


def test_large_batch_event_sized():
    rng = np.random.default_rng(11)
    lens = rng.integers(300, 720, 200_000)
    blob = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8).tobytes()
    msgs, o = [], 0
    for n in lens:
        msgs.append(blob[o:o + n])
        o += n
    _check(msgs)


def test_empty_batch_and_device_resident_bench_entry():
    from babble_amd.hashgraph import sha256_batch, sha256_bench, sha256_bench_messages
    assert sha256_batch(np.zeros(0, np.uint8), np.zeros(1, np.int64)).shape == (0, 32)
    r = sha256_bench(5000, 0, 300, seed=9, warmup=1, iters=2, n_sample=300)
    msgs = sha256_bench_messages(300, 0, 300, 9)
    assert [bytes(d) for d in r["sample"]] == [hashlib.sha256(m).digest() for m in msgs]
    assert r["ms_per_launch"] > 0 and r["bytes"] > 0
