"""Batched ECDSA P-256 verify on the GPU (hgx_p256_verify_batch, Event.Verify event.go:142-152)
against libcrypto's answers (tests/golden/p256_vectors.txt, oracle/p256_ref.c): valid
signatures, malleated s, digests 0 / N / 2^256-1, single-bit corruptions of digest, r and s,
the wrong key, r or s out of [1, N-1], and public keys that are not curve points."""
import numpy as np
import pytest

from test_p256_fixtures import load_vectors

pytestmark = pytest.mark.gpu


def _batch(rows):
    keys, kid, cols = [], [], ([], [], [])
    for pub, dg, r, s, *_ in rows:
        if pub not in keys:
            keys.append(pub)
        kid.append(keys.index(pub))
        for c, v in zip(cols, (dg, r, s)):
            c.append(np.frombuffer(v, np.uint8))
    return (np.stack([np.frombuffer(k, np.uint8) for k in keys]), np.array(kid, np.int32),
            *[np.stack(c) for c in cols])


def _expected(rows):
    return np.array([e if kok else 2 for _, _, _, _, e, kok, _ in rows], np.uint8)


def test_verify_matches_libcrypto():
    from babble_amd.hashgraph import p256_verify
    rows = load_vectors()
    got = p256_verify(*_batch(rows))
    exp = _expected(rows)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, [(int(i), rows[i][6], int(got[i]), int(exp[i])) for i in bad[:20]]


def test_verify_large_batch_and_bench_entry():
    """Many signatures over few keys (a sync batch), shuffled; the bench entry's results too."""
    from babble_amd.hashgraph import p256_verify, p256_verify_bench
    rows = load_vectors()
    rng = np.random.default_rng(7)
    sel = rng.integers(0, len(rows), 20000)
    big = [rows[i] for i in sel]
    cols = _batch(big)
    exp = _expected(big)
    assert np.array_equal(p256_verify(*cols), exp)
    r = p256_verify_bench(*cols, warmup=1, iters=2)
    assert np.array_equal(r["out"], exp) and r["ms_per_launch"] > 0


def test_empty_and_bad_key_index():
    from babble_amd.hashgraph import p256_verify
    rows = load_vectors()[:4]
    keys, kid, dg, r, s = _batch(rows)
    kid = kid.copy()
    kid[0] = 99   # no such key
    out = p256_verify(keys, kid, dg, r, s)
    assert out[0] == 2
