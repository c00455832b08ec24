"""Generates tests/golden/p256_pool256.npz: a signature pool for bench.py's insert_verify leg at
c3's key footprint (256 participants, one P-256 key each, 16 valid signatures per key over
seeded random digests), signed by libcrypto (oracle/p256_ref sign: derived keys
SHA-256("hgx test key" | k) mod N, random nonces). tests/test_p256_fixtures.py re-verifies every
signature with libcrypto.  python tests/golden/make_p256_pool.py"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import hgref  # noqa: E402

K, PER = 256, 16
rng = np.random.default_rng(20251018)
dig = rng.integers(0, 256, (K * PER, 32), dtype=np.uint8)
kid = np.repeat(np.arange(K, dtype=np.uint32), PER)
keys, r, s = hgref.sign_batch(K, kid, dig)
np.savez_compressed(os.path.join(HERE, "p256_pool256.npz"), keys=keys, digest=dig.reshape(K, PER, 32),
                    r=r.reshape(K, PER, 32), s=s.reshape(K, PER, 32))
print("wrote", K, "keys x", PER, "signatures")
