"""The ECDSA P-256 known answers (tests/golden/p256_vectors.txt) re-checked against the
container's libcrypto by oracle/p256_ref.c (the generator that wrote them). CPU only."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VEC = os.path.join(ROOT, "tests", "golden", "p256_vectors.txt")


def load_vectors():
    rows = []
    with open(VEC) as f:
        for line in f:
            pub, dg, r, s, exp, kok, tag = line.split()
            rows.append((bytes.fromhex(pub), bytes.fromhex(dg), bytes.fromhex(r), bytes.fromhex(s), int(exp),
                         int(kok), tag))
    return rows


def test_vectors_cover_the_cases():
    rows = load_vectors()
    tags = {r[6] for r in rows}
    for t in ("valid", "edge-digest", "malleated-s", "digest-bit", "r-bit", "s-bit", "other-key", "r-zero",
              "s-zero", "r-eq-N", "s-eq-N", "r-gt-N", "key-off-curve", "key-x-ge-p", "key-bad-prefix"):
        assert t in tags, t
    assert sum(r[4] for r in rows) >= 150 and sum(1 - r[4] for r in rows) >= 500


def test_libcrypto_agrees_with_vectors():
    try:
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "p256_ref"])
    except (OSError, subprocess.CalledProcessError) as e:
        pytest.skip(f"cannot build oracle/p256_ref (gcc + libcrypto): {e}")
    out = subprocess.run([os.path.join(ROOT, "oracle", "p256_ref"), "check", VEC], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
