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


def test_libcrypto_verifies_the_256_key_pool(tmp_path):
    """tests/golden/p256_pool256.npz (bench.py insert_verify at c3's 256 keys; written by
    tests/golden/make_p256_pool.py through libcrypto): every signature re-verified by libcrypto."""
    import numpy as np
    try:
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "p256_ref"])
    except (OSError, subprocess.CalledProcessError) as e:
        pytest.skip(f"cannot build oracle/p256_ref (gcc + libcrypto): {e}")
    z = np.load(os.path.join(ROOT, "tests", "golden", "p256_pool256.npz"))
    keys, dg, r, s = z["keys"], z["digest"], z["r"], z["s"]
    assert keys.shape == (256, 65) and dg.shape == (256, 16, 32) and len({k.tobytes() for k in keys}) == 256
    f = tmp_path / "pool.txt"
    with open(f, "w") as o:
        for k in range(256):
            for i in range(16):
                o.write(f"{keys[k].tobytes().hex()} {dg[k, i].tobytes().hex()} {r[k, i].tobytes().hex()} "
                        f"{s[k, i].tobytes().hex()} 1 1 pool\n")
    out = subprocess.run([os.path.join(ROOT, "oracle", "p256_ref"), "check", str(f)], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
