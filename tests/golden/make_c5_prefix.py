"""Golden digests of the CPU oracle (tests/hgref.py, oracle/) on a prefix of bench.py's c5 workload:
1 024 peers, 341 of them silent, 30% stale other-parents (trace.gossip seed 1), the first E events.
The oracle takes minutes at this size, so the GPU test (tests/test_gpu_round_pb.py) compares against
these SHA-256 digests of every per-event output instead of running it.

    PYTHONPATH=tests python tests/golden/make_c5_prefix.py [E]
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

import hgref
from babble_amd import trace as gtrace

N, SILENT, STALE, DEPTH, SEED = 1024, 341, 0.3, 4, 1
KEYS = ("round", "witness", "famous", "rr", "cts", "order")
SCALARS = ("last_round", "undecided", "lcr", "lcre", "consensus_tx", "pending_loaded")


def digest(a) -> str:
    a = np.ascontiguousarray(np.asarray(a, dtype=np.int64))
    return hashlib.sha256(a.tobytes()).hexdigest()


def summarize(res) -> dict:
    out = {k: digest(res[k]) for k in KEYS}
    for k in SCALARS:
        v = res[k]
        out[k] = v if isinstance(v, (int, str)) or v is None else (list(v) if hasattr(v, "__len__") else int(v))
    return out


def main():
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 150000
    t = gtrace.gossip(N, E, SEED, n_silent=SILENT, stale_prob=STALE, stale_depth=DEPTH)
    t0 = time.time()
    res = hgref.oracle_run(t).results()
    doc = {"workload": "c5 prefix", "n": N, "silent": SILENT, "stale": STALE, "depth": DEPTH, "seed": SEED, "E": E,
           "oracle_s": round(time.time() - t0, 1), "digests": summarize(res)}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c5_prefix.json")
    with open(path, "w") as f:
        json.dump(doc, f, indent=1, default=int)
    print(json.dumps(doc, default=int))


if __name__ == "__main__":
    main()
