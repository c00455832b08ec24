"""Golden digests of the CPU oracle (tests/hgref.py -> oracle/hg_oracle.c, the restatement of
hashgraph.go:616-858) over bench.py's WHOLE headline traces, so the GPU tests can pin every
per-event output, the consensus order, the blocks and the block hashes at full size without
running the single-threaded oracle on the box (c3 takes ~25 min of oracle time here, c5 ~40).

    PYTHONPATH=tests:. python tests/golden/make_full_digests.py c3|c5 [E]

Writes tests/golden/<cfg>_full.json (or <cfg>_<E>.json for a prefix). The trace is
bench.make_trace(cfg, rank 0): trace.gossip(n, E, seed 1, ...) with the config's silent peers and
stale other-parents -- exactly what bench.py times.
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

import hgref  # noqa: E402

KEYS = ("round", "witness", "famous", "rr", "cts", "order")
SCALARS = ("last_round", "undecided", "lcr", "lcre", "consensus_tx", "pending_loaded")


def digest(a) -> str:
    a = np.ascontiguousarray(np.asarray(a, dtype=np.int64))
    return hashlib.sha256(a.tobytes()).hexdigest()


def block_digests(blocks) -> dict:
    """blocks: [(rr, ntx, tx_nil, committed, hash32)] in SetBlock order."""
    meta = np.array([[b[0], b[1], int(bool(b[2])), int(bool(b[3]))] for b in blocks] or np.zeros((0, 4)), np.int64)
    h = hashlib.sha256()
    for b in blocks:
        h.update(bytes(b[4]))
    return {"n_blocks": len(blocks), "blocks_meta": digest(meta), "block_hashes": h.hexdigest()}


def summarize(res, with_blocks=True) -> dict:
    out = {k: digest(res[k]) for k in KEYS}
    for k in SCALARS:
        v = res[k]
        out[k] = v if isinstance(v, (int, str)) or v is None else (list(v) if hasattr(v, "__len__") else int(v))
    if with_blocks:
        out.update(block_digests(res["blocks"]))
    return out


def main():
    import bench
    cfg = sys.argv[1]
    n, E_full, G, silent, stale, depth, desc = bench.CONFIGS[cfg]
    assert G == 1, "one graph per config (c1, c2, c3, c5)"
    E = int(sys.argv[2]) if len(sys.argv) > 2 else E_full
    from babble_amd import trace as gtrace
    t = gtrace.gossip(n, E, 1, n_silent=silent, stale_prob=stale, stale_depth=depth)
    t0 = time.time()
    o = hgref.oracle_run(t)
    t_run = time.time() - t0
    res = o.results()
    doc = {"workload": desc if E == E_full else f"{desc}: first {E} events", "config": cfg, "n": n,
           "silent": silent, "stale": stale, "depth": depth, "seed": 1, "E": E,
           "oracle_s": round(t_run, 1), "digests": summarize(res)}
    name = f"{cfg}_full.json" if E == E_full else f"{cfg}_{E}.json"
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(doc, f, indent=1, default=int)
    print(json.dumps({k: v for k, v in doc.items() if k != "digests"}, default=int), flush=True)


if __name__ == "__main__":
    main()
