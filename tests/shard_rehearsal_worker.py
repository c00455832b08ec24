"""Child process of test_gpu_sharded.py: the chain-sharded recurrence rehearsal with W shard streams,
run where GPU_MAX_HW_QUEUES >= W + 2 was set before the HIP runtime started (each shard's launch
needs a hardware queue of its own: its workgroups wait for the other shards' granules). Prints
"OK <rounds_ms>" when the run is bit-exact with the single persistent launch and the oracle.
argv: n E seed shards [remote [chunk]]: remote = 1 writes the other shards' windows through the
cross-device path (hgx_set_shard_remote); chunk = events per RunConsensus call (0 = one call)."""
import sys

import numpy as np

import hgref
from babble_amd import trace as gtrace
from babble_amd.hashgraph import Hashgraph

n, E, seed, shards = (int(a) for a in sys.argv[1:5])
remote = len(sys.argv) > 5 and sys.argv[5] == "1"
chunk = int(sys.argv[6]) if len(sys.argv) > 6 and int(sys.argv[6]) > 0 else E
t = gtrace.gossip(n, E, seed, stale_prob=0.1, stale_depth=3)


def run(w):
    h = Hashgraph(n, capacity=E)
    h.set_round_shards(w)
    if w == 1:
        h.set_round_kernel("persistent")
    elif remote:
        h.set_shard_remote(True)
    for lo in range(0, E, chunk):
        h.insert_trace(t, lo, min(E, lo + chunk))
        h.RunConsensus()
    return h


hs, h1 = run(shards), run(1)
ph = hs.phase_times()
assert ph["round_p_runs"] > 0 and ph["round_p_fallbacks"] == 0, ph
a, b = hs.results(), h1.results()
for k in ("round", "witness", "famous", "rr", "cts"):
    assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k
assert list(a["order"]) == list(b["order"])
o = (hgref.oracle_run(t, chunk) if chunk < E else hgref.oracle_run(t)).results()
for k in ("round", "rr", "cts"):
    assert np.array_equal(np.asarray(a[k]), np.asarray(o[k])), k
assert list(a["order"]) == list(o["order"])
print("OK", ph["rounds_ms"])
