"""C3's mode: one graph row-sharded over ranks (hgx_set_shard). Two gloo ranks
(child processes) share the GPU; each computes the consensus timestamps of its half of the
creators and all-gathers them between FindOrder's halves. Their results must be bit-exact with
the unsharded single-context run and with the oracle."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import hgref
from babble_amd import trace as gtrace

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("n,E,chunk", [(64, 12000, 12000), (256, 30000, 3000)])
def test_row_sharded_world2_bit_exact(tmp_path, n, E, chunk):
    from babble_amd.hashgraph import Hashgraph
    world, port = 2, _port()
    outs = [str(tmp_path / f"r{r}.npz") for r in range(world)]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "shard_worker.py"), str(r), str(world), str(port),
                               outs[r], str(n), str(E), str(chunk)], env=env) for r in range(world)]
    try:
        rcs = [p.wait(timeout=200) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0] * world, rcs
    t = gtrace.gossip(n, E, 77, stale_prob=0.1, stale_depth=2)
    h = Hashgraph(n, capacity=E)
    for lo in range(0, E, chunk):
        h.insert_trace(t, lo, min(E, lo + chunk))
        h.RunConsensus()
    ref = h.results()
    o = hgref.oracle_run(t, chunk=chunk).results()
    assert list(ref["order"]) == list(o["order"])
    for r in range(world):
        z = np.load(outs[r])
        assert list(z["order"]) == list(ref["order"]), r
        for k in ("rr", "cts", "round"):
            assert np.array_equal(z[k], np.asarray(ref[k])), (r, k)
    assert len(ref["order"]) > 0
