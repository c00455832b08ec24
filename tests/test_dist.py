"""Multi-rank path of bench.py on CPU (gloo, world_size 2): one seed-sharded replica per
rank, no data-path collective; ranks only barrier and reduce the timing (max) and the
ordered-event counts (sum). DESIGN.md §6."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import bench
    import hgref
    red = bench.Reducer(world, rank, backend="gloo")
    tr, G = bench.make_trace("c1", rank)
    o = hgref.oracle_run(tr)          # each rank's replica, checked by the CPU oracle
    ordered = len(o.consensus_events())
    red.barrier()
    t_max = red.max(float(rank + 1))
    total = red.sum(float(ordered))
    out[rank] = (int(tr.creator.sum() + tr.op.sum()), ordered, t_max, total)
    red.dist.destroy_process_group()


def test_bench_reducer_gloo_world2():
    world, port = 2, _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    r0, r1 = out[0], out[1]
    assert r0[0] != r1[0], "ranks must get different (seed-sharded) traces"
    assert r0[1] > 0 and r1[1] > 0
    assert r0[2] == r1[2] == 2.0                      # max over ranks of rank+1
    assert r0[3] == r1[3] == float(r0[1] + r1[1])     # whole-job ordered events


def test_reducer_single_rank_is_identity():
    import bench
    red = bench.Reducer(1)
    red.barrier()
    assert red.max(3.5) == 3.5 and red.sum(7.0) == 7.0


def test_bench_self_launch_without_launcher():
    """`bench.py --gpus 2` with no torch.distributed.run around it starts the launcher itself (a child
    process) instead of printing a one-GPU line: both ranks meet and reduce over gloo (no GPU here)."""
    import json
    import subprocess
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]   # rank 0 prints the one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_reporting"] == 2 and d["max_rank"] == 1.0 and d["backend"] == "gloo"


def test_bench_refuses_mismatched_launcher():
    """Under a launcher, --gpus must equal the ranks it started (never a line whose n_gpus disagrees)."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--launch-check"],
                       capture_output=True, text=True, timeout=120, cwd=ROOT, env=env)
    assert r.returncode != 0 and "launcher started 2 ranks" in r.stderr
