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


@pytest.mark.parametrize("n,E,chunk", [(64, 12000, 4000), (256, 30000, 30000)])
def test_shard_exchange_through_torch_device_tensors(n, E, chunk):
    """The RCCL path of bench.py --sharded hands torch-allocated device buffers to
    hgx_shard_export / hgx_shard_import (dst_on_device = 1). torch bundles its own HIP and HSA
    runtimes; babble_amd loads torch first, so libhgx binds to that same runtime (one HIP
    runtime per process), and the exchange touches the buffers from a kernel only
    (k_cts_shard_copy). Two ranks' contexts in one process exchange through torch tensors on the
    GPU; every rank's export read back by torch equals its host-pointer export, and both ranks'
    results are bit-exact with the unsharded context. The process maps exactly one HIP runtime."""
    import ctypes as C
    import torch
    from babble_amd.hashgraph import Hashgraph
    world = 2
    t = gtrace.gossip(n, E, 77, stale_prob=0.1, stale_depth=2)
    hs = []
    for r in range(world):
        h = Hashgraph(n, capacity=E)
        h.set_shard(r, world)
        hs.append(h)
    ref = Hashgraph(n, capacity=E)
    dev = torch.device("cuda", 0)
    for lo in range(0, E, chunk):
        hi = min(E, lo + chunk)
        ref.insert_trace(t, lo, hi)
        ref.RunConsensus()
        err = C.create_string_buffer(256)
        for h in hs:
            h.insert_trace(t, lo, hi)
            h.DivideRounds()
            h.DecideFame()
            assert h.L.hgx_find_order_begin(h.ctx, err) == 0
        counts = [int(hs[0].L.hgx_shard_values(hs[0].ctx, r)) for r in range(world)]
        assert counts == [int(hs[1].L.hgx_shard_values(hs[1].ctx, r)) for r in range(world)]
        bufs = []
        for r, h in enumerate(hs):
            d = torch.full((max(1, counts[r]),), -7, dtype=torch.int64, device=dev)
            torch.cuda.synchronize()
            if counts[r]:
                assert h.L.hgx_shard_export(h.ctx, C.c_void_p(d.data_ptr()), 1) == 0
                host = np.zeros(counts[r], np.int64)
                assert h.L.hgx_shard_export(h.ctx, host.ctypes.data_as(C.c_void_p), 0) == 0
                assert np.array_equal(d[:counts[r]].cpu().numpy(), host), r
            bufs.append(d)
        for r, h in enumerate(hs):
            for q in range(world):
                if q != r and counts[q]:
                    src = bufs[q].clone()   # a fresh torch allocation, read by libhgx's kernel
                    torch.cuda.synchronize()
                    assert h.L.hgx_shard_import(h.ctx, q, C.c_void_p(src.data_ptr()), 1) == 0
            assert h.L.hgx_find_order_end(h.ctx, err) == 0
    want = ref.results()
    assert len(want["order"]) > 0
    for r, h in enumerate(hs):
        got = h.results()
        assert list(got["order"]) == list(want["order"]), r
        for k in ("rr", "cts", "round"):
            assert np.array_equal(np.asarray(got[k]), np.asarray(want[k])), (r, k)
    maps = open(f"/proc/{os.getpid()}/maps").read()
    libs = sorted({ln.split()[-1] for ln in maps.splitlines() if "libamdhip64" in ln})
    print("HIP runtimes mapped:", libs)
    assert len(libs) == 1, libs   # one HIP runtime in the process (babble_amd._lib._one_hip_runtime)


# ---- the chain-sharded recurrence (hgx_create_sharded / hgx_set_round_shards) ---------
# W shard contexts in one process, each holding the whole DAG; shard k builds its chains' events'
# firstDescendants, launches its chains' workgroups of the persistent recurrence (candidate rows and
# granules written into every shard's window), computes its events' consensus timestamps. Here every
# shard is on device 0 (the box has one GPU): the same code as shards on separate devices, whose windows
# are peer-mapped.
@pytest.mark.parametrize("n,E,seed,shards,chunk", [(64, 16000, 81, 2, None), (256, 30000, 83, 2, None),
                                                   (256, 24000, 85, 2, 6000)])
def test_chain_sharded_recurrence_rehearsal(n, E, seed, shards, chunk):
    """W shard contexts whose persistent launches over disjoint chain blocks (on W streams) hand
    candidate rows and granules to each other through the shards' windows: bit-exact with the single
    context and with the oracle, no fallback."""
    from babble_amd.hashgraph import Hashgraph
    t = gtrace.gossip(n, E, seed, stale_prob=0.1, stale_depth=3)

    def run(w):
        h = Hashgraph(n, capacity=E)
        h.set_round_shards(w)
        if w == 1:
            h.set_round_kernel("persistent")
        for lo in range(0, E, chunk or E):
            h.insert_trace(t, lo, min(E, lo + (chunk or E)))
            h.RunConsensus()
        return h

    hs, h1 = run(shards), run(1)
    ph = hs.phase_times()
    assert ph["round_p_runs"] > 0 and ph["round_p_fallbacks"] == 0, ph
    a, b = hs.results(), h1.results()
    for k in ("round", "witness", "famous", "rr", "cts"):
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k
    assert list(a["order"]) == list(b["order"])
    o = hgref.oracle_run(t, chunk).results() if chunk else hgref.oracle_run(t).results()
    for k in ("round", "rr", "cts"):
        assert np.array_equal(np.asarray(a[k]), np.asarray(o[k])), k
    assert list(a["order"]) == list(o["order"])


def _rehearse(n, E, seed, shards, remote=0, chunk=0):
    env = dict(os.environ, GPU_MAX_HW_QUEUES=str(shards + 4), PYTHONPATH=os.pathsep.join([HERE, os.path.dirname(HERE)]))
    r = subprocess.run([sys.executable, os.path.join(HERE, "shard_rehearsal_worker.py"), str(n), str(E), str(seed),
                        str(shards), str(remote), str(chunk)], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("OK"), (r.stdout[-2000:], r.stderr[-3000:])


@pytest.mark.parametrize("n,E,seed,shards", [(64, 16000, 82, 4), (256, 30000, 84, 4), (256, 30000, 86, 8)])
def test_chain_sharded_recurrence_rehearsal_more_streams(n, E, seed, shards):
    """W = 4, 8 shard streams: a child process with GPU_MAX_HW_QUEUES = W + 4 (one hardware queue
    per shard, so the shards' workgroups are resident together)."""
    _rehearse(n, E, seed, shards)


@pytest.mark.parametrize("n,E,seed,shards,chunk", [(64, 16000, 87, 3, 0), (64, 16000, 88, 5, 4000),
                                                   (200, 30000, 89, 7, 0), (100, 20000, 90, 6, 5000)])
def test_chain_sharded_uneven_chain_blocks(n, E, seed, shards, chunk):
    """Shard chain blocks of unequal size (W does not divide the chains: C k / W rounds down), one-shot
    and chunked: every split-dependent piece -- the firstDescendants target range, the recurrence's
    workgroups, the timestamp tiles of a block and the exchange offsets -- must agree on the split.
    (On ONE device, 256 chains in W = 6 or 7 launches do not all become resident -- every workgroup
    waits, gives up and the steps run, bit-exact -- while W = 2, 4, 8 do; tools/gpurun/r06_diag_w7.sh.
    An 8-GPU node runs one shard per device.)"""
    _rehearse(n, E, seed, shards, 0, chunk)


@pytest.mark.parametrize("n,E,seed,shards,chunk", [(64, 16000, 82, 2, 0), (64, 16000, 82, 4, 0),
                                                   (256, 30000, 86, 8, 0), (256, 24000, 85, 4, 6000),
                                                   (100, 20000, 90, 3, 5000)])
def test_chain_sharded_cross_device_instructions(n, E, seed, shards, chunk):
    """hgx_set_shard_remote: every other shard's window is written through the cross-device path
    (system-scope sc0 sc1 stores of the candidate rows and granules, as into a peer-mapped window on
    another GPU; the round rows and timestamps always go through the device-to-device copies), so the
    one-GPU box executes the instructions an 8-GPU node's shards execute: bit-exact with one context
    and the oracle, no fallback."""
    _rehearse(n, E, seed, shards, 1, chunk)


@pytest.mark.parametrize("n,E,seed,chunk", [(64, 12000, 91, None), (256, 24000, 93, 4000)])
def test_sharded_context_device_placement(n, E, seed, chunk):
    """hgx_create_sharded with an explicit device per shard (both 0 here): the drop-in calls on the
    one handle, bit-exact with a plain context and the oracle (rounds, witnesses, fame, round
    received, timestamps, order, blocks, UndecidedRounds, LastConsensusRound)."""
    from babble_amd.hashgraph import Hashgraph
    t = gtrace.gossip(n, E, seed, stale_prob=0.1, stale_depth=2)
    hs = Hashgraph(n, capacity=E, shard_devices=[0, 0])
    h1 = Hashgraph(n, capacity=E)
    for lo in range(0, E, chunk or E):
        hi = min(E, lo + (chunk or E))
        for h in (hs, h1):
            h.insert_trace(t, lo, hi)
            h.RunConsensus()
    ph = hs.phase_times()
    assert ph["round_p_runs"] > 0 and ph["round_p_fallbacks"] == 0, ph
    a, b = hs.results(), h1.results()
    for k in ("round", "witness", "famous", "rr", "cts"):
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k
    for k in ("order", "undecided", "lcr", "lcre", "last_round"):
        assert list(np.atleast_1d(a[k])) == list(np.atleast_1d(b[k])), k
    assert hs.Blocks() == h1.Blocks()
    o = hgref.oracle_run(t, chunk).results() if chunk else hgref.oracle_run(t).results()
    assert list(a["order"]) == list(o["order"])
    assert len(a["order"]) > 0


def test_sharded_context_rules():
    """What a chain-sharded context refuses: shards beyond the hardware queues of a shared device, an
    insert before the shards are set up, batched graphs, and the calls it does not serve."""
    import ctypes as C
    from babble_amd.hashgraph import Hashgraph
    from babble_amd._lib import HgxError
    q = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    h = Hashgraph(16, capacity=1000)
    with pytest.raises(ValueError):
        h.set_round_shards(q - 1)   # q - 1 shards on one device need q + 1 queues
    t = gtrace.gossip(16, 500, 5)
    h.insert_trace(t, 0, 100)
    with pytest.raises(ValueError):
        h.set_round_shards(2)       # not on a context holding events
    with pytest.raises(ValueError):
        Hashgraph(16, capacity=1000, n_graphs=2, shard_devices=[0, 0])
    hs = Hashgraph(16, capacity=1000, shard_devices=[0, 0])
    err = C.create_string_buffer(256)
    assert hs.L.hgx_find_order_begin(hs.ctx, err) != 0
    assert hs.L.hgx_set_shard(hs.ctx, 0, 2) != 0
    with pytest.raises(HgxError):
        hs.Reset(np.zeros(16, np.int32), np.zeros(16, np.int32), np.zeros(16, np.int32))
    hs.insert_trace(t)
    hs.RunConsensus()
    h1 = Hashgraph(16, capacity=1000)
    h1.insert_trace(t)
    h1.RunConsensus()
    assert list(hs.results()["order"]) == list(h1.results()["order"])
    with pytest.raises(ValueError):
        hs.set_round_shards(1)      # back to one context is refused too: it holds events


def test_bench_sharded_line():
    """bench.py --sharded: C3's single-graph mode in one process, the recurrence chain-sharded over
    --gpus devices (two shards on the box's one GPU), full-size property checks on the result."""
    import json
    root = os.path.dirname(HERE)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--sharded", "--gpus", "2", "--config", "c2",
                        "--steps", "2", "--warmup", "1"], capture_output=True, text=True, timeout=300, cwd=root)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["shards"] == 2 and line["scaling"] == "strong" and line["value"] > 0, line
    assert line["checks"]["full_size"]["result"] == "pass"
    ph = line["config"]["phase_ms_last_step"]
    assert ph["round_p_runs"] > 0 and ph["round_p_fallbacks"] == 0, ph
