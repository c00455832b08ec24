#!/usr/bin/env python3
"""bench.py -- consensus-ordered events/sec of the MI355X Hashgraph engine.

Workload (BASELINE.json metric "consensus-ordered events/sec at N=256 peers"): one synthetic
random-gossip hashgraph per GPU (configs[2]: 256 peers, 10M events, fits one MI355X), seeded
per rank (weak scaling: independent 256-peer simulations, no data-path collective --
DESIGN.md §6). The trace is in host RAM when the clock starts. A step is one whole pass of
the hot path, from the first event append to the order in host memory:

    hgx_clear -> hgx_insert_and_run: InsertEvent for every event (the event columns copied to
    HBM, parent/index validation + append on the GPU) -> DivideRounds -> DecideFame -> FindOrder,
    in one call (Bootstrap, hashgraph.go:1008-1037); the payload columns (timestamps, hash, S,
    transactions) are copied while DivideRounds runs

Side legs on the same line: the step with the columns already in HBM (hbm_resident), the
SyncLimit-chunked schedule (chunked_sync), event ids (ingest_sha256), signature checks
(ingest_p256_verify), and the InsertEvent pass with Event.Verify (insert_verify).

After the timed steps (outside the clock) the run is checked: the GPU against the CPU oracle
on a prefix of the same trace (every output, bit-exact), and the full-size result against
the order properties the reference guarantees (a permutation of the received events sorted
by (round received, consensus timestamp, S), rounds monotone along every chain, blocks
consistent). A failed check exits non-zero without a result line.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c1|c2|c4|c5]
  (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N; without a launcher,
  --gpus N > 1 starts that launcher itself as a child process before any GPU call and exits with
  its status, so the line always carries N ranks' work)

At N > 1 the line also carries `sharded`: C3's single-graph mode (one graph whose round recurrence is
chain-sharded over all N devices, hgx_create_sharded) timed by rank 0 in a child process
after every rank has released its GPU memory (the other ranks wait on the host).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# what each dominant-kernel candidate is bound by; achieved/peak/frac stay the
# SURVEY 8(d) HBM figures and `valu` carries the issue-rate fraction beside them
BOUND = {
    "round_search": "latency: sequential round recurrence (per round an all-to-all of every chain's candidate "
                    "row, 64 KB into each compute unit, then a 5-level dependent search); neither HBM nor VALU",
    "cts_median": "latency: dependent firstDescendants -> timestamp gathers",
    "fd_build": "VALU issue per (tile, target chain)",
}

CONFIGS = {
    # name: (n, events per graph, graphs per GPU, silent, stale_prob, stale_depth, description)
    "c1": (4, 1024, 1, 0, 0.0, 1, "4 peers, 1,024 gossip events"),
    "c2": (64, 1 << 20, 1, 0, 0.0, 1, "64 peers, 1,048,576 gossip events, one hashgraph"),
    "c3": (256, 10_000_000, 1, 0, 0.0, 1, "256 peers, 10,000,000 gossip events, one hashgraph per GPU"),
    "c4": (16, 16384, 512, 0, 0.0, 1, "512 independent 16-peer sims x 16,384 events per GPU (4096 over 8 GPUs)"),
    "c5": (1024, 1 << 20, 1, 341, 0.3, 4, "1024 peers (341 = 1/3 silent, 30% stale other-parents), 1,048,576 events"),
}

# oracle sample (events of graph 0's trace) for the prefix parity check and the CPU baseline:
# about 10-30 s of single-threaded oracle work
SAMPLE = {4: 1024, 16: 16384, 64: 100_000, 256: 100_000, 1024: 16_000}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_trace(cfg, rank):
    from babble_amd import trace
    n, E, G, silent, stale, depth, _ = CONFIGS[cfg]
    seeds = [1 + rank * G + g for g in range(G)]
    if G == 1:
        return trace.gossip(n, E, seeds[0], n_silent=silent, stale_prob=stale, stale_depth=depth), G
    return trace.concat_graphs([trace.gossip(n, E, s, n_silent=silent, stale_prob=stale, stale_depth=depth)
                                for s in seeds]), G


def kernel_bytes(name, n, E, m, compact, sort_passes=1):
    """SURVEY §8(d) algorithmic bytes of one pass, per kernel: E events,
    m events received by the pass, coordinates of `cb` bytes (2 compact, 4 int32); the sort moves
    2 x 44 bytes per consensus event in each of its radix passes."""
    cb = 2 if compact else 4
    return {
        "la_sweep": (3 * cb * n + 16) * E,      # la_build: read 2 parent rows, write the row (12n+16 int32)
        "fd_build": 2 * cb * n * E,             # read LA once, write FD (8n int32)
        "round_search": (4 * n + 16) * E,       # round_assign: 4n+16 per event (witness rows amortised)
        "round_received": 16 * E,
        "cts_median": (cb * n + 8 * n + 12) * m,  # FD row + <= n timestamp gathers + outputs
        "order_sort": 2 * 44 * m * sort_passes,
        "layout": 64 * E,
    }.get(name)


def host_cpu():
    """The host's CPU model (/proc/cpuinfo) and its logical CPU count (nproc)."""
    model = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model, os.cpu_count()


def cpu_baseline(t, n, budget_note, ordered_frac=None):
    """The oracle (single-threaded C restatement of the reference loops, oracle/hg_oracle.c)
    on a bounded prefix of the same workload, timed on this host: InsertEvent (one C batch
    call) + DivideRounds + DecideFame + FindOrder. Returns the baseline and the oracle.
    When the bounded sample decides no round (c5: 1/3 silent peers make a round span ~20 k
    events, so ordering anything takes minutes of oracle time), the rate is a labelled
    extrapolation: the oracle's events/s over the sample times the fraction of
    the full trace a GPU pass orders (ordered_frac), i.e. assuming the CPU cost per event stays
    what the sample measured."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import hgref
    o = hgref.Oracle(n)
    t0 = time.perf_counter()
    o.insert_trace(t)
    o.divide_rounds()
    rc, msg = o.decide_fame()
    if not rc:
        rc, msg = o.find_order()
    dt = time.perf_counter() - t0
    if rc:
        raise RuntimeError(f"oracle consensus failed: {msg}")
    ordered = len(o.consensus_events())
    value, note = (ordered / dt) if ordered else None, ""
    if not ordered and ordered_frac:
        value = t.E / dt * ordered_frac
        note = (f"; no round is decided within the sample, so the value is an EXTRAPOLATION: {t.E / dt:.0f} "
                f"events/s through the oracle x {ordered_frac:.3f} (the fraction of the full trace one GPU pass "
                f"orders)")
    elif not ordered:
        note = " (no round is decided within the sample: no rate is reported)"
    model, nproc = host_cpu()
    base = dict(value=value, unit="consensus-ordered events/s", cores=1, kind="port", cpu_model=model, nproc=nproc,
                sample=f"first {t.E} events of the {budget_note} trace (seed 1), oracle InsertEvent+DivideRounds+"
                       f"DecideFame+FindOrder single-threaded (1 of the host's {nproc} logical CPUs, {model}), "
                       f"{ordered} events ordered in {dt:.2f}s{note}")
    return base, o


def prefix_parity(t, o, device):
    """GPU vs oracle on the same prefix: every output bit-exact (fails loudly)."""
    from babble_amd.hashgraph import Hashgraph
    h = Hashgraph(t.n, capacity=t.E, device=device)
    h.insert_trace(t)
    h.RunConsensus()
    a, b = h.results(), o.results()
    for k in ("round", "witness", "famous", "rr", "cts"):
        if not np.array_equal(np.asarray(a[k]), np.asarray(b[k])):
            bad = np.nonzero(np.asarray(a[k]) != np.asarray(b[k]))[0][:5]
            raise SystemExit(f"PARITY FAILURE on the {t.E}-event prefix: {k} differs at gids {bad.tolist()}")
    if list(a["order"]) != list(b["order"]):
        raise SystemExit(f"PARITY FAILURE on the {t.E}-event prefix: consensus order")
    for k in ("last_round", "undecided", "lcr", "lcre", "consensus_tx", "pending_loaded"):
        if a[k] != b[k]:
            raise SystemExit(f"PARITY FAILURE on the {t.E}-event prefix: {k} {a[k]} != {b[k]}")
    if [(x["rr"], x["ntx"], x["tx_nil"], x["committed"]) for x in a["blocks"]] != [tuple(x[:4]) for x in b["blocks"]]:
        raise SystemExit(f"PARITY FAILURE on the {t.E}-event prefix: blocks")
    # block hashes: SHA256(json(Block)) over the GPU order's transactions (block.go:26-53)
    from babble_amd.hashgraph import block_hash
    order = h.ConsensusEvents()
    gh = []
    for blk in h.Blocks():
        txs = []
        for g in order[blk["first"]:blk["first"] + blk["n_events"]]:
            txs.extend(t.txs(int(g)) or [])
        gh.append(block_hash(blk["rr"], txs, blk["tx_nil"]))
    if gh != [x[4] for x in b["blocks"]]:
        raise SystemExit(f"PARITY FAILURE on the {t.E}-event prefix: block hashes")
    h.close()
    return {"events": int(t.E), "ordered": int(len(b["order"])), "rounds": int(b["last_round"]) + 1,
            "blocks": len(gh),
            "outputs": "round, witness, fame, round received, consensus timestamp, order, UndecidedRounds, "
                       "LastConsensusRound, LastCommitedRoundEvents, counters, blocks, block hashes",
            "result": "bit-exact"}


def full_size_checks(h, tr, G):
    """Order properties of the full-size run (hashgraph.go:753-858, consensus_sorter.go)."""
    E, n = tr.E, tr.n
    rnd, wit, _ = h.rounds()
    rr, cts = h.received()
    creator = tr.creator.astype(np.int64)
    fails = []

    def check(ok, what):
        if not ok:
            fails.append(what)

    # per chain (creator), events in Index order == gid order of that creator
    order_c = np.lexsort((np.arange(E), creator))
    c_sorted = creator[order_c]
    same = c_sorted[1:] == c_sorted[:-1]
    r_c, rr_c = rnd[order_c], rr[order_c]
    check(np.all(r_c[1:][same] >= r_c[:-1][same]), "round non-decreasing along every chain")
    rcv = rr_c >= 0
    check(np.all(~(rcv[1:] & ~rcv[:-1] & same)), "received events of a chain form a prefix")
    check(np.all(rr_c[1:][same & rcv[1:]] >= rr_c[:-1][same & rcv[1:]]), "round received non-decreasing along chains")
    check(np.all(rr[rr >= 0] > rnd[rr >= 0]), "round received > round")
    first = np.ones(E, bool)
    first[1:] = ~same
    check(np.all(wit[order_c][first] == 1), "first event of every chain is a witness")
    sp = tr.sp
    has_sp = sp >= 0
    check(np.all(wit[has_sp] == (rnd[has_sp] > rnd[sp[has_sp]])), "witness iff round > round(self-parent)")
    total = 0
    for g in range(G):
        order = h.ConsensusEvents(g)
        total += len(order)
        in_g = (creator // n) == g
        recv_g = np.nonzero(in_g & (rr >= 0))[0]
        check(len(order) == len(recv_g) and np.array_equal(np.sort(order), recv_g),
              f"graph {g}: order is a permutation of the received events")
        if len(order) < 2:
            continue
        o_rr, o_cts = rr[order], cts[order]
        check(np.all(o_rr[1:] >= o_rr[:-1]), f"graph {g}: round received non-decreasing along the order")
        eq_rr = o_rr[1:] == o_rr[:-1]
        check(np.all(o_cts[1:][eq_rr] >= o_cts[:-1][eq_rr]), f"graph {g}: consensus timestamp non-decreasing "
                                                            "within a round received")
        tie = eq_rr & (o_cts[1:] == o_cts[:-1])
        if tie.any():
            s = tr.s[order]
            a, b = s[:-1][tie], s[1:][tie]
            diff = a != b
            idx = np.argmax(diff, axis=1)
            rows = np.arange(len(idx))
            check(np.all(diff.any(axis=1)) and np.all(a[rows, idx] < b[rows, idx]),
                  f"graph {g}: S strictly increasing within equal (round received, timestamp)")
        blocks = h.Blocks(g)
        check(sum(b["n_events"] for b in blocks) == len(order), f"graph {g}: blocks cover the order")
        check(all(b1["rr"] < b2["rr"] for b1, b2 in zip(blocks, blocks[1:])), f"graph {g}: one block per rr")
        check(sum(b["ntx"] for b in blocks) == h.ConsensusTransactions(g), f"graph {g}: block transactions")
        check(all(int(rr[order[b["first"]]]) == b["rr"] for b in blocks), f"graph {g}: block rr")
    if fails:
        raise SystemExit("FULL-SIZE CHECK FAILURE: " + "; ".join(fails))
    return {"events": int(E), "ordered": int(total),
            "properties": ["order is a permutation of the received events", "rr non-decreasing along the order",
                           "cts non-decreasing within rr", "S strictly increasing within (rr, cts) ties",
                           "round non-decreasing along every chain", "received events form a chain prefix",
                           "rr non-decreasing along chains", "rr > round", "witness iff round > round(sp)",
                           "blocks: one per rr, cover the order, transaction totals"], "result": "pass"}


class Reducer:
    """Timing/count reductions over the ranks of a multi-GPU run (one replica per rank,
    DESIGN.md §6: no data-path collective). backend "nccl" (RCCL) on GPUs; "gloo" keeps
    the same code testable on CPU (tests/test_dist.py)."""

    def __init__(self, world, local_rank=0, backend="nccl"):
        self.world, self.dist, self.device, self.cpu_group = world, None, "cpu", None
        if world > 1:
            import datetime
            import torch
            import torch.distributed as dist
            if backend == "auto":   # RCCL when every rank has a GPU of its own, else gloo (ranks share one)
                backend = "nccl" if torch.cuda.device_count() >= world else "gloo"
            self.backend = backend
            if backend == "nccl":
                torch.cuda.set_device(local_rank)
                dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
                self.device = f"cuda:{local_rank}"
            elif not dist.is_initialized():
                dist.init_process_group(backend)
            self.dist = dist
            # host-side waits (the sharded leg: no collective kernel may sit on a GPU it uses)
            self.cpu_group = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=3600)) \
                if backend != "gloo" else None

    def cpu_barrier(self):
        if self.dist is not None:
            self.dist.barrier(group=self.cpu_group)

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def _reduce(self, x, op):
        if self.dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64, device=self.device)
        self.dist.all_reduce(t, op=op)
        return float(t.item())

    def max(self, x):
        return x if self.dist is None else self._reduce(x, self.dist.ReduceOp.MAX)

    def sum(self, x):
        return x if self.dist is None else self._reduce(x, self.dist.ReduceOp.SUM)

    def shard_exchange(self, h, world, rank):
        """FindOrder of a row-sharded graph (hgx_find_order_begin / _end): the ranks' consensus
        timestamps all-gathered in between, device buffers over RCCL (xGMI), host over gloo."""
        import ctypes as C
        import torch
        err = C.create_string_buffer(256)
        L = h.L
        if L.hgx_find_order_begin(h.ctx, err):
            raise SystemExit("hgx_find_order_begin failed")
        counts = [int(L.hgx_shard_values(h.ctx, r)) for r in range(world)]
        mx = max(1, max(counts))
        on_dev = self.device != "cpu"
        mine = torch.zeros(mx, dtype=torch.int64, device=self.device)
        if counts[rank] and L.hgx_shard_export(h.ctx, C.c_void_p(mine.data_ptr()), 1 if on_dev else 0):
            raise SystemExit("hgx_shard_export failed")
        allv = torch.empty(world * mx, dtype=torch.int64, device=self.device)
        self.dist.all_gather_into_tensor(allv, mine)
        if on_dev:
            torch.cuda.synchronize()
        for r in range(world):
            if r != rank and counts[r]:
                ptr_r = C.c_void_p(allv.data_ptr() + 8 * r * mx)
                if L.hgx_shard_import(h.ctx, r, ptr_r, 1 if on_dev else 0):
                    raise SystemExit("hgx_shard_import failed")
        if L.hgx_find_order_end(h.ctx, err):
            raise SystemExit("hgx_find_order_end failed")


# SHA-256 compression in gfx950 lane instructions per 64-byte block (3-input v_bitop3/v_add3):
# 64 rounds x (6 rotates + 2 xor3 + Ch + Maj + 4 adds) + 48 schedule words x (4 rotates + 2 shifts
# + 2 xor3 + 3 adds); VALU peak = 32 lanes/clk/SIMD x 4 SIMD x 256 CU x 2.4 GHz (MI355X_MICROARCH.md)
SHA_OPS_PER_BLOCK = 64 * 14 + 48 * 11
VALU_PEAK_TOPS = 32 * 4 * 256 * 2.4e9 / 1e12


def ingest_leg(count, steps, warmup, device):
    """Side leg: Event.Hash ids (hashgraph/event.go:171-180) of `count` synthetic
    event bodies of Go-JSON event size (400..560 B, PRNG bytes), HBM-resident, hashed by
    k_sha256_batch; device time per launch from HIP events on the launch stream (hgx_sha256_bench)."""
    import hashlib
    from babble_amd.hashgraph import sha256_bench, sha256_bench_messages
    lo, hi, seed = 400, 560, 5
    r = sha256_bench(count, lo, hi, seed, warmup=max(1, warmup), iters=steps, n_sample=64, device=device)
    msgs = sha256_bench_messages(64, lo, hi, seed)
    assert all(hashlib.sha256(m).digest() == bytes(d) for m, d in zip(msgs, r["sample"])), "SHA-256 mismatch"
    ms = r["ms_per_launch"]
    achieved = r["blocks"] * SHA_OPS_PER_BLOCK / (ms * 1e-3) / 1e12
    return {"kernel": "k_sha256_batch", "events": count, "bytes": r["bytes"], "ms_per_launch": ms,
            "event_ids_per_s": count / (ms * 1e-3), "input_GB_per_s": r["bytes"] / (ms * 1e-3) / 1e9,
            "roofline": {"bound": "valu", "achieved": achieved, "peak": VALU_PEAK_TOPS, "unit": "Tlane-op/s",
                         "frac": achieved / VALU_PEAK_TOPS, "ops_per_block": SHA_OPS_PER_BLOCK,
                         "blocks_per_launch": r["blocks"]}}


def chunked_leg(h, tr, sync_limit, check):
    """The real caller's schedule: Core.Sync inserts at most SyncLimit events
    (cmd/babble/main.go:83-85) and Core.RunConsensus follows every sync (node/core.go:190-303);
    the incremental DivideRounds/FindOrder work on the new events only. Wall clock over the
    whole trace; every sync's events come from host memory, as Core hands them over."""
    import gc
    h.clear()
    h.set_kernel_timing(False)
    calls, worst = 0, 0.0
    per_call = []
    gc.collect()
    gc.disable()   # (a collector pause of this process is not the library's latency: one measured 14.7 ms call)
    t0 = time.perf_counter()
    for lo in range(0, tr.E, sync_limit):
        c0 = time.perf_counter()
        h.insert_trace(tr, lo, min(tr.E, lo + sync_limit))
        c1 = time.perf_counter()
        h.RunConsensus()
        c2 = time.perf_counter()
        per_call.append((c2 - c0, c1 - c0))
        worst = max(worst, c2 - c0)
        calls += 1
    el = time.perf_counter() - t0
    gc.enable()
    # the five slowest calls: (call index, ms, of which insert ms) -- where the outliers sit in the run
    top = sorted(range(calls), key=lambda i: -per_call[i][0])[:5]
    worst_calls = [[i, round(per_call[i][0] * 1e3, 3), round(per_call[i][1] * 1e3, 3)] for i in top]
    ordered = int(h.L.hgx_consensus_events_count(h.ctx, 0))
    res = {"sync_limit": sync_limit, "calls": calls, "events": int(tr.E), "ordered": ordered,
           "value": ordered / el, "unit": "consensus-ordered events/s", "inserted_events_per_s": tr.E / el,
           "ms_per_call": el * 1e3 / calls, "worst_call_ms": worst * 1e3, "seconds": el,
           "worst_calls": worst_calls,
           "p99_call_ms": sorted(x[0] for x in per_call)[int(0.99 * (calls - 1))] * 1e3,
           "note": "RunConsensus after every SyncLimit inserted events; same trace as the headline"}
    if check:
        res["full_size_checks"] = full_size_checks(h, tr, 1)["result"]
    return res


def p256_leg(count, steps, warmup, device):
    """Side leg (second half): Event.Verify (hashgraph/event.go:142-152) of
    `count` signatures over 6 creator keys (a sync batch), drawn from libcrypto's known answers
    (tests/golden/p256_vectors.txt: valid, corrupted and bad-key rows), HBM-resident; device time
    per verify launch from HIP events, the key tables built once before (hgx_p256_verify_bench, as a
    context builds them when its keys are set); every result is
    checked against libcrypto's."""
    from babble_amd.hashgraph import p256_verify_bench
    rows = []
    with open(os.path.join(ROOT, "tests", "golden", "p256_vectors.txt")) as f:
        for line in f:
            pub, dg, r, s, exp, kok, _ = line.split()
            rows.append((pub, dg, r, s, int(exp) if int(kok) else 2))
    keys = sorted({r[0] for r in rows})
    sel = np.random.default_rng(11).integers(0, len(rows), count)
    kid = np.array([keys.index(rows[i][0]) for i in range(len(rows))], np.int32)[sel]
    cols = [np.stack([np.frombuffer(bytes.fromhex(rows[i][c]), np.uint8) for i in range(len(rows))])[sel]
            for c in (1, 2, 3)]
    exp = np.array([r[4] for r in rows], np.uint8)[sel]
    kb = np.stack([np.frombuffer(bytes.fromhex(k), np.uint8) for k in keys])
    res = p256_verify_bench(kb, kid, *cols, warmup=max(1, warmup), iters=steps, device=device)
    assert np.array_equal(res["out"], exp), "P-256 verify differs from libcrypto"
    ms = res["ms_per_launch"]
    out = {"kernel": "k_p256_verify", "signatures": count, "keys": len(keys), "ms_per_launch": ms,
           "verifies_per_s": count / (ms * 1e-3), "valid_fraction": float((exp == 1).mean()),
           "check": "bit-exact vs libcrypto 3.0.2 (ECDSA_do_verify)"}
    # VALU issue roofline from the PMC pass of this leg (tools/gpurun/pmc_p256.sh: SQ_INSTS_VALU
    # over the same 1 M-signature launch): wave instructions x 64 lanes per launch / this line's ms
    vf = os.path.join(ROOT, "profiles", "valu_p256.json")
    try:
        vj = json.load(open(vf)).get("p256_verify") or {}
        if vj.get("valu_insts_per_pass") and vj.get("dispatches") and count == (1 << 20):
            per = vj["valu_insts_per_pass"] / vj["dispatches"]
            ach = 64.0 * per / (ms * 1e-3) / 1e12
            out["roofline"] = {"bound": "valu", "achieved": ach, "peak": VALU_PEAK_TOPS, "unit": "Tlane-op/s",
                               "frac": ach / VALU_PEAK_TOPS, "valu_insts_per_launch": per,
                               "lane_ops_per_verify": 64.0 * per / count,
                               "source": "profiles/valu_p256.json (rocprofv3 --pmc SQ_INSTS_VALU, this leg's launch)"}
    except (OSError, ValueError):
        pass
    return out


def _signature_pool():
    """libcrypto signatures of tests/golden/p256_pool256.npz (tests/golden/make_p256_pool.py): 256
    keys, 16 valid signatures each. Returns keys [K, 65] and digest / r / s [K, 16, 32]."""
    z = np.load(os.path.join(ROOT, "tests", "golden", "p256_pool256.npz"))
    return z["keys"], z["digest"], z["r"], z["s"]


def insert_verify_leg(h, tr, steps, ref, sha_ms, device):
    """InsertEvent with Event.Verify (hashgraph.go:356-363, event.go:142-152) over the whole
    headline trace: clear -> hgx_insert_events_verified_device (batched P-256 verify of every
    event merged with the parent/index checks' first-failure rule) -> DivideRounds -> DecideFame
    -> FindOrder, columns HBM-resident. Participant c signs with its own libcrypto key c % 256 (c3:
    256 distinct keys, the context's key footprint: 256 comb tables) and event (c, Index) carries
    that key's signature number Index % 16 (the S column is the signature's S, so the consensus
    tie-break runs on these S). Checked: every event is accepted, and rounds / round received /
    timestamps equal the headline run's (they do not depend on S). `ref` = (rr, cts) of the
    headline run."""
    from babble_amd.hashgraph import DeviceBuffer, DeviceTrace
    from babble_amd import trace as gtrace
    pk, pdig, pr, ps = _signature_pool()
    nk, per = pk.shape[0], pdig.shape[1]
    keys = np.stack([pk[c % nk] for c in range(h.n)])
    kk = (tr.creator % h.n) % nk
    pick = tr.index % per
    dig = np.ascontiguousarray(pdig[kk, pick])
    sr = np.ascontiguousarray(pr[kk, pick])
    ss = np.ascontiguousarray(ps[kk, pick])
    t2 = gtrace.GossipTrace(**{**tr.__dict__, "s": ss})
    dtr, dd, dr = DeviceTrace(t2, device=device), DeviceBuffer(dig, device), DeviceBuffer(sr, device)
    del dig, sr, ss
    h.set_participant_keys(np.stack([keys[p % h.n] for p in range(h.n * h.G)]))

    def step():
        h.clear()
        ins = h.insert_verified_device(dtr, dd.addr, dr.addr)
        h.DivideRounds()
        h.DecideFame()
        h.FindOrder()
        return ins

    step()
    t0 = time.perf_counter()
    for _ in range(steps):
        ins = step()
    el = (time.perf_counter() - t0) / steps
    rr, cts = h.received()
    ok = ins == tr.E and np.array_equal(rr, ref[0]) and np.array_equal(cts, ref[1])
    ordered = int(h.L.hgx_consensus_events_count(h.ctx, 0))
    dtr.close(), dd.close(), dr.close()
    if not ok:
        raise SystemExit(f"INSERT-VERIFY CHECK FAILURE: accepted {ins} of {tr.E}, rr/cts equal to the headline: "
                         f"{np.array_equal(rr, ref[0])}/{np.array_equal(cts, ref[1])}")
    res = {"value": ordered / el, "unit": "consensus-ordered events/s", "ms_per_step": el * 1e3,
           "signatures_verified_per_step": int(tr.E), "keys": int(min(nk, h.n)),
           "step": "clear + InsertEvent with Event.Verify (batched P-256 verify + parent/index checks, device) + "
                   "DivideRounds + DecideFame + FindOrder, columns HBM-resident",
           "check": "every event accepted; rounds received and consensus timestamps equal the headline run's",
           "signatures": "libcrypto 3.0.2 signatures (tests/golden/p256_pool256.npz: one key per participant, 16 "
                         "signatures per key, cycled by Index)"}
    if sha_ms:
        res["with_event_ids_ms"] = el * 1e3 + sha_ms
        res["with_event_ids_value"] = ordered / (el + sha_ms * 1e-3)
        res["with_event_ids_note"] = "plus one k_sha256_batch launch over the trace's event bodies (ingest_sha256)"
    return res


def device_of(local_rank):
    """The rank's GPU; ranks beyond the visible devices share them (gloo rehearsals on one GPU)."""
    try:
        import torch
        nd = torch.cuda.device_count()
    except Exception:
        nd = 0
    return local_rank % nd if nd > 0 else local_rank


def exchange_floor(dev, chains, n, rounds):
    """roofline.latency's measured floor (hgx_exchange_floor_bench): per round of the persistent
    recurrence, every chain's workgroup publishes its n-byte candidate row + granule and polls every
    other chain's -- k_round_p's all-to-all hand-off with the search taken out; chains = 2 is one
    1-to-1 hand-off each way. Returns (us per round at `chains`, us per 1-to-1 round) or None."""
    import ctypes as C
    from babble_amd import _lib
    L = _lib.lib()
    out = []
    for c in (chains, 2):
        us = C.c_double(0.0)
        if L.hgx_exchange_floor_bench(int(dev), int(c), int(n), int(max(1, rounds)), C.byref(us)) != 0:
            return None
        out.append(us.value)
    return out


def latency_roofline(dev, n, chains, rounds, ms_per_pass):
    """The recurrence is a latency chain (neither HBM nor VALU bound): its floor is rounds x the
    exchange of one round. frac = floor / the kernel's measured time per pass."""
    if not (16 < n <= 256) or chains < 2 or rounds < 1 or ms_per_pass <= 0:
        return None
    fl = exchange_floor(dev, chains, n, min(rounds, 4096))
    if fl is None:
        return {"error": "hgx_exchange_floor_bench failed"}
    floor_ms = rounds * fl[0] * 1e-3
    return {"rounds": int(rounds), "exchange_us_per_round": fl[0], "handoff_1to1_us_per_round": fl[1],
            "floor_ms": floor_ms, "frac": floor_ms / ms_per_pass, "us_per_round_measured": ms_per_pass * 1e3 / rounds,
            "note": f"floor = rounds x the measured all-to-all exchange of one round ({chains} resident workgroups "
                    f"publishing an {n}-byte row + granule write-through and polling all the others', no search; "
                    "hgx_exchange_floor_bench, this run, same GPU); frac = floor / the kernel's ms per pass"}


def run_sharded(args):
    """C3's north-star single-graph mode (BASELINE configs[2]): ONE graph whose round recurrence is
    chain-sharded over `--gpus` devices in one process (hgx_create_sharded): shard k
    builds its chains' firstDescendants, runs their workgroups of the persistent recurrence (its
    candidate rows and granules written into every shard's window over the peer mapping) and their
    consensus timestamps; inserts, lastAncestors, fame, round received and the sort are replicated.
    With fewer devices than shards, shards share a device (the same code: its windows are then local).
    The columns are handed over as the headline's (hgx_events32, host RAM at the start of each step).
    Strong scaling: value = the graph's ordered events per step / the step's wall time."""
    from babble_amd import trace
    from babble_amd.hashgraph import Hashgraph, compact_columns
    import torch
    n, E, G, silent, stale, depth, desc = CONFIGS[args.config]
    if G != 1 or n > 256:
        raise SystemExit("--sharded: one graph of at most 256 peers per run (c1, c2, c3)")
    ndev = max(1, torch.cuda.device_count())
    devs = [k % ndev for k in range(args.gpus)]
    if args.remote_windows and len(set(devs)) == len(devs):
        args.remote_windows = False   # (every window is remote already)
    tr = trace.gossip(n, E, 1, n_silent=silent, stale_prob=stale, stale_depth=depth)
    h = Hashgraph(n, capacity=tr.E, shard_devices=devs)
    if args.remote_windows:
        h.set_shard_remote(True)
    cols = compact_columns(tr)

    def step():
        h.clear()
        h.insert_and_run32(cols)
        return int(h.L.hgx_consensus_events_count(h.ctx, 0))

    h.set_kernel_timing(False)
    for w in range(max(1, args.warmup)):
        tw = time.time()
        ordered = step()
        log(f"[sharded x{len(devs)}] warmup {w}: {ordered} ordered in {time.time() - tw:.2f}s  {h.phase_times()}")
    # shard 0's kernels on one untimed pass (HIP events on its stream)
    h.set_kernel_timing(True)
    h.reset_stats()
    step()
    ks_w = h.kernel_stats()
    h.set_kernel_timing(False)
    t0 = time.perf_counter()
    ordered = 0
    for _ in range(args.steps):
        ordered = step()
    t_el = time.perf_counter() - t0
    ph = h.phase_times()
    if ph["round_p_fallbacks"]:
        raise SystemExit(f"--sharded: the sharded recurrence fell back to per-launch steps: {ph}")
    checks = {"full_size": "skipped"}
    if not args.no_check:
        checks["full_size"] = full_size_checks(h, tr, 1)
    rounds = int(h.LastRound()) + 1
    rs = ks_w.get("round_search", {"ms": 0.0, "launches": 0})
    line = {
        "metric": "consensus-ordered events/sec at N=256 peers (1 GPU and 8-GPU batched sims)",
        "value": ordered * args.steps / t_el, "unit": "consensus-ordered events/s", "n_gpus": len(set(devs)),
        "shards": len(devs), "steps": args.steps, "warmup": args.warmup, "ms_per_step": t_el * 1e3 / args.steps,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "int32",
        "data": "synthetic (seeded random-gossip trace), in host RAM at the start of every step",
        "config": {"workload": desc, "config": args.config, "peers": n, "events": int(tr.E),
                   "shard_devices": devs, "windows": "remote (system-scope stores, test switch)" if args.remote_windows
                   else ("peer-mapped across devices" if len(set(devs)) > 1 else "local (shards share the device)"),
                   "host_columns": "hgx_events32 (61 B/event)",
                   "parallelism": f"one graph, round recurrence chain-sharded x{len(devs)} over devices {devs} "
                                  f"(firstDescendants, recurrence workgroups and consensus timestamps per chain "
                                  f"block; the rest replicated), one process",
                   "phase_ms_last_step": {k: round(float(v), 3) for k, v in ph.items()}},
        "rounds": rounds,
        "kernels_shard0_ms": {k: round(v["ms"], 4) for k, v in ks_w.items()},
        "checks": checks}
    if rs["ms"] > 0:
        b = kernel_bytes("round_search", n, tr.E, 0, ph["compact"])
        ach = b / (rs["ms"] * 1e-3) / 1e9
        line["roofline"] = {"kernel": "round_search", "bound": BOUND["round_search"], "achieved": ach,
                            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "traffic": None,
                            "ms_per_pass": rs["ms"], "algorithmic_bytes_per_pass": b,
                            "note": "shard 0's k_round_p launch (its chain block; every shard's launch spans the "
                                    "whole recurrence, the rounds are shared)"}
    if not args.no_cpu_baseline:
        sample = min(E, SAMPLE.get(n, 20000))
        ts = trace.gossip(n, sample, 1, n_silent=silent, stale_prob=stale, stale_depth=depth)
        line["cpu_baseline"], _ = cpu_baseline(ts, n, desc)
    print(json.dumps(line), flush=True)


def sharded_leg(args, world):
    """rank 0 of an N-rank run: C3's single-graph mode over all N devices, in a child process
    (bench.py --sharded --gpus N) so that a failure there cannot take the replica line with it.
    Returns the child's line, or an error record."""
    import subprocess
    n, E, G, *_ = CONFIGS[args.config]
    if G != 1 or n > 256 or world > n:
        return {"skipped": f"{args.config}: the chain-sharded mode takes one graph of at most 256 peers and at "
                           f"most one shard per chain"}
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "ROLE_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID",
                        "TORCHELASTIC_RESTART_COUNT", "TORCHELASTIC_MAX_RESTARTS", "GROUP_WORLD_SIZE")}
    try:
        import torch
        ndev = max(1, torch.cuda.device_count())
    except Exception:
        ndev = 1
    per_dev = -(-world // ndev)
    if per_dev > 1:   # shards sharing a device need a hardware queue each (hgx_create_sharded)
        env["GPU_MAX_HW_QUEUES"] = str(max(int(env.get("GPU_MAX_HW_QUEUES", "4")), per_dev + 4))
    cmd = [sys.executable, os.path.abspath(__file__), "--sharded", "--gpus", str(world), "--config", args.config,
           "--steps", str(args.steps), "--warmup", str(args.warmup), "--no-cpu-baseline"]
    if args.no_check:
        cmd.append("--no-check")
    t0 = time.time()
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900)
    except subprocess.TimeoutExpired:
        return {"error": "the sharded leg did not finish within 900 s"}
    sys.stderr.write(r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"exit status {r.returncode}", "stderr_tail": r.stderr[-1500:]}
    d = json.loads(lines[-1])
    d["leg_seconds"] = round(time.time() - t0, 1)
    return d


def run_sharded_ranks(args, red, world, rank, local_rank):
    """The multi-process form of C3's mode (torch.distributed ranks, RCCL): every rank holds the
    whole DAG and runs every phase but the consensus-timestamp medians, computed per creator block
    and all-gathered between the halves of FindOrder (hgx_set_shard). Strong scaling."""
    from babble_amd import trace
    from babble_amd.hashgraph import DeviceTrace, Hashgraph
    n, E, G, silent, stale, depth, desc = CONFIGS[args.config]
    tr = trace.gossip(n, E, 1, n_silent=silent, stale_prob=stale, stale_depth=depth)
    dev = device_of(local_rank)
    h = Hashgraph(n, capacity=tr.E, device=dev)
    h.set_shard(rank, world)
    dtr = DeviceTrace(tr, device=dev)

    def step():
        h.clear()
        h.insert_device(dtr)
        h.DivideRounds()
        h.DecideFame()
        red.shard_exchange(h, world, rank)
        return int(h.L.hgx_consensus_events_count(h.ctx, 0))

    for _ in range(max(1, args.warmup)):
        step()
    red.barrier()
    t0 = time.perf_counter()
    ordered = 0
    for _ in range(args.steps):
        ordered = step()
    t_el = time.perf_counter() - t0
    red.barrier()
    t_max = red.max(t_el)
    if rank == 0:
        print(json.dumps({
            "metric": "consensus-ordered events/sec at N=256 peers (1 GPU and 8-GPU batched sims)",
            "value": ordered * args.steps / t_max, "unit": "consensus-ordered events/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": t_max * 1e3 / args.steps,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "int32",
            "data": "synthetic (seeded random-gossip trace, the same on every rank), resident in HBM",
            "config": {"workload": desc, "config": args.config, "peers": n, "events": int(tr.E),
                       "parallelism": f"row-sharded x{world}: consensus timestamps per creator block, "
                                      f"all-gather over {'RCCL' if red.device != 'cpu' else 'gloo'}",
                       "phase_ms_last_step": {k: round(float(v), 3) for k, v in h.phase_times().items()}}}),
              flush=True)


def self_launch(args) -> int:
    """`--gpus N` (N > 1) without torch.distributed.run: run it as a child process -- one rank per GPU,
    127.0.0.1 rendezvous, this script with the same arguments -- and return its exit status. Nothing in
    this process has initialised a GPU at this point."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    log(f"[launch] --gpus {args.gpus} without a launcher: {' '.join(cmd)}")
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true", help="skip the oracle leg (and the prefix parity check)")
    ap.add_argument("--no-ingest", action="store_true", help="skip the batched event-id SHA-256 side leg")
    ap.add_argument("--no-check", action="store_true", help="skip the full-size property checks")
    ap.add_argument("--no-chunked", action="store_true", help="skip the SyncLimit-chunked schedule leg")
    ap.add_argument("--sync-limit", type=int, default=1000)
    ap.add_argument("--columns", default="compact", choices=["packed", "compact", "wide"],
                    help="how the caller hands the events over: hgx_events32 (61 B per event, the default: what a "
                         "caller fills from its events), hgx_events_packed (10 B structure + 45 B payload, built from "
                         "hgx_events32 by a host pass the `packed_columns` leg times) or hgx_events (108 B)")
    ap.add_argument("--wide", action="store_true", help="= --columns wide")
    ap.add_argument("--host-memory", default="pageable", choices=["pageable", "pinned"],
                    help="where the caller keeps the host columns: ordinary (pageable) memory, or page-locked "
                         "buffers from hgx_host_alloc (Core's sync buffers allocated once through the C ABI)")
    ap.add_argument("--sharded", action="store_true",
                    help="C3's single-graph mode in one process: the round recurrence chain-sharded over --gpus devices "
                         "(shards share a device when there are fewer; strong scaling) instead of replicas")
    ap.add_argument("--sharded-ranks", action="store_true",
                    help="C3's mode over torch.distributed ranks: consensus timestamps per creator block, all-gathered")
    ap.add_argument("--backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="rank reductions: auto = RCCL when every rank has its own GPU, else gloo")
    ap.add_argument("--remote-windows", action="store_true",
                    help="--sharded: the shards' window stores take the cross-device path even on a shared device")
    ap.add_argument("--no-sharded-leg", action="store_true", help="N > 1: skip the single-graph sharded leg")
    ap.add_argument("--launch-check", action="store_true",
                    help="ranks meet, reduce and report only (no GPU work): the self-launch's CPU test")
    ap.add_argument("--round-kernel", default="auto",
                    help="DivideRounds' round kernel (Hashgraph.set_round_kernel; measurement A/B, e.g. auto-steps)")
    ap.add_argument("--fame-tally", default="popc", choices=["popc", "vote", "mfma"],
                    help="DecideFame's vote tally (Hashgraph.set_fame_tally; measurement A/B)")
    ap.add_argument("--round-shards", type=int, default=1,
                    help="the chain-sharded recurrence with W shards on this rank's GPU (measurement)")
    args = ap.parse_args()
    if args.sharded or args.round_shards > 1:
        # shards that share a device need a hardware queue each (their launches wait for each
        # other): set before the HIP runtime starts
        need = max(args.gpus, args.round_shards) + 4
        os.environ["GPU_MAX_HW_QUEUES"] = str(max(int(os.environ.get("GPU_MAX_HW_QUEUES", "4")), need))

    launched = "WORLD_SIZE" in os.environ
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.sharded:
        if world > 1:
            raise SystemExit("--sharded runs one process over --gpus devices (not under torch.distributed.run)")
        return run_sharded(args)
    if not launched and args.gpus > 1:
        # no launcher: start one (a child process; nothing here has touched a GPU) and take its status
        return self_launch(args)
    if launched and world > 1 and args.gpus not in (1, world):
        raise SystemExit(f"--gpus {args.gpus} but the launcher started {world} ranks")
    red = Reducer(world, local_rank, backend=args.backend)
    if args.launch_check:
        red.barrier()
        ranks = int(red.sum(1.0))
        t_max = red.max(float(rank))
        if rank == 0:
            print(json.dumps({"launch_check": True, "n_gpus": world, "ranks_reporting": ranks, "max_rank": t_max,
                              "backend": getattr(red, "backend", None)}), flush=True)
        if red.dist is not None:
            red.dist.destroy_process_group()
        return 0
    if args.sharded_ranks:
        if world < 2:
            raise SystemExit("--sharded-ranks needs torch.distributed.run with >= 2 ranks")
        return run_sharded_ranks(args, red, world, rank, local_rank)

    from babble_amd.hashgraph import DeviceTrace, Hashgraph, compact_columns, pack_columns, pinned_columns
    n, E, G, *_ = CONFIGS[args.config]
    if args.wide:
        args.columns = "wide"
    t0 = time.time()
    tr, G = make_trace(args.config, rank)
    log(f"[rank {rank}] trace {tr.E} events generated in {time.time() - t0:.1f}s")
    dev = device_of(local_rank)   # one GPU per rank (ranks share a GPU only in gloo rehearsals)
    h = Hashgraph(n, capacity=tr.E, device=dev, n_graphs=G)
    if args.round_kernel != "auto":
        h.set_round_kernel(args.round_kernel)
    if args.fame_tally != "popc":
        h.set_fame_tally(args.fame_tally)
    if args.round_shards > 1:   # the one-GPU rehearsal of a chain-sharded recurrence
        h.set_round_shards(args.round_shards)
    # the columns as the caller hands them over, built before the clock: hgx_events_packed (u16
    # creator, int32 Index, u16 parent distances + exceptions; the 45-byte compact payload), or
    # hgx_events32 (int32 Index and parents, the coin byte, ntx -1 = nil; 61 B per event), or
    # hgx_events (108 B)
    cols = None if args.columns == "wide" else compact_columns(tr)
    if cols is not None and args.host_memory == "pinned":
        cols = pinned_columns(cols)
    pk = pack_columns(cols, 0) if args.columns == "packed" else None
    if pk is not None:
        log(f"[rank {rank}] packed columns: {len(pk['exc_pos'])} exceptions")

    def step():
        """from the first event append (the trace in host RAM, as the caller holds
        it: the H2D copy of every event column is inside the step) to the order in host memory.
        One hgx_insert_and_run = hgx_insert_events + DivideRounds + DecideFame + FindOrder."""
        h.clear()
        if pk is not None:
            h.insert_and_run_packed(pk)
        elif cols is None:
            h.insert_and_run(tr)
        else:
            h.insert_and_run32(cols)
        return sum(int(h.L.hgx_consensus_events_count(h.ctx, g)) for g in range(G))

    h.set_kernel_timing(False)
    for w in range(max(1, args.warmup)):
        tw = time.time()
        ordered = step()
        log(f"[rank {rank}] warmup {w}: {ordered} ordered in {time.time() - tw:.2f}s  {h.phase_times()}")
    # the kernels ranked on one post-warmup pass with every launch timed (HIP events on the
    # context stream; no first-touch costs): the per-kernel table and the dominant kernel
    h.set_kernel_timing(True)
    h.reset_stats()
    step()
    ks_w, nw = h.kernel_stats(), 1
    dom = max(ks_w, key=lambda k: ks_w[k]["ms"])
    log(f"[rank {rank}] kernel profile (ms per pass / launches): " +
        ", ".join(f"{k}={v['ms'] / nw:.2f}/{v['launches'] // nw}" for k, v in
                  sorted(ks_w.items(), key=lambda kv: -kv[1]['ms'])))

    # timed region: the dominant kernel alone is instrumented
    h.set_kernel_timing(dom)
    h.reset_stats()
    red.barrier()
    t_start = time.perf_counter()   # every hgx call returns with its work complete (order in host memory)
    total = 0
    for _ in range(args.steps):
        total += step()
    t_el = time.perf_counter() - t_start
    red.barrier()
    t_max = red.max(t_el)
    total_all = red.sum(total)
    ks = h.kernel_stats()
    phases = h.phase_times()
    h.set_kernel_timing(False)

    # side leg: the same step with the event columns already resident in HBM (no H2D)
    dtr = DeviceTrace(tr, device=dev)

    def step_hbm():
        h.clear()
        h.insert_device(dtr)
        h.DivideRounds()
        h.DecideFame()
        h.FindOrder()

    step_hbm()
    th = time.perf_counter()
    for _ in range(args.steps):
        step_hbm()
    t_hbm = (time.perf_counter() - th) / args.steps

    checks = {"full_size": "skipped"}
    if not args.no_check:
        tc = time.time()
        checks["full_size"] = full_size_checks(h, tr, G)
        log(f"[rank {rank}] full-size checks passed in {time.time() - tc:.1f}s")
    rounds_pass = int(h.LastRound()) + 1 if G == 1 else None

    # side leg: the packed columns (hgx_events_packed) built from the headline's columns by
    # the host pass a caller holding hgx_events32 would run (hgx_pack_events32), timed inside the step
    packed = None
    if cols is not None and args.columns == "compact":
        h.clear()
        h.insert_and_run_packed(pack_columns(cols, 0))
        t_pack, tq0 = 0.0, time.perf_counter()
        for _ in range(args.steps):
            tq = time.perf_counter()
            pk2 = pack_columns(cols, 0)
            t_pack += time.perf_counter() - tq
            h.clear()
            h.insert_and_run_packed(pk2)
        t_all = (time.perf_counter() - tq0) / args.steps
        t_pack /= args.steps
        m1 = total // max(1, args.steps)
        packed = {"value_incl_pack": m1 / t_all, "ms_per_step_incl_pack": t_all * 1e3, "pack_ms": t_pack * 1e3,
                  "value_excl_pack": m1 / (t_all - t_pack), "ms_per_step_excl_pack": (t_all - t_pack) * 1e3,
                  "exceptions": int(len(pk2["exc_pos"])), "unit": "consensus-ordered events/s",
                  "note": "hgx_insert_and_run_packed (10 B structure + 45 B payload per event cross PCIe) after "
                          "hgx_pack_events32 on the host (one thread) inside the step; not the headline"}

    result = None
    if rank == 0:
        m_pass = total // max(1, args.steps)
        per_pass = {}
        tj_all = {}
        tf = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
        if os.path.exists(tf):
            try:
                tj_all = json.load(open(tf))
            except Exception:
                tj_all = {}
        # the radix sort's passes in the per-kernel pass (libhgx counts 24 bytes per event and pass)
        srt = ks_w.get("order_sort", {})
        sort_passes = max(1, round(srt.get("bytes", 0) / (24.0 * m_pass))) if m_pass else 1
        for k, v in ks_w.items():
            ms = v["ms"] / nw
            b = kernel_bytes(k, n, tr.E, m_pass, phases["compact"], sort_passes)
            pmc = tj_all.get(k, {}).get("bytes_per_pass") if isinstance(tj_all.get(k), dict) else None
            per_pass[k] = {"ms": round(ms, 4), "launches": v["launches"] // nw,
                           "algorithmic_bytes": b, "GB_per_s": (b / (ms * 1e-3) / 1e9) if (b and ms > 0) else None,
                           # the PMC-measured bytes of the same kernel (profiles/traffic_<cfg>.json) over this
                           # line's time: for gathers (cts_median) the model counts L2 hits as bytes, this does not
                           "pmc_GB_per_s": (pmc / (ms * 1e-3) / 1e9) if (pmc and ms > 0) else None}
        r = ks.get(dom, {"ms": 0, "launches": 0})
        dom_ms = r["ms"] / max(1, args.steps)
        dom_bytes = kernel_bytes(dom, n, tr.E, m_pass, phases["compact"], sort_passes)
        achieved = dom_bytes / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 and dom_bytes else 0.0
        traffic, valu = None, None
        tf = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
        if os.path.exists(tf):
            try:
                tj = json.load(open(tf)).get(dom)
                traffic = tj.get("bytes_per_pass") if isinstance(tj, dict) else None
            except Exception:
                traffic = None
        vf = os.path.join(ROOT, "profiles", f"valu_{args.config}.json")
        if os.path.exists(vf):
            try:
                vj = json.load(open(vf)).get(dom)
                if isinstance(vj, dict) and vj.get("valu_insts_per_pass"):
                    lane_ops = 64.0 * vj["valu_insts_per_pass"]
                    v_ach = lane_ops / (dom_ms * 1e-3) / 1e12 if dom_ms > 0 else 0.0
                    valu = {"achieved": v_ach, "peak": VALU_PEAK_TOPS, "unit": "Tlane-op/s",
                            "frac": v_ach / VALU_PEAK_TOPS, "valu_insts_per_pass": vj["valu_insts_per_pass"],
                            "frac_profiled": vj.get("frac_profiled"),
                            "source": f"profiles/valu_{args.config}.json (rocprofv3 --pmc SQ_INSTS_VALU, "
                                      "64 lanes per wave instruction, over this line's ms_per_pass)"}
            except Exception:
                valu = None
        result = {
            "metric": "consensus-ordered events/sec at N=256 peers (1 GPU and 8-GPU batched sims)",
            "value": total_all / t_max,
            "unit": "consensus-ordered events/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": t_max * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (seeded random-gossip traces, synthetic event ids/signatures), in host RAM at "
                    "the start of every step (hgx_insert_events copies the columns to HBM inside the step)",
            "config": {"workload": CONFIGS[args.config][6], "config": args.config, "peers": n,
                       "events_per_gpu": int(tr.E), "graphs_per_gpu": G,
                       "ordered_events_per_step_per_gpu": int(m_pass),
                       "step": ("clear + hgx_insert_and_run" +
                                {"wide": "", "compact": "32", "packed": "_packed"}[args.columns] +
                                ": InsertEvent (H2D of the event columns + device validation) + DivideRounds + "
                                "DecideFame + FindOrder, the payload columns' H2D beside DivideRounds; order in "
                                "host memory"),
                       "host_columns": {
                           "wide": "hgx_events (108 B/event)",
                           "compact": "hgx_events32 (int32 Index/parents, coin byte, ntx -1 = nil: 61 B/event)",
                           "packed": "hgx_events_packed (u16 creator, int32 Index, u16 parent distances: 10 B "
                                     "structure + 45 B payload per event; %d exceptions)" % (
                                         len(pk["exc_pos"]) if pk is not None else 0)}[args.columns],
                       "host_memory": args.host_memory if cols is not None else "pageable",
                       "parallelism": f"replicas x{world} (seed-sharded)" +
                                      (f"; recurrence rehearsed in {args.round_shards} chain blocks on one GPU"
                                       if args.round_shards > 1 else ""),
                       "phase_ms_last_step": {k: round(float(v), 3) for k, v in phases.items()},
                       "dominant_kernel": dom},
            "roofline": {"kernel": dom, "bound": BOUND.get(dom, "hbm"), "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "ms_per_pass": dom_ms, "launches_per_pass": r["launches"] // max(1, args.steps),
                         "algorithmic_bytes_per_pass": dom_bytes, "valu": valu,
                         "note": "per pass: SURVEY 8(d) bytes of the kernel's role over all its launches / "
                                 "its summed device time (HIP events on the context stream, timed steps); "
                                 "traffic = PMC bytes per pass (profiles/traffic_<cfg>.json: FETCH_SIZE x2 only "
                                 "for wide streaming kernels, Infinity-Cache hits included); valu = VALU issue "
                                 "rate from SQ_INSTS_VALU (profiles/valu_<cfg>.json)"},
            "kernels_per_pass": per_pass,
            "sort_radix_passes": sort_passes,
            "packed_columns": packed,
            "hbm_resident": {"value": total // max(1, args.steps) / t_hbm, "unit": "consensus-ordered events/s",
                             "ms_per_step": t_hbm * 1e3,
                             "note": "the same step with the event columns already in HBM (hgx_insert_events_device, "
                                     "no H2D inside the step); not the headline"},
            "checks": checks,
        }
        if dom == "round_search" and rounds_pass and phases.get("round_p_runs", 0) > 0:
            try:
                result["roofline"]["latency"] = latency_roofline(dev, n, n, rounds_pass, dom_ms)
            except Exception as e:  # reported, never fatal
                result["roofline"]["latency"] = {"error": str(e)}
        if not args.no_ingest:
            try:
                result["ingest_sha256"] = ingest_leg(int(tr.E), args.steps, args.warmup, dev)
            except Exception as e:  # reported, never fatal
                result["ingest_sha256"] = {"error": str(e)}
            try:
                result["ingest_p256_verify"] = p256_leg(1 << 20, args.steps, args.warmup, dev)
            except Exception as e:  # reported, never fatal
                result["ingest_p256_verify"] = {"error": str(e)}
        if G == 1 and not args.no_ingest:
            try:
                sha = result.get("ingest_sha256", {}).get("ms_per_launch")
                tv = time.time()
                result["insert_verify"] = insert_verify_leg(h, tr, args.steps, h.received(), sha, dev)
                # next to `value`: the same step with Event.Verify inside InsertEvent (hashgraph.go:358-363),
                # columns HBM-resident (the headline and its CPU baseline both leave Verify out)
                result["value_with_verify"] = result["insert_verify"].get("value")
                log(f"[rank {rank}] insert+verify leg in {time.time() - tv:.1f}s")
            except SystemExit:
                raise
            except Exception as e:  # reported, never fatal
                result["insert_verify"] = {"error": str(e)}
        if G == 1 and not args.no_chunked:
            tcl = time.time()
            result["chunked_sync"] = chunked_leg(h, tr, args.sync_limit, not args.no_check)
            log(f"[rank {rank}] chunked schedule: {result['chunked_sync']['calls']} calls in "
                f"{time.time() - tcl:.1f}s")
        if world == 1 and not args.no_cpu_baseline:
            from babble_amd import trace
            _, _, _, silent, stale, depth, desc = CONFIGS[args.config]
            sample = min(E, SAMPLE.get(n, 20000))
            ts = trace.gossip(n, sample, 1, n_silent=silent, stale_prob=stale, stale_depth=depth)
            base, o = cpu_baseline(ts, n, desc, ordered_frac=m_pass / max(1, int(tr.E)))
            result["cpu_baseline"] = base
            checks["prefix_parity"] = prefix_parity(ts, o, dev)
            log(f"[rank {rank}] prefix parity ({sample} events) bit-exact")
    if world > 1 and not args.no_sharded_leg:
        # C3's single-graph mode over all N devices: every rank releases its GPU memory first, and the
        # other ranks wait on the host (no collective kernel may occupy a GPU the leg's persistent
        # recurrence needs whole)
        h.close()
        dtr.close()
        try:
            import torch
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
        except Exception:
            pass
        red.cpu_barrier()
        if rank == 0:
            tsl = time.time()
            result["sharded"] = sharded_leg(args, world)
            log(f"[rank 0] sharded leg in {time.time() - tsl:.1f}s")
        red.cpu_barrier()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if red.dist is not None:
        red.dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
