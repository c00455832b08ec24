"""Bit-exact parity of the headline workloads IN FULL: bench.py's c3 trace (256 peers, 10 M events,
seed 1) and c5 trace (1 024 peers, 341 silent, 30 % stale other-parents, 1 M events), run through the
C ABI as bench.py hands them over, against SHA-256 digests of every output of the CPU oracle
(oracle/hg_oracle.c, the restatement of hashgraph.go:616-858) over the same whole traces --
tests/golden/make_full_digests.py, run in the build container (the oracle needs ~25 / ~40 min there).

Compared: round, witness, fame, round received and consensus timestamp of every event, the consensus
order, UndecidedRounds, LastConsensusRound, LastCommitedRoundEvents, ConsensusTransactions,
PendingLoadedEvents, every block's (RoundReceived, #transactions, nil, committed) and every block's hash
(SHA256 of the Go JSON of Block, block.go:26-53, over the GPU order's transactions)."""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

import hgref

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(HERE, "golden"))


def gpu_block_digests(h, t):
    """The GPU's blocks in make_full_digests' digest form; each block's hash from the GPU order's
    transactions (payload bytes of the generated trace, include/hgx.h hgx_trace_tx_payload)."""
    from babble_amd.hashgraph import block_hash
    order = np.asarray(h.ConsensusEvents(), np.int64)
    blocks = h.Blocks()
    has = (np.asarray(t.ntx) > 0) & (np.asarray(t.txnil) == 0)
    creator, seq = np.asarray(t.creator), np.asarray(t.tx_seq)
    out = []
    for b in blocks:
        sel = order[b["first"]:b["first"] + b["n_events"]]
        sel = sel[has[sel]]
        txs = [hgref.gossip_payload(int(c), int(q)) for c, q in zip(creator[sel], seq[sel])]
        out.append((b["rr"], b["ntx"], b["tx_nil"], b["committed"], block_hash(b["rr"], txs, b["tx_nil"])))
    return out


def _check(cfg, columns):
    import bench
    import make_full_digests as mk
    from babble_amd.hashgraph import Hashgraph, compact_columns, pack_columns
    path = os.path.join(HERE, "golden", f"{cfg}_full.json")
    if not os.path.exists(path):
        pytest.fail(f"{path} missing: PYTHONPATH=tests:. python tests/golden/make_full_digests.py {cfg}")
    doc = json.load(open(path))
    t, G = bench.make_trace(cfg, 0)
    assert G == 1 and t.E == doc["E"] and t.n == doc["n"]
    h = Hashgraph(t.n, capacity=t.E)
    cols = compact_columns(t)
    if columns == "packed":
        assert h.insert_and_run_packed(pack_columns(cols, 0)) == t.E
    else:
        assert h.insert_and_run32(cols) == t.E
    ph = h.phase_times()
    assert ph["round_p_fallbacks"] == 0, ph
    res = h.results()
    got = mk.summarize(res, with_blocks=False)
    got.update(mk.block_digests(gpu_block_digests(h, t)))
    want = doc["digests"]
    bad = [k for k in want if got.get(k) != want[k]]
    assert not bad, {k: (got.get(k), want[k]) for k in bad}
    assert got["n_blocks"] > 0 and len(res["order"]) > 0
    return res


def test_c3_headline_workload_bit_exact_in_full():
    """The metric's configuration (BASELINE configs[2]), all 10 M events, hgx_events32 as bench.py's
    headline hands them over."""
    res = _check("c3", "compact")
    assert len(res["order"]) > 9_000_000


def test_c5_workload_bit_exact_in_full():
    """BASELINE configs[4] (1 024 peers, a third silent, multi-round fame), all 1 048 576 events, the
    persistent big-n recurrence (k_round_pb), the packed host columns."""
    _check("c5", "packed")
