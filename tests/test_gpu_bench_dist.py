"""bench.py's multi-rank replica path on the GPU: two ranks launched by
torch.distributed.run share the one GPU of the test box over gloo (the driver's 8-GPU run uses
RCCL, one GPU per rank). Each rank runs libhgx on its own seed-sharded trace; the line must
report both ranks' work, and every rank's full-size checks must pass."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("cfg", ["c1", "c4"])
def test_bench_replicas_world2(cfg):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--config", cfg, "--backend", "gloo", "--steps", "2", "--warmup", "1",
           "--no-cpu-baseline", "--no-ingest", "--no-chunked"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]   # rank 0 prints the one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["scaling"] == "weak"
    per_gpu = d["config"]["ordered_events_per_step_per_gpu"]
    assert per_gpu > 0
    # value = both ranks' ordered events over the max-over-ranks time of the 2 timed steps
    assert d["value"] * d["ms_per_step"] * 1e-3 >= 1.5 * per_gpu   # rank 1 ordered about as many
    assert d["checks"]["full_size"]["result"] == "pass"


@pytest.mark.parametrize("cfg", ["c1", "c2"])
def test_bench_self_launch_and_sharded_leg(cfg):
    """`bench.py --gpus 2` with no launcher (the driver's form): it launches the two ranks itself, the
    line carries both ranks' work, and rank 0 adds the single-graph leg -- one graph whose recurrence is
    chain-sharded over the N devices (both shards on the box's one GPU here) -- with no fallback and the
    full-size checks passing."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", cfg, "--steps", "2",
           "--warmup", "1", "--no-cpu-baseline", "--no-ingest", "--no-chunked"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    assert d["value"] * d["ms_per_step"] * 1e-3 >= 1.5 * d["config"]["ordered_events_per_step_per_gpu"]
    sh = d["sharded"]
    assert "error" not in sh, sh
    assert sh["shards"] == 2 and sh["scaling"] == "strong" and sh["value"] > 0, sh
    ph = sh["config"]["phase_ms_last_step"]
    assert ph["round_p_runs"] > 0 and ph["round_p_fallbacks"] == 0, ph
    assert sh["checks"]["full_size"]["result"] == "pass"
    assert d["packed_columns"]["pack_ms"] > 0
