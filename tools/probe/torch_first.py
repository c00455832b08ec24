"""Probe: libhgx when torch's HIP runtime (same SONAME libamdhip64.so.7) is loaded first.
Runs c3-shaped passes with and without per-kernel timing; prints the mapped HIP runtime,
the persistent-round counters and every error. Usage: python tools/probe/torch_first.py [n] [E] [torch|hgx]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
E = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
first = sys.argv[3] if len(sys.argv) > 3 else "torch"
if first == "torch":
    import torch
    print("torch devices", torch.cuda.device_count(), flush=True)
from babble_amd import _lib, trace  # noqa: E402
from babble_amd.hashgraph import Hashgraph  # noqa: E402
_lib.lib()
if first != "torch":
    import torch
    print("torch devices", torch.cuda.device_count(), flush=True)
maps = open(f"/proc/{os.getpid()}/maps").read()
print("HIP runtimes:", sorted({ln.split()[-1] for ln in maps.splitlines() if "amdhip64" in ln}), flush=True)
t = trace.gossip(n, E, 1)
h = Hashgraph(n, capacity=E)
for p, timing in enumerate([False, True, False]):
    h.set_kernel_timing(timing)
    for name, fn in (("clear", h.clear), ("insert", lambda: h.insert_trace(t)), ("divide", h.DivideRounds),
                     ("fame", h.DecideFame), ("order", h.FindOrder)):
        try:
            fn()
        except Exception as e:
            print(f"pass {p} timing {timing}: {name} ERROR {e!r}", flush=True)
            break
    ph = h.phase_times()
    print(f"pass {p} timing {timing}: ordered {len(h.ConsensusEvents())} runs {ph['round_p_runs']} "
          f"fallbacks {ph['round_p_fallbacks']} fail {ph['round_p_fail_round']}/{ph['round_p_fail_chain']} "
          f"rounds_ms {ph['rounds_ms']:.2f}", flush=True)
