"""Probe: can torch (its bundled HIP runtime) and libhgx (system ROCm) share a process, in
either initialisation order?"""
import ctypes, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
order = sys.argv[1]
def hgx():
    from babble_amd.hashgraph import Hashgraph
    h = Hashgraph(4, capacity=16)
    print("libhgx ctx ok", flush=True)
    return h
def tch():
    import torch
    print("torch", torch.__version__, torch.version.hip, "available", torch.cuda.is_available(), flush=True)
    x = torch.ones(4, device="cuda")
    print("torch tensor ok", float(x.sum()), flush=True)
if order == "torch_first":
    tch(); h = hgx()
else:
    h = hgx(); tch()
maps = open(f"/proc/{os.getpid()}/maps").read()
print(sorted({l.split()[-1] for l in maps.splitlines() if "amdhip64" in l}))
