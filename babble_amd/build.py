"""Builds libhgx.so in-tree for gfx950 (hipcc), plus the test oracle (gcc).

Usage: python -m babble_amd.build   (or __graft_entry__.build())
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libhgx.so")
SOURCES = ["hgx_kernels.hip", "hgx_rounds.hip", "hgx_round_k.hip", "hgx_round_p.hip", "hgx_round_pb.hip", "hgx_round_g.hip", "hgx_la_wave.hip", "hgx_insert.hip", "hgx_sha256.hip", "hgx_p256.hip", "hgx_cts.hip", "hgx_engine.cpp", "hgx_api.cpp", "hgx_goenc.cpp", "hgx_trace.cpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-result",
         "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_lib(force: bool = False, verbose: bool = True, variant: str = "") -> str:
    """variant "prof": -DHGX_STEP_PROF build into libhgx_prof.so (phase timing of the round step)."""
    out = OUT if not variant else os.path.join(HERE, f"libhgx_{variant}.so")
    # variant "exp*": experiment build with the macros listed in HGX_EXP_DEFS (comma separated)
    extra = ["-DHGX_STEP_PROF", "-DHGX_LA_ROWSTATS"] if variant == "prof" else \
        [f"-D{d}" for d in os.environ.get("HGX_EXP_DEFS", "").split(",") if d] if variant.startswith("exp") else []
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    deps = srcs + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")] + \
        [os.path.join(ROOT, "include", "hgx.h")]
    if not force and not _newer(out, deps):
        return out
    objdir = os.path.join(HERE, "build" + (f"_{variant}" if variant else ""))
    os.makedirs(objdir, exist_ok=True)
    objs = []
    procs = []
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer(o, [s] + deps[len(srcs):]):
            cmd = [HIPCC] + FLAGS + extra + ["-c", s, "-o", o]
            if s.endswith(".cpp"):
                cmd = [HIPCC] + FLAGS + extra + ["-x", "hip", "-c", s, "-o", o] if "engine" in s else \
                    [HIPCC] + [f for f in FLAGS if not f.startswith("--offload")] + ["-c", s, "-o", o]
            if verbose:
                print(" ".join(cmd), flush=True)
            procs.append(subprocess.Popen(cmd))
    for p in procs:
        if p.wait() != 0:
            raise RuntimeError("hipcc failed")
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    return out


def build_oracle(verbose: bool = True) -> str:
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    return os.path.join(ROOT, "oracle", "liboracle_hg.so")


if __name__ == "__main__":
    if "--variant" in sys.argv:
        build_lib(force="--force" in sys.argv, variant=sys.argv[sys.argv.index("--variant") + 1])
    else:
        build_lib(force="--force" in sys.argv)
        build_oracle()
