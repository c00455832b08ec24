"""Probe for the P-256 verify PMC pass: the bench's ingest_p256_verify leg once (1 M signatures,
one warmup + one timed launch). Usage: python tools/probe/p256_pmc.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

r = bench.p256_leg(1 << 20, 1, 1, 0)
print(r, flush=True)
