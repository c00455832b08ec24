"""Worker of tests/test_gpu_sharded.py: one rank of a row-sharded graph (gloo all-gather of
the consensus timestamps between FindOrder's halves). Writes its results to <out>.npz."""
import os
import sys

import numpy as np


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    n, E, chunk = int(sys.argv[5]), int(sys.argv[6]), int(sys.argv[7])
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from babble_amd import trace as gtrace
    from babble_amd.hashgraph import Hashgraph

    def all_gather(local, counts):
        mx = max(counts)
        buf = torch.zeros(mx, dtype=torch.int64)
        buf[:len(local)] = torch.from_numpy(local)
        parts = [torch.zeros(mx, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(parts, buf)
        return [p[:c].numpy() for p, c in zip(parts, counts)]

    t = gtrace.gossip(n, E, 77, stale_prob=0.1, stale_depth=2)
    h = Hashgraph(n, capacity=E)
    h.set_shard(rank, world)
    for lo in range(0, E, chunk):
        h.insert_trace(t, lo, min(E, lo + chunk))
        h.RunConsensusSharded(all_gather)
    r = h.results()
    np.savez(out, order=np.asarray(r["order"]), rr=np.asarray(r["rr"]), cts=np.asarray(r["cts"]),
             round=np.asarray(r["round"]), lcr=np.array([r["lcr"] if r["lcr"] is not None else -99]))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
