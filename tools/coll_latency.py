#!/usr/bin/env python3
"""GPU (measurement tool): in-stream cost of the row-tile path's collective,
an RCCL allreduce (sum) of u64 node totals, on a 1-rank communicator (the
only one a one-GPU box has).  HIP events on the collective's stream bracket
N back-to-back allreduces (no host sync between them), so the figure is the
per-collective GPU-side time, not a host round trip.
    python3 tools/coll_latency.py [N]     (one JSON line per size)"""
import json
import os
import sys


def main():
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda:0")
    for words in (8, 64, 512, 4096, 16384):
        t = torch.ones(words, dtype=torch.int64, device=dev)
        for _ in range(20):
            dist.all_reduce(t)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(n):
            dist.all_reduce(t)
        b.record()
        b.synchronize()
        us = a.elapsed_time(b) * 1e3 / n
        print(json.dumps({"u64": words, "calls": n, "us_per_allreduce_in_stream": round(us, 2)}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
