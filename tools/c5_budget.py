#!/usr/bin/env python3
"""GPU: inputs of the C5-at-N-ranks latency budget.

    python3 tools/c5_budget.py [nranks]      (prints JSON lines)

1. C5 (16384^2, K=1024) through the loopback row sharding at N ranks on this
   GPU: the collectives every rank enqueued per call (count, element sizes),
   the call's wall time (N ranks share one GPU here: an upper bound of one
   rank's chain, not the 8-GPU time);
2. C5 on one GPU unsharded (the N=1 reference of the same call);
3. RCCL allreduce latency of the C5 collective sizes on a 1-rank
   communicator (torch.distributed, backend nccl = RCCL), median of 200.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import torch.distributed as dist
    import dq_fixtures as fx
    from __graft_entry__ import load_package
    pkg = load_package()
    nr = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    n = 16384
    t = torch.from_numpy(fx.xorshift(n * n).view(np.int32)).to("cuda:0")
    o = torch.empty_like(t)
    logs = None
    ts = []
    for i in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _, logs, _ = pkg.loopback_rows_device([t], [o], n, n, 1024, nr)
        ts.append((time.perf_counter() - t0) * 1e3)
    sizes = sorted(set(logs[0]))
    print(json.dumps({"what": "c5_loopback", "ranks": nr, "collectives_per_call": len(logs[0]),
                      "identical_on_all_ranks": all(lg == logs[0] for lg in logs),
                      "u64_per_collective_min_max": [int(min(logs[0])), int(max(logs[0]))],
                      "distinct_sizes": len(sizes), "ms_per_call_shared_gpu": [round(x, 3) for x in ts[1:]]}),
          flush=True)
    ts = []
    for i in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pkg.quant_device(t, o, 1024)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    print(json.dumps({"what": "c5_one_gpu", "ms_per_call": [round(x, 3) for x in ts[1:]]}), flush=True)
    del t, o
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29517")
    dist.init_process_group("nccl", rank=0, world_size=1)
    res = {}
    for cnt in (8 * 2, 8 * 64, 8 * 1024, 8 * 2048):
        x = torch.zeros(cnt, dtype=torch.int64, device="cuda:0")
        for _ in range(20):
            dist.all_reduce(x)
        torch.cuda.synchronize()
        lat = []
        for _ in range(200):
            t0 = time.perf_counter()
            dist.all_reduce(x)
            torch.cuda.synchronize()
            lat.append((time.perf_counter() - t0) * 1e6)
        res[str(cnt)] = round(float(np.median(lat)), 1)
    print(json.dumps({"what": "rccl_allreduce_1rank_us_median", "u64_elements": res}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
