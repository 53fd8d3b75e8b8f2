#!/usr/bin/env python3
"""GPU: the C5 tile (16384^2, K=1024) through quant_rows_device with NSHARD
virtual row shards, CALLS timed calls after one warm-up (for rocprofv3 kernel
statistics of the sharded vs unsharded path).
    python3 tools/c5_shards.py NSHARD [CALLS]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import dq_fixtures as fx
    from __graft_entry__ import load_package
    ns = int(sys.argv[1])
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    pkg = load_package()
    w = 16384
    t = torch.from_numpy(fx.xorshift(w * w).view(np.int32)).to("cuda:0")
    o = torch.empty_like(t)
    big = fx.load_json("big.json")["16384x16384_k1024"]
    for i in range(calls + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ct, _ = pkg.quant_rows_device([t], [o], 1024, widths=[w], nshard=ns)
        torch.cuda.synchronize()
        ok = [int(v) for v in ct[0]] == big["ct"]
        print("nshard %d call %.3f ms rounds %d planned %d ct_ok %s" % (ns, (time.perf_counter() - t0) * 1e3,
              pkg.last_rounds(), pkg.last_planned_rounds(), ok), file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
