#!/usr/bin/env python3
"""GPU: row-shard timing on one GPU -- C5 (16384^2, K=1024) as one shard and
as 8 virtual row shards, and the C4 share (8 x 4K) as 8-shard row tiles vs the
frame batch.  Each timed call's outputs are checked against the fixtures.

    python3 tools/shard_timing.py [steps]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def timeit(fn, steps):
    import torch
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / steps


def main():
    import torch
    import dq_fixtures as fx
    from __graft_entry__ import load_package
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    pkg = load_package()
    res = {}
    big = fx.load_json("big.json")["16384x16384_k1024"]
    w5 = 16384
    t5 = torch.from_numpy(fx.xorshift(w5 * w5).view(np.int32)).to("cuda:0")
    o5 = torch.empty_like(t5)
    for ns in (1, 8):
        last = {}

        def c5():
            last["ct"], _ = pkg.quant_rows_device([t5], [o5], 1024, widths=[w5], nshard=ns)
        res["c5_nshard%d_ms" % ns] = round(timeit(c5, steps), 3)
        ok = [int(v) for v in last["ct"][0]] == big["ct"] and \
            "%016x" % fx.fnv(o5.cpu().numpy().view(np.uint32)) == big["out_fnv"]
        res["c5_nshard%d_ok" % ns] = ok
        res["c5_nshard%d_planned" % ns] = pkg.last_planned_rounds()
    del t5, o5
    torch.cuda.empty_cache()
    fix = fx.load_json("c4.json")
    frames = [torch.from_numpy(fx.xorshift(3840 * 2160, seed=fx.SEED + f).view(np.int32)).to("cuda:0")
              for f in range(8)]
    outs = [torch.empty_like(t) for t in frames]
    for ns in (1, 8):
        last = {}

        def rows():
            last["cts"], _ = pkg.quant_rows_device(frames, outs, 256, widths=[3840] * 8, nshard=ns)
        res["c4share_rows_nshard%d_ms" % ns] = round(timeit(rows, steps), 3)
        res["c4share_rows_nshard%d_ok" % ns] = all(
            [int(v) for v in last["cts"][f]] == fix["f%02d" % f]["ct"] and
            "%016x" % fx.fnv(outs[f].cpu().numpy().view(np.uint32)) == fix["f%02d" % f]["out_fnv"]
            for f in range(8))
        res["c4share_rows_nshard%d_planned" % ns] = pkg.last_planned_rounds()

    def batch():
        pkg.quant_batch_device(frames, outs, 256)
    pkg.set_lanes(1)
    res["c4share_batch_1lane_ms"] = round(timeit(batch, steps), 3)
    pkg.set_lanes(0)
    res["c4share_batch_ms"] = round(timeit(batch, steps), 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
