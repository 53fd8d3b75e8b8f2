#!/usr/bin/env python3
"""GPU: ms per call of C3, C2 (one frame per call) and the C4 per-GPU share
(8 x 4K in one call, default lanes) for the engine options in the
environment, outputs checked against the reference fixtures.  One JSON line.
    DQ_HIP_...=... python3 tools/ab_timing.py TAG [calls]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import bench
    from __graft_entry__ import load_package
    tag = sys.argv[1]
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    pkg = load_package()
    dev = torch.device("cuda", 0)
    out = {"tag": tag, "env": {k: v for k, v in os.environ.items() if k.startswith("DQ_HIP_")}}

    def timed(fn, n):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        ts.sort()
        return {"min": round(ts[0], 3), "median": round(ts[len(ts) // 2], 3)}

    for cfg in ("c3", "c2"):
        w, h, k = bench.CONFIGS[cfg]
        t_in = torch.from_numpy(pkg.synth_frame(w * h, 0).view(np.int32)).to(dev)
        t_out = torch.empty_like(t_in)
        last = {}

        def one():
            last["ct"], _ = pkg.quant_device(t_in, t_out, k, max_iters=10)
        out[cfg] = timed(one, calls)
        out[cfg]["ok"] = bench.check_frame(pkg, t_out, last["ct"], bench.frame_fixture(w, h, k, 0))
        out[cfg]["rounds"] = pkg.last_rounds()
    w, h, k = bench.CONFIGS["c3"]
    frames = [torch.from_numpy(pkg.synth_frame(w * h, f).view(np.int32)).to(dev) for f in range(8)]
    outs = [torch.empty_like(f) for f in frames]
    last = {}

    def batch():
        last["cts"], _ = pkg.quant_batch_device(frames, outs, k, max_iters=10)
    out["c4share"] = timed(batch, calls)
    out["c4share"]["ok"] = all(bench.check_frame(pkg, outs[i], last["cts"][i], bench.frame_fixture(w, h, k, i))
                               for i in range(8))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
