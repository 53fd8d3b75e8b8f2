#!/usr/bin/env python3
"""GPU: per-call latency of single-frame quant_recurse calls (C3 / C2 /
C4-share batch), median and 10th / 90th percentiles over many calls.
    python3 tools/latency.py [calls]      (prints one JSON line)"""
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
    import dq_fixtures as fx
    from __graft_entry__ import load_package
    pkg = load_package()
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    res = {"env": {k: v for k, v in os.environ.items() if k.startswith("DQ_HIP")}}
    for cfg, (w, h, k, nf) in {"c3": (3840, 2160, 256, 1), "c2": (1920, 1080, 256, 1),
                               "c4share": (3840, 2160, 256, 8)}.items():
        ins = [torch.from_numpy(fx.xorshift(w * h, seed=fx.SEED + f).view(np.int32)).to("cuda:0") for f in range(nf)]
        outs = [torch.empty_like(t) for t in ins]
        n = calls if nf == 1 else max(10, calls // 8)
        ts = []
        for i in range(20 + n):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if nf == 1:
                pkg.quant_device(ins[0], outs[0], k)
            else:
                pkg.quant_batch_device(ins, outs, k)
            torch.cuda.synchronize()
            if i >= 20:
                ts.append((time.perf_counter() - t0) * 1e3)
        ts = np.array(ts)
        res[cfg] = {"median_ms": round(float(np.median(ts)), 4), "p10": round(float(np.percentile(ts, 10)), 4),
                    "p90": round(float(np.percentile(ts, 90)), 4), "calls": int(len(ts))}
        del ins, outs
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
