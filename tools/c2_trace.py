#!/usr/bin/env python3
"""GPU: per-round host trace (DQ_HIP_TRACE=2) of one frame of a config, after
warm-up calls.    python3 tools/c2_trace.py [c2|c3] [calls]"""
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
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    w, h, k = {"c2": (1920, 1080, 256), "c3": (3840, 2160, 256)}[cfg]
    pkg = load_package()
    t_in = torch.from_numpy(fx.xorshift(w * h).view(np.int32)).to("cuda:0")
    t_out = torch.empty_like(t_in)
    for _ in range(calls):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ct, _ = pkg.quant_device(t_in, t_out, k)
        torch.cuda.synchronize()
        print("%s call %.3f ms rounds %d planned %d swept %d" % (cfg, (time.perf_counter() - t0) * 1e3,
              pkg.last_rounds(), pkg.last_planned_rounds(), pkg.last_points_swept()), file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
