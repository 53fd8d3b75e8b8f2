#!/usr/bin/env python3
"""GPU: host-side phase trace (DQ_HIP_TRACE=1 lines on stderr) of N C3 calls
(one 4K frame, K=256) after warm-up, plus the Python-side time per call.
    DQ_HIP_TRACE=1 python3 tools/c3_trace.py [N]"""
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    t = torch.from_numpy(fx.xorshift(3840 * 2160).view(np.int32)).to("cuda:0")
    o = torch.empty_like(t)
    st = torch.cuda.current_stream()
    for _ in range(5):
        pkg.quant_device(t, o, 256, stream=st)
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        pkg.quant_device(t, o, 256, stream=st)
        ts.append((time.perf_counter() - t0) * 1e6)
    torch.cuda.synchronize()
    print("python per call us:", [round(x, 1) for x in ts], flush=True)


if __name__ == "__main__":
    main()
