"""C3 latency anatomy: one 3840x2160 K=256 frame per call.

    DQ_HIP_TRACE=2 python tools/c3_trace.py [calls]

Prints ms per call; with DQ_HIP_TRACE=1/2 the engine prints its host-side
phase breakdown (per round with 2) on stderr.  Under rocprofv3 --kernel-trace
the kernel timeline of the same calls shows the GPU idle gaps between rounds.
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
from __graft_entry__ import load_package  # noqa: E402
import dq_fixtures as fx  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 10
pkg = load_package()
dev = torch.device("cuda:0")
px = fx.xorshift(3840 * 2160)
t = torch.from_numpy(px.view(np.int32)).to(dev)
o = torch.empty_like(t)
s = torch.cuda.current_stream(dev)
for _ in range(3):
    pkg.quant_device(t, o, 256, stream=s)
torch.cuda.synchronize()
ts = []
for _ in range(calls):
    t0 = time.perf_counter()
    pkg.quant_device(t, o, 256, stream=s)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
ts = np.array(ts) * 1e3
print("c3 ms per call: min %.3f median %.3f max %.3f (rounds %d)" %
      (ts.min(), np.median(ts), ts.max(), pkg.last_rounds()), flush=True)
