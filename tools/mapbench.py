#!/usr/bin/env python3
"""GPU (development tool): map_colors_mps alone on the 8 x 4K step's pixels
(one 66.4 M-pixel job, frame 0's 256-colour reference colortable), timed
with HIP events over N calls of the library's device map entry (cell build +
map).  Use DQ_HIP_LIB to time a kernel variant.
    python3 tools/mapbench.py [N]        (one JSON line)"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import dq_fixtures as fx
    from __graft_entry__ import load_package
    pkg = load_package()
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    W, H = 3840, 2160
    px = np.concatenate([fx.xorshift(W * H, seed=fx.SEED + f) for f in range(8)])
    pal = np.array(fx.load_json("c4.json")["f00"]["ct"], np.uint32)
    t = torch.from_numpy(px.view(np.int32)).to("cuda:0")
    o = torch.empty_like(t)
    for _ in range(3):
        pkg.map_device(t, o, pal)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        pkg.map_device(t, o, pal)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    ok = None
    if not os.environ.get("DQ_HIP_LIB"):
        ref = np.zeros(W * H, np.uint32)
        import ctypes
        fx.oracle().dqo_map(fx.vp(px[:W * H]), ctypes.c_uint32(W * H), fx.vp(ref), fx.vp(pal), ctypes.c_int(len(pal)))
        ok = bool(np.array_equal(o[:W * H].cpu().numpy().view(np.uint32), ref))
    print(json.dumps({"lib": os.path.basename(os.environ.get("DQ_HIP_LIB", "tree")), "ms_per_call": round(ms, 4),
                      "px": int(px.size), "k": int(pal.size), "frame0_vs_oracle": ok}), flush=True)


if __name__ == "__main__":
    main()
