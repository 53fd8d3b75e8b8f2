#!/usr/bin/env python3
"""GPU: the weighted path (allPixelsUnique=0) on C3's frame: N timed calls
after warm-up, verified against the reference build's fixture (c4.json
frame 0; the uniform-weight and weighted outputs are equal on 4K noise).
    python3 tools/weighted_c3.py [N]        (one JSON line)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from __graft_entry__ import load_package
    pkg = load_package()
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    w, h, k = bench.CONFIGS["c3"]
    t = bench.upload_frames(torch, pkg, torch.device("cuda", 0), w, h, [0])[0]
    o = torch.empty_like(t)
    st = torch.cuda.current_stream()
    for _ in range(2):
        ct, _ = pkg.quant_device(t, o, k, stream=st, all_pixels_unique=0)
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        ct, _ = pkg.quant_device(t, o, k, stream=st, all_pixels_unique=0)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    ok = bench.check_frame(pkg, o, ct, bench.frame_fixture(w, h, k, 0))
    print(json.dumps({"weighted_c3_ms": sorted(ts)[len(ts) // 2], "all_ms": [round(x, 3) for x in ts],
                      "verified": ok, "seq_tiles_last_call": pkg.last_seq_tiles()}))


if __name__ == "__main__":
    main()
