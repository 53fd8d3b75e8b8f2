"""BGR24 pack / unpack throughput on 4K frames.

Algorithmic bytes: 3 B read + 4 B written per pixel (both directions).
Launches go to a dedicated torch stream (a non-NULL handle: NULL would select
the library's own stream), timed with torch.cuda.Event on that stream.
Prints one JSON line.  Usage: python tools/bench_bgr24.py [--frames 8] [--reps 50]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    a = ap.parse_args()
    pkg = load_package()
    w, h, f = a.width, a.height, a.frames
    n = w * h
    st = torch.cuda.Stream()
    bgr = [torch.randint(0, 256, (3 * n,), dtype=torch.uint8, device="cuda:0") for _ in range(f)]
    px = [torch.empty(n, dtype=torch.int32, device="cuda:0") for _ in range(f)]
    out = {}
    for name in ("pack", "unpack"):
        def step():
            for i in range(f):
                if name == "pack":
                    pkg.pack_bgr24_device(bgr[i], w, h, px[i], stream=st)
                else:
                    pkg.unpack_bgr24_device(px[i], w, h, bgr[i], stream=st)
        with torch.cuda.stream(st):
            for _ in range(5):
                step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(a.reps):
            step()
        e1.record(st)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / (a.reps * f)
        gbps = 7.0 * n / (us * 1e-6) / 1e9
        out[name] = {"us_per_frame": round(us, 2), "GBps": round(gbps, 1), "frac_of_8TBps": round(gbps / 8000, 4),
                     "Gpix_per_s": round(n / us / 1e3, 2)}
    print(json.dumps({"workload": "%d x %dx%d BGR24 frames, %d reps" % (f, w, h, a.reps),
                      "alg_bytes_per_pixel": 7, **out}))


if __name__ == "__main__":
    main()
