"""Time genHistogramsForBlocks on the GPU: full-frame map onto
the 125-colour palette + 4x4 block modes, on a synthetic 4K frame resident in
HBM, and the CPU oracle on the same frame (dqo_map + dqo_block_hist, one
thread).  Prints one JSON line.

    python tools/bench_blockhist.py [--w 3840 --h 2160 --steps 50]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--w", type=int, default=3840)
    ap.add_argument("--h", type=int, default=2160)
    ap.add_argument("--dim", type=int, default=4)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--cpu", type=int, default=1)
    args = ap.parse_args()
    import torch
    from __graft_entry__ import load_package
    import dq_fixtures as fx
    pkg = load_package()
    w, h, dim = args.w, args.h, args.dim
    # natural-image-like: smooth gradients + noise (many uniform blocks, some ties)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.int64)
    noise = fx.xorshift(w * h, seed=42).reshape(h, w).astype(np.int64)
    r = (xx * 255 // max(w - 1, 1) + (noise & 15)) & 0xFF
    g = (yy * 255 // max(h - 1, 1) + ((noise >> 8) & 15)) & 0xFF
    b = ((xx + yy) * 255 // (w + h) + ((noise >> 16) & 15)) & 0xFF
    frame = ((r << 16) | (g << 8) | b).astype(np.uint32)
    bw, bh = pkg.block_grid(w, h, dim)
    dev = torch.device("cuda:0")
    t_in = torch.from_numpy(frame.reshape(-1).view(np.int32)).to(dev)
    t_q = torch.empty_like(t_in)
    t_mode = torch.empty(bw * bh, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream()
    for _ in range(3):
        pkg.block_hist_device(t_in, w, h, t_q, t_mode, superpixel_dim=dim, stream=st)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(args.steps):
        pkg.block_hist_device(t_in, w, h, t_q, t_mode, superpixel_dim=dim, stream=st)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.steps
    out = {"metric": "block_hist_frames_per_s", "value": 1000.0 / ms, "ms_per_frame": ms,
           "width": w, "height": h, "dim": dim, "blocks": bw * bh,
           "gpix_per_s": w * h / ms / 1e6}
    if args.cpu:
        orc = fx.oracle()
        px = frame.reshape(-1)
        q = np.zeros_like(px)
        pal = fx.subdivided_colors()
        mode = np.zeros(bw * bh, np.uint32)
        t0 = time.perf_counter()
        orc.dqo_map(fx.vp(px), ctypes.c_uint32(px.size), fx.vp(q), fx.vp(pal), ctypes.c_int(125))
        orc.dqo_block_hist(fx.vp(q), ctypes.c_uint32(w), ctypes.c_uint32(h), ctypes.c_uint32(bw),
                           ctypes.c_uint32(bh), ctypes.c_uint32(dim), fx.vp(mode), None, None, None)
        cpu_s = time.perf_counter() - t0
        gpu_mode = t_mode.cpu().numpy().view(np.uint32)
        out.update({"cpu_port_s_per_frame": cpu_s, "cpu_cores": 1,
                    "match_oracle": bool(np.array_equal(gpu_mode, mode)),
                    })
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
