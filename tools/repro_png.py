#!/usr/bin/env python3
"""GPU: the sample PNGs through the fused BGR24 path, one K at a time, with a
progress line before every call (stderr, unbuffered).
    python3 tools/repro_png.py NAME [K ...]   (K suffixed w: weighted)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import dq_fixtures as fx
    from test_bgr24 import _png_bgr
    from __graft_entry__ import load_package
    pkg = load_package()
    name = sys.argv[1]
    ks = sys.argv[2:] or ["4", "16", "125", "256", "4w", "16w"]
    fix = fx.load_json("png.json")[name]
    bgr, w, h = _png_bgr(name)
    d_bgr = torch.from_numpy(bgr.reshape(-1)).to("cuda:0")
    d_out = torch.empty(w * h, dtype=torch.int32, device="cuda:0")
    for ks_ in ks:
        weighted = ks_.endswith("w")
        k = int(ks_.rstrip("w"))
        print("call %s K=%d weighted=%d" % (name, k, weighted), file=sys.stderr, flush=True)
        ct, _ = pkg.quant_bgr24_device(d_bgr, w, h, d_out, k, all_pixels_unique=0 if weighted else 1)
        torch.cuda.synchronize()
        key = "k%d_weighted" % k if weighted else "k%d" % k
        ok = [int(v) for v in ct] == fix[key]["ct"] and \
            "%016x" % fx.fnv(d_out.cpu().numpy().view(np.uint32)) == fix[key]["out_fnv"]
        print("  ok=%s rounds=%d planned=%d" % (ok, pkg.last_rounds(), pkg.last_planned_rounds()),
              file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
