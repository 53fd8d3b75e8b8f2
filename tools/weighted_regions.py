#!/usr/bin/env python3
"""The app's live weighted call at region sizes.

ClusteringSegmentation.cpp:1779-1803 calls quant_recurse(N_region, ..., K=4,
allPixelsUnique=0) once per superpixel region, then map_colors_mps on the
region (:2434).  This times that call on the GPU (dq_hip_quant_weighted_dev:
calc_color_table + the exact ordered FP64 folds + dedup + map) at N ~ 10^3
.. 10^6 on square crops of the reference's sample image (tests/golden/png),
beside the reference build itself (oracle/_ref/libdqref.so, one core) on the
same inputs, and checks the GPU's colortable and output against the
reference's.  One JSON line per size.

    python3 tools/weighted_regions.py [--k 4] [--sides 32,100,316,1000]
"""
import argparse
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
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--sides", default="32,100,316,1000")
    ap.add_argument("--image", default="batman")
    ap.add_argument("--calls", type=int, default=0, help="GPU calls per size (0: by size)")
    a = ap.parse_args()
    import bench
    import torch
    from __graft_entry__ import load_package
    pkg = load_package()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream(dev)
    rows = bench.weighted_regions(pkg, torch, dev, stream, a.k, [int(s) for s in a.sides.split(",")],
                                  a.image, calls=a.calls)
    for r in rows:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
