#!/usr/bin/env python3
"""GPU probe: which skewed 2 x 4K batches (one lane) send a later host round
into a record finalised at the PS_STATS last planned round (cursor fixes)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def design(name, n, seed):
    rng = np.random.default_rng(seed)
    if name == "noise99_flat1":
        px = rng.integers(0, 1 << 24, n, dtype=np.uint32)
        px[: n // 100] = 0x123456
    elif name == "noise50_flat4":
        px = np.empty(n, np.uint32)
        h = n // 2
        px[:h] = rng.integers(0, 1 << 24, h, dtype=np.uint32)
        px[h:] = np.repeat(np.array([0x102030, 0x405060, 0xA0B0C0, 0xF0E0D0], np.uint32), (n - h + 3) // 4)[:n - h]
    elif name == "two_cubes":
        px = rng.integers(0, 1 << 24, n, dtype=np.uint32)
        m = n // 5
        px[:m] = rng.integers(0, 16, m, dtype=np.uint32) * 0x010101 + 0x404040
    elif name == "gradient":
        i = np.arange(n, dtype=np.uint64)
        px = ((i * 2654435761) >> 8).astype(np.uint32) & 0x00FFFFFF
        px[: n // 2] &= 0x0F0F0F
    elif name == "powerlaw":
        r = (rng.pareto(1.5, n) * 20).clip(0, 255).astype(np.uint32)
        g = (rng.pareto(1.5, n) * 20).clip(0, 255).astype(np.uint32)
        b = (rng.pareto(1.5, n) * 20).clip(0, 255).astype(np.uint32)
        px = (r << 16) | (g << 8) | b
    return px


def main():
    import torch
    from __graft_entry__ import load_package
    pkg = load_package()
    pkg.set_lanes(1)
    n = 3840 * 2160
    for name in ("noise99_flat1", "noise50_flat4", "two_cubes", "gradient", "powerlaw"):
        ts = [torch.from_numpy(design(name, n, s).view(np.int32)).to("cuda:0") for s in (1, 2)]
        for k in (256, 100, 1000):
            outs = [torch.empty_like(t) for t in ts]
            pkg.quant_batch_device(ts, outs, k)
            torch.cuda.synchronize()
            print(json.dumps({"design": name, "k": k, "fixes": pkg.last_cursor_fixes(), "rounds": pkg.last_rounds(),
                              "planned": pkg.last_planned_rounds()}), flush=True)


if __name__ == "__main__":
    main()
