#!/usr/bin/env python3
"""GPU: how often a later round partitions a record finalised at a frame's
last planned (PS_STATS) round -- the cursor fix-up path --
over the bench's batches and a K sweep, each call verified against the
reference build's fixtures where they exist (c4.json frames).
    python3 tools/cursor_fix_probe.py        (JSON lines)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from __graft_entry__ import load_package
    pkg = load_package()
    dev = torch.device("cuda", 0)
    w, h, k = bench.CONFIGS["c3"]
    for lanes in (1, 4):
        pkg.set_lanes(lanes)
        for f0 in (0, 8, 16, 24, 32, 40, 48, 56):
            ids = list(range(f0, f0 + 8))
            ts = bench.upload_frames(torch, pkg, dev, w, h, ids)
            outs = [torch.empty_like(t) for t in ts]
            cts, _ = pkg.quant_batch_device(ts, outs, k)
            torch.cuda.synchronize()
            ok = all(bench.check_frame(pkg, outs[i], cts[i], bench.frame_fixture(w, h, k, ids[i]))
                     for i in range(len(ids)))
            print(json.dumps({"lanes": lanes, "frames": ids, "cursor_fixes": pkg.last_cursor_fixes(),
                              "rounds": pkg.last_rounds(), "verified": ok}), flush=True)


if __name__ == "__main__":
    main()
