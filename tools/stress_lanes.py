#!/usr/bin/env python3
"""GPU: repeated 8 x 4K batch calls over the default engine lanes (run it with
GPU_MAX_HW_QUEUES=8 for the 4-lane default), interleaved with single-frame
calls: every call's colortables against the reference's fixtures, the output
hashes every 50th call.  Prints one JSON line.
    python3 tools/stress_lanes.py [calls]"""
import json
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
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    w, h = 3840, 2160
    fix = fx.load_json("c4.json")
    ins = [torch.from_numpy(fx.xorshift(w * h, seed=fx.SEED + f).view(np.int32)).to("cuda:0") for f in range(8)]
    outs = [torch.empty_like(t) for t in ins]
    bad = []
    t0 = time.perf_counter()
    for c in range(calls):
        if c % 5 == 4:   # a single-frame call between batches
            ct, _ = pkg.quant_device(ins[c % 8], outs[c % 8], 256)
            cts = {c % 8: ct}
        else:
            got, _ = pkg.quant_batch_device(ins, outs, 256)
            cts = dict(enumerate(got))
        torch.cuda.synchronize()
        for f, ct in cts.items():
            if [int(v) for v in ct] != fix["f%02d" % f]["ct"]:
                bad.append({"call": c, "frame": f, "what": "colortable"})
        if c % 50 == 0:
            for f in cts:
                if "%016x" % fx.fnv(outs[f].cpu().numpy().view(np.uint32)) != fix["f%02d" % f]["out_fnv"]:
                    bad.append({"call": c, "frame": f, "what": "output hash"})
        if bad:
            break
    print(json.dumps({"calls": c + 1, "lanes": pkg.get_lanes(), "seconds": round(time.perf_counter() - t0, 1),
                      "bad": bad[:5], "ok": not bad}), flush=True)
    sys.exit(0 if not bad else 1)


if __name__ == "__main__":
    main()
