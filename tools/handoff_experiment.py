#!/usr/bin/env python3
"""GPU experiment: the C4 share (8 x 4K, K=256) under the hand-off debug knobs,
one engine lane, with the library named by DQ_HIP_LIB (e.g. a build of an
older protocol).  Prints per call which frames match the reference fixtures.

    DQ_HIP_LIB=path python3 tools/handoff_experiment.py FLAGS CALLS
"""
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
    flags, calls = int(sys.argv[1]), int(sys.argv[2])
    pkg = load_package()
    fix = fx.load_json("c4.json")
    t_in = [torch.from_numpy(fx.xorshift(3840 * 2160, seed=fx.SEED + f).view(np.int32)).to("cuda:0")
            for f in range(8)]
    t_out = [torch.empty_like(t) for t in t_in]
    pkg.set_lanes(1)
    pkg.set_debug(flags)
    bad = 0
    for c in range(calls):
        cts, _ = pkg.quant_batch_device(t_in, t_out, 256)
        torch.cuda.synchronize()
        res = []
        for f in range(8):
            ref = fix["f%02d" % f]
            ok_ct = [int(v) for v in cts[f]] == ref["ct"]
            ok_out = "%016x" % fx.fnv(t_out[f].cpu().numpy().view(np.uint32)) == ref["out_fnv"]
            res.append("ok" if ok_ct and ok_out else ("out" if ok_ct else "ct"))
        bad += sum(r != "ok" for r in res)
        print(json.dumps({"lib": os.path.basename(pkg.LIB_PATH), "flags": flags, "call": c, "frames": res}),
              flush=True)
    pkg.set_debug(0)
    print(json.dumps({"lib": os.path.basename(pkg.LIB_PATH), "flags": flags, "calls": calls,
                      "frames_wrong": bad}), flush=True)


if __name__ == "__main__":
    main()
