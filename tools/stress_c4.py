"""Repeat the C4 batch call (8 distinct 4K frames, seed + f) many times and
compare every call's colortables and outputs with the reference fixtures
(first call, by hash) and with the first call (later calls, on the GPU).
Development tool: hunting rare run-to-run differences.

    python tools/stress_c4.py CALLS [lanes ...]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import __graft_entry__ as ge  # noqa: E402
import dq_fixtures as fx  # noqa: E402


def main():
    calls = int(sys.argv[1])
    lanes = [int(x) for x in sys.argv[2:]] or [1, 3]
    pkg = ge.load_package()
    fix = fx.load_json("c4.json")
    w, h, k = 3840, 2160, 256
    frames = [torch.from_numpy(fx.xorshift(w * h, seed=fx.SEED + f).view(np.int32)).cuda() for f in range(8)]
    outs = [torch.empty_like(t) for t in frames]
    ref_out = None
    bad = 0
    for c in range(calls):
        pkg.set_lanes(lanes[c % len(lanes)])
        cts, _ = pkg.quant_batch_device(frames, outs, k)
        torch.cuda.synchronize()
        errs = []
        for f in range(8):
            if [int(v) for v in cts[f]] != fix["f%02d" % f]["ct"]:
                got = [int(v) for v in cts[f]]
                d = next((i for i, (x, y) in enumerate(zip(got, fix["f%02d" % f]["ct"])) if x != y), None)
                errs.append("f%d ct (first diff %s, k %d/%d)" % (f, d, len(got), len(fix["f%02d" % f]["ct"])))
        if ref_out is None:
            for f in range(8):
                if "%016x" % fx.fnv(outs[f].cpu().numpy().view(np.uint32)) != fix["f%02d" % f]["out_fnv"]:
                    errs.append("f%d out hash" % f)
            ref_out = [o.clone() for o in outs]
        else:
            for f in range(8):
                if not torch.equal(outs[f], ref_out[f]):
                    errs.append("f%d out (%d px differ)" % (f, int((outs[f] != ref_out[f]).sum())))
        if errs:
            bad += 1
            print("call %d lanes %d: %s" % (c, lanes[c % len(lanes)], "; ".join(errs)), flush=True)
        elif c % 100 == 0:
            print("call %d ok" % c, flush=True)
    print("calls %d, bad %d" % (calls, bad), flush=True)


if __name__ == "__main__":
    main()
