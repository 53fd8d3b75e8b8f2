"""Repeat one quant_device call on a fixed input and report run-to-run
differences (development tool: nondeterminism hunting).

    python tools/repeat_check.py [png-name|xorshift] K REPS [fixed_point 0/1] [planned 0/1]
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
    name, k, reps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    fp = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    plan = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    pkg = ge.load_package()
    if name == "xorshift":
        px = fx.xorshift(1 << 20, seed=21)
    else:
        px = fx.load_png_u32(os.path.join(fx.GOLDEN, "png", name + ".png"))[0]
    pkg.set_fixed_point(bool(fp))
    pkg.set_planned_rounds(bool(plan))
    t_in = torch.from_numpy(np.ascontiguousarray(px, np.uint32).view(np.int32)).to("cuda:0")
    outs = []
    for r in range(reps):
        t_out = torch.empty_like(t_in)
        ct, _ = pkg.quant_device(t_in, t_out, k)
        torch.cuda.synchronize()
        out = t_out.cpu().numpy().view(np.uint32).copy()
        tr = pkg.last_trace(k).copy()
        outs.append((out, np.asarray(ct).copy(), tr))
        o0, c0, t0 = outs[0]
        same = np.array_equal(out, o0) and np.array_equal(ct, c0) and np.array_equal(tr, t0)
        msg = "rep %d: %s" % (r, "same" if same else "DIFFERS")
        if not same:
            bad = np.nonzero((tr != t0).any(axis=1))[0]
            msg += " (out px differ %d, ct differ %d, first trace row %s: %s vs %s)" % (
                int((out != o0).sum()), int((np.asarray(ct) != c0).sum()),
                bad[:1], tr[bad[:1]].tolist(), t0[bad[:1]].tolist())
        print(msg, flush=True)


if __name__ == "__main__":
    main()
