"""test_fixed_point_finalisation_is_exact's sequence, repeated, reporting every
mismatch (development tool: nondeterminism hunting).

    python tools/repeat_fp.py REPS
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


def run(pkg, px, k):
    t_in = torch.from_numpy(np.ascontiguousarray(px, np.uint32).view(np.int32)).to("cuda:0")
    t_out = torch.empty_like(t_in)
    ct, _ = pkg.quant_device(t_in, t_out, k)
    torch.cuda.synchronize()
    return t_out.cpu().numpy().view(np.uint32).copy(), np.asarray(ct).copy(), pkg.last_trace(k).copy()


def main():
    reps = int(sys.argv[1])
    pkg = ge.load_package()
    cases = [("xs1M", fx.xorshift(1 << 20, seed=21)), ("xs300k", fx.xorshift(300000, seed=22) & 0xF8FCF8)]
    for name in ("batman", "cookie"):
        cases.append((name, fx.load_png_u32(os.path.join(fx.GOLDEN, "png", name + ".png"))[0]))
    ref = {}
    bad = 0
    for r in range(reps):
        for name, px in cases:
            for k in (16, 256):
                for fp, plan in ((0, 1), (1, 0), (1, 1)):
                    pkg.set_fixed_point(bool(fp))
                    pkg.set_planned_rounds(bool(plan))
                    out, ct, tr = run(pkg, px, k)
                    key = (name, k)
                    if key not in ref:
                        ref[key] = (out, ct, tr, fp, plan)
                        continue
                    o0, c0, t0, fp0, pl0 = ref[key]
                    if not (np.array_equal(out, o0) and np.array_equal(ct, c0) and np.array_equal(tr, t0)):
                        bad += 1
                        rows = np.nonzero((tr != t0).any(axis=1))[0]
                        print("rep %d %s k=%d fp=%d plan=%d DIFFERS from fp=%d plan=%d: px %d, ct %d, trace rows %s"
                              % (r, name, k, fp, plan, fp0, pl0, int((out != o0).sum()),
                                 int((ct != c0).sum()) if len(ct) == len(c0) else -1, rows[:8].tolist()),
                              flush=True)
                        if len(rows):
                            print("   first row got %s want %s" % (tr[rows[0]].tolist(), t0[rows[0]].tolist()))
        print("rep %d done, mismatches so far %d" % (r, bad), flush=True)
    pkg.set_fixed_point(True)
    pkg.set_planned_rounds(True)


if __name__ == "__main__":
    main()
