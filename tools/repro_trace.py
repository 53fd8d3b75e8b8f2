"""Repeat one sample-image quant on the device path and compare every run with
the reference fixtures (ct, output hash, split trace); print the first
differing trace rows.  Development tool (nondeterminism hunt).

    python tools/repro_trace.py [name] [k] [reps] [plan 0|1]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import dq_fixtures as fx  # noqa: E402
from __graft_entry__ import load_package  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "batman"
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    pkg = load_package()
    if len(sys.argv) > 4:
        pkg.set_planned_rounds(sys.argv[4] == "1")
    fix = fx.load_json("png.json")[name]
    arrs = fx.load_npz("png.npz")
    px, w, h = fx.load_png_u32(os.path.join(fx.GOLDEN, "png", name + ".png"))
    ref_tr = arrs["trace_%s_k%d" % (name, k)]
    t_in = torch.from_numpy(np.ascontiguousarray(px, np.uint32).view(np.int32)).to("cuda:0")
    t_out = torch.empty_like(t_in)
    bad = 0
    for r in range(reps):
        ct, _ = pkg.quant_device(t_in, t_out, k)
        torch.cuda.synchronize()
        out = t_out.cpu().numpy().view(np.uint32)
        tr = pkg.last_trace(k)
        ok_ct = [int(v) for v in ct] == fix["k%d" % k]["ct"]
        ok_out = "%016x" % fx.fnv(out) == fix["k%d" % k]["out_fnv"]
        ok_tr = np.array_equal(tr, ref_tr)
        if not (ok_ct and ok_out and ok_tr):
            bad += 1
            rows = np.nonzero((tr != ref_tr).any(axis=1))[0] if tr.shape == ref_tr.shape else []
            print("rep %d: ct %s out %s trace %s; differing rows %s" % (r, ok_ct, ok_out, ok_tr, list(rows[:8])))
            for i in rows[:4]:
                print("   row %d: got %s ref %s" % (i, list(tr[i]), list(ref_tr[i])))
            print("   planned rounds %d of %d" % (pkg.last_planned_rounds(), pkg.last_rounds()))
    print("%s k=%d: %d of %d runs differ" % (name, k, bad, reps))


if __name__ == "__main__":
    main()
