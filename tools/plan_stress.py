"""Stress device-planned rounds against host-planned ones: many inputs in a
random order (stale buffers from the previous call differ every time).

    python tools/plan_stress.py [iters] [seed]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
from __graft_entry__ import load_package  # noqa: E402
import dq_fixtures as fx  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 100
rng = np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 1)
os.environ["DQ_HIP_QUIET"] = "1"
pkg = load_package()
imgs = [fx.load_png_u32(os.path.join(fx.GOLDEN, "png", n + ".png"))[0] for n in ("batman", "cookie")]
cases = []
for px in imgs:
    for k in (4, 16, 125, 256):
        cases.append((px, k))
for s in range(4):
    cases.append((fx.xorshift(200000 + 77777 * s, seed=900 + s) & [0xFFFFFF, 0xF0F0F0, 0xE0C0E0, 0xFFFFFF][s],
                  [64, 256, 32, 1024][s]))
dev = torch.device("cuda:0")
tins = [torch.from_numpy(np.ascontiguousarray(px).view(np.int32)).to(dev) for px, _ in cases]
tout = [torch.empty_like(t) for t in tins]


def run(i):
    ct, _ = pkg.quant_device(tins[i], tout[i], cases[i][1])
    torch.cuda.synchronize()
    return ct, tout[i].cpu().numpy().copy(), pkg.last_trace(cases[i][1])


pkg.set_planned_rounds(False)
ref = [run(i) for i in range(len(cases))]
pkg.set_planned_rounds(True)
bad = 0
for it in range(iters):
    i = int(rng.integers(len(cases)))
    ct, out, tr = run(i)
    ok = np.array_equal(ct, ref[i][0]) and np.array_equal(out, ref[i][1]) and np.array_equal(tr, ref[i][2])
    if not ok:
        bad += 1
        d = np.nonzero(np.any(tr != ref[i][2], axis=1))[0] if tr.shape == ref[i][2].shape else [-1]
        print("MISMATCH iter %d case %d (n=%d k=%d): first trace diff at split %s; rounds %d planned %d"
              % (it, i, len(cases[i][0]), cases[i][1], d[:3], pkg.last_rounds(), pkg.last_planned_rounds()),
              flush=True)
print("stress: %d / %d mismatches" % (bad, iters), flush=True)
