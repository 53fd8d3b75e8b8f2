"""Determinism / parity of device-planned rounds on the sample images.

    python tools/plan_debug.py [reps]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401
from __graft_entry__ import load_package  # noqa: E402
import dq_fixtures as fx  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
pkg = load_package()
png = fx.load_json("png.json")
for name in ("batman", "cookie"):
    px, w, h = fx.load_png_u32(os.path.join(fx.GOLDEN, "png", name + ".png"))
    for k in (16, 125, 256):
        fix = png[name]["k%d" % k]
        for plan in (0, 1):
            pkg.set_planned_rounds(plan)
            bad = 0
            for r in range(reps):
                out, ct = pkg.quant_recurse(px, k, 1)
                ok = [int(v) for v in ct] == fix["ct"] and "%016x" % fx.fnv(out) == fix["out_fnv"]
                bad += 0 if ok else 1
            print("%s k=%d plan=%d: %d/%d bad (rounds %d, planned %d)" %
                  (name, k, plan, bad, reps, pkg.last_rounds(), pkg.last_planned_rounds()), flush=True)
