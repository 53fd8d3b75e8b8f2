#!/usr/bin/env python3
"""GPU: the weighted path (allPixelsUnique = 0) on 4K frames -- uniform noise
(6.6 M unique colours) and a duplicate-heavy one (12-bit colours) -- timed,
with outputs compared to a second library (DQ_HIP_REF_LIB, e.g. round 2's
lane-0 ordered folds) when given.   python3 tools/weighted_timing.py [calls]"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def run(pkg, t_in, t_out, k, calls):
    import torch
    ts = []
    for _ in range(calls):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ct, _ = pkg.quant_device(t_in, t_out, k, all_pixels_unique=0)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    return ct, t_out.cpu().numpy().view(np.uint32).copy(), ts


def main():
    import torch
    import dq_fixtures as fx
    from __graft_entry__ import load_package
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    pkg = load_package()
    n = 3840 * 2160
    frames = {"noise": fx.xorshift(n), "dup12": fx.xorshift(n, seed=fx.SEED + 77) & 0xF0F0F0}
    ref = None
    if os.environ.get("DQ_HIP_REF_LIB"):
        ref = ctypes.CDLL(os.environ["DQ_HIP_REF_LIB"])
    out = {}
    for name, px in frames.items():
        for k in (4, 256):
            t_in = torch.from_numpy(px.view(np.int32)).to("cuda:0")
            t_out = torch.empty_like(t_in)
            ct, o, ts = run(pkg, t_in, t_out, k, calls)
            rec = {"ms": [round(x, 2) for x in ts], "k_out": len(ct), "seq_tiles": pkg.last_seq_tiles(),
                   "rounds": pkg.last_rounds(), "ct_hash": "%016x" % fx.fnv(np.asarray(ct, np.uint32)),
                   "out_hash": "%016x" % fx.fnv(o)}
            if ref is not None:
                kk = ctypes.c_uint32(k)
                rct = np.zeros(k, np.uint32)
                t_o2 = torch.empty_like(t_in)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                ref.dq_hip_quant_weighted_dev(0, ctypes.c_void_p(t_in.data_ptr()), ctypes.c_uint32(n),
                                              ctypes.c_void_p(t_o2.data_ptr()), ctypes.byref(kk),
                                              ctypes.c_void_p(rct.ctypes.data), 10, None)
                torch.cuda.synchronize()
                rec["ref_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
                rec["same_as_ref"] = bool([int(v) for v in ct] == [int(v) for v in rct[:kk.value]] and
                                          np.array_equal(o, t_o2.cpu().numpy().view(np.uint32)))
            out["%s_k%d" % (name, k)] = rec
            print(json.dumps({name + "_k%d" % k: rec}), flush=True)


if __name__ == "__main__":
    main()
