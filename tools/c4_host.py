"""Host-side time of the C4 share (8 x 4K frames per call): the Python call's
wall time against the engine's own trace lines (DQ_HIP_TRACE=1, stderr).
Development tool.

    DQ_HIP_TRACE=1 python tools/c4_host.py [steps] [lanes]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from __graft_entry__ import load_package  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    lanes = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    pkg = load_package()
    if lanes:
        pkg.set_lanes(lanes)
    dev = torch.device("cuda:0")
    n = 3840 * 2160
    frames = []
    for f in range(8):
        px = pkg.synth_frame(n, f)
        frames.append(torch.from_numpy(px.view("int32")).to(dev))
    outs = [torch.empty_like(f) for f in frames]
    torch.cuda.synchronize()
    for _ in range(3):
        pkg.quant_batch_device(frames, outs, 256)
    torch.cuda.synchronize()
    for s in range(steps):
        t0 = time.perf_counter()
        pkg.quant_batch_device(frames, outs, 256)
        t1 = time.perf_counter()
        print("step %d: python call %.1f us" % (s, (t1 - t0) * 1e6), file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
