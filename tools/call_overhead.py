"""Fixed per-call cost of the batched C ABI: 8 tiny frames (4096 px), K=16."""
import sys, time
sys.path.insert(0, ".")
import torch
from __graft_entry__ import load_package
pkg = load_package()
dev = torch.device("cuda:0")
for npx in (4096, 65536):
    frames = [torch.randint(0, 1 << 24, (npx,), dtype=torch.int32, device=dev) for _ in range(8)]
    outs = [torch.empty_like(f) for f in frames]
    for lanes in (1, 2):
        pkg.set_lanes(lanes)
        for _ in range(5):
            pkg.quant_batch_device(frames, outs, 16)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(50):
            pkg.quant_batch_device(frames, outs, 16)
        torch.cuda.synchronize()
        print("px %6d lanes %d: %.1f us per call" % (npx, lanes, (time.perf_counter() - t0) / 50 * 1e6), flush=True)
