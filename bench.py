#!/usr/bin/env python3
"""bench.py -- DivQuant hot path (quant_recurse: cluster + dedup + map) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3] [--frames F]

One step = quant_recurse semantics (K=256, max_iters=10) on every frame this
rank owns (F synthetic uniform-random 24-bit RGB frames of the config's shape,
already resident in HBM).  N>1 (launched by torch.distributed.run, one rank per
GPU): frames are independent objects, so each rank owns its own F frames and
there is no data-path collective ("scaling": "weak"); the barrier and the
max-over-ranks timing use the process group only.

Prints ONE JSON line on rank 0.  `roofline` is measured live on the library's
stream with HIP events around every launch of the dominant kernel (the 2-means
statistics pass); `cpu_baseline` times the reference DivQuant (oracle/_ref,
built from the unmodified reference sources) or, if that build is absent, the
oracle's restatement, on one frame, on one host core, rank 0 only.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {   # BASELINE.json configs (C4/C5 are multi-GPU shapes)
    "c1": (256, 256, 16),
    "c2": (1920, 1080, 256),
    "c3": (3840, 2160, 256),
    "c5": (16384, 16384, 1024),
}
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--frames", type=int, default=1, help="frames per rank per step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="skip the HIP-event roofline region")
    return ap.parse_args()


def cpu_baseline(w, h, k):
    """Reference DivQuant on one frame, one core (rank 0, N=1 only)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import dq_fixtures as fx
    px = fx.xorshift(w * h)
    out = np.zeros(w * h, np.uint32)
    ct = np.zeros(k, np.uint32)
    kk = ctypes.c_uint32(k)
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libdqref.so")
    if os.path.exists(ref_so):
        lib = ctypes.CDLL(ref_so)
        kind = "reference"
        fn = lib.quant_recurse
        args = (ctypes.c_uint32(w * h), fx.vp(px), fx.vp(out), ctypes.byref(kk), fx.vp(ct), ctypes.c_int(1))
    else:
        lib = fx.oracle()
        kind = "port"
        fn = lib.dqo_quant_recurse
        args = (ctypes.c_uint32(w * h), fx.vp(px), fx.vp(out), ctypes.byref(kk), fx.vp(ct))
    # the reference prints two timer lines on stdout: keep our stdout one JSON line
    sys.stdout.flush()
    saved = os.dup(1)
    devnull = os.open(os.devnull, os.O_WRONLY)
    os.dup2(devnull, 1)
    try:
        t0 = time.perf_counter()
        fn(*args)
        dt = time.perf_counter() - t0
    finally:
        ctypes.CDLL(None).fflush(None)
        os.dup2(saved, 1)
        os.close(saved)
        os.close(devnull)
    return {"value": round(w * h / dt / 1e6, 4), "unit": "Mpix/s", "cores": 1, "kind": kind,
            "sample": "one %dx%d frame, K=%d, quant_recurse(allPixelsUnique=1), %.2f s, single thread "
                      "(host has %d cores)" % (w, h, k, dt, os.cpu_count() or 0)}


def init_dist():
    """(rank, world, local_rank) from the torchrun environment; one process
    per GPU over RCCL ("nccl"), or gloo without a GPU (CPU tests)."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        dist.init_process_group("nccl" if torch.cuda.is_available() else "gloo")
    return rank, world, local


def frame_seed(rank, frame):
    """Each rank owns its own frames (weak scaling, no data-path collective)."""
    return 0x5EED + 1000 * rank + frame


def timed_region(step, steps, world, sync):
    """Barrier + device sync on both sides of exactly `steps` steps."""
    import torch.distributed as dist
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if world > 1:
        dist.barrier()
    return time.perf_counter() - t0


def max_over_ranks(dt, world, device="cpu"):
    import torch
    import torch.distributed as dist
    if world == 1:
        return dt
    t = torch.tensor([dt], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def main():
    a = parse()
    import torch
    from __graft_entry__ import load_package

    rank, world, local = init_dist()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pkg = load_package()

    w, h, k = CONFIGS[a.config]
    n = w * h
    frames = []
    for f in range(a.frames):
        g = torch.Generator(device=dev)
        g.manual_seed(frame_seed(rank, f))
        frames.append(torch.randint(0, 1 << 24, (n,), dtype=torch.int32, device=dev, generator=g))
    outs = [torch.empty_like(f) for f in frames]
    stream = torch.cuda.current_stream(dev)

    def step():
        if a.frames == 1:
            pkg.quant_device(frames[0], outs[0], k, max_iters=10, device=local, stream=stream)
        else:   # one batched call: every pass of a round covers all frames
            pkg.quant_batch_device(frames, outs, k, max_iters=10, device=local, stream=stream)

    for _ in range(a.warmup):
        step()
    # --- timed region: no per-launch events (they would perturb the timing)
    pkg.set_timing(False, device=local)
    dt = timed_region(step, a.steps, world, lambda: torch.cuda.synchronize(dev))
    # --- roofline region: the same steps again with HIP events around every
    # launch (on the library's launch stream) for per-kernel durations
    timing = not a.no_timing
    stats = {}
    if timing:
        pkg.reset_stats(device=local)
        pkg.set_timing(True, device=local)
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize(dev)
        pkg.set_timing(False, device=local)
        stats = pkg.get_stats(device=local)
    rounds = pkg.last_rounds(device=local)
    swept = pkg.last_points_swept(device=local)

    dt = max_over_ranks(dt, world, dev)
    total_px = n * a.frames * a.steps * world
    value = total_px / dt / 1e6

    if rank == 0:
        km = stats.get("pass_kmeans", (0, 0.0, 0.0))
        roof = None
        if timing and km[0] > 0 and km[1] > 0:
            gbs = km[2] / (km[1] / 1e3) / 1e9
            roof = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None,
                    "kernel": "pass_kernel<PASS_KMEANS>",
                    "launches": km[0], "avg_launch_us": round(km[1] * 1e3 / km[0], 2),
                    "alg_bytes_per_launch": round(km[2] / km[0])}
        # whole-pipeline algorithmic bytes (BASELINE.md B_alg = 4N + 44*sum|C_j| + 8N)
        per_frame_ms = dt * 1e3 / (a.steps * a.frames)
        res = {
            "metric": "Mpixels/sec DivQuant K=%d on %dx%d RGB" % (k, w, h),
            "value": round(value, 2),
            "unit": "Mpix/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt * 1e3 / a.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8x3 pixels, u64 sums, f64 epilogue",
            "data": "synthetic uniform-random 24-bit RGB frames (torch.randint on device)",
            "config": {"workload": "quant_recurse %dx%d K=%d max_iters=10 (cluster+dedup+map)" % (w, h, k),
                       "frames_per_rank_per_step": a.frames, "parallelism": "frames-per-rank x%d" % world},
            "roofline": roof,
            "detail": {"ms_per_frame": round(per_frame_ms, 3), "rounds_last_frame": rounds,
                       "points_swept_last_frame": swept,
                       "kernels": {kname: {"launches": v[0], "ms": round(v[1], 3),
                                           "GBps": round(v[2] / (v[1] / 1e3) / 1e9, 1) if v[1] > 0 and v[2] > 0 else None}
                                   for kname, v in stats.items() if v[0]}},
        }
        if world == 1 and not a.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(w, h, k)
        print(json.dumps(res), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
