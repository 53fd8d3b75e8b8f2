#!/usr/bin/env python3
"""bench.py -- DivQuant hot path (quant_recurse: cluster + dedup + map) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3]
                    [--mode frames|rows] [--frames F]

Workload (BASELINE.json metric "Mpixels/sec DivQuant K=256 on 4K RGB"):

* --mode frames (default): one step = quant_recurse (K=256, max_iters=10,
  cluster + colortable dedup + map) on each of the F synthetic uniform-random
  24-bit 3840x2160 frames this rank owns, already resident in HBM, in ONE
  batched call (every pass of a split round is one launch over all F frames).
  Default F = 8: C4's per-GPU share (C4 = 64 4K frames over 8 GPUs, so
  --gpus 8 is exactly C4).  Frames are independent objects: no data-path
  collective, "scaling": "weak".  The single-frame latency of C3 (one 4K
  frame per call) is measured in the same run and reported in detail.c3.
* --mode rows: ONE frame of the config (e.g. --config c5: the 16384x16384
  K=1024 gigapixel tile) row-tile sharded over the N ranks; every pass's
  integer node totals are allreduced with RCCL over xGMI ("scaling":
  "strong": the total work is fixed).

N>1 is launched by torch.distributed.run, one rank per GPU.  Prints ONE JSON
line on rank 0.  `roofline` is the kernel with the largest measured time in
the step, timed live on the library's stream with HIP events around every
launch, against the 8 TB/s HBM peak; `traffic` comes from the committed
rocprofv3 PMC counters of the same command (profiles/pmc_traffic.json, see
tools/pmc_bench.sh) when they exist.  `cpu_baseline` times the reference
DivQuant (oracle/_ref, built from the unmodified reference sources) -- or,
if that build is absent, the oracle's restatement -- on one 4K frame, one
host core, rank 0 at N=1 only.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

# The engine overlaps frames on two lanes (HIP streams); with HIP's default
# of 4 hardware queues per process the lanes' streams and torch's sometimes
# share a queue and serialise (measured: ~1 run in 5 at the one-lane speed).
# 8 queues keep them apart; set before HIP initialises (torch import).
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {   # BASELINE.json configs (C4 = 64 x c3 frames; C5 = c5 row-sharded)
    "c1": (256, 256, 16),
    "c2": (1920, 1080, 256),
    "c3": (3840, 2160, 256),
    "c5": (16384, 16384, 1024),
}
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# algorithmic bytes of the kernel kinds the roofline may name (bytes per point
# the engine attributes to each launch: 4 read, +4 written for the partition)
ROOF_KERNELS = {"pass_kmeans": "pass_kernel<PASS_KMEANS>", "partition": "partsplit_kernel",
                "pass_split": "pass_kernel<PASS_SPLIT>", "pass_init": "pass_kernel<PASS_INIT>",
                "map": "map_kernel"}
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--mode", default="frames", choices=["frames", "rows"])
    ap.add_argument("--frames", type=int, default=8, help="frames per rank per step (frames mode)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="skip the HIP-event roofline region")
    ap.add_argument("--no-c3", action="store_true", help="skip the single-frame C3 measurement")
    ap.add_argument("--lanes", type=int, default=0,
                    help="engine lanes per batch (0: library default); the roofline region always uses 1")
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


def row_range(h, rank, world):
    """Row-tile sharding: rank r owns rows [r*H/N, (r+1)*H/N)."""
    return h * rank // world, h * (rank + 1) // world


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


def pick_roofline(stats, pmc_key):
    """The roofline object of the kernel kind with the largest measured time."""
    cand = {k: v for k, v in stats.items() if k in ROOF_KERNELS and v[0] > 0 and v[1] > 0 and v[2] > 0}
    if not cand:
        return None
    kind = max(cand, key=lambda k: cand[k][1])
    launches, ms, alg = cand[kind]
    gbs = alg / (ms / 1e3) / 1e9
    roof = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None,
            "kernel": ROOF_KERNELS[kind], "launches": launches,
            "avg_launch_us": round(ms * 1e3 / launches, 2),
            "alg_bytes_per_launch": round(alg / launches),
            "share_of_step_kernel_time": round(ms / sum(v[1] for v in stats.values() if v[1] > 0), 3),
            "measured": "HIP events around every launch on the engine's stream, one engine lane "
                        "(kernels not overlapped), same workload as the timed region"}
    if os.path.exists(PMC_FILE):
        try:
            pmc = json.load(open(PMC_FILE)).get(pmc_key, {}).get(ROOF_KERNELS[kind])
        except ValueError:
            pmc = None
        if pmc:
            roof["traffic"] = round(pmc["hbm_bytes_per_launch"])
            roof["traffic_source"] = pmc["source"]
    return roof


def main():
    a = parse()
    import torch
    from __graft_entry__ import load_package

    rank, world, local = init_dist()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pkg = load_package()
    stream = torch.cuda.current_stream(dev)

    w, h, k = CONFIGS[a.config]
    n = w * h
    if a.mode == "frames":
        nf = a.frames
        frames = []
        for f in range(nf):
            g = torch.Generator(device=dev)
            g.manual_seed(frame_seed(rank, f))
            frames.append(torch.randint(0, 1 << 24, (n,), dtype=torch.int32, device=dev, generator=g))
        outs = [torch.empty_like(f) for f in frames]

        def step():   # one batched call: every pass of a round covers all frames
            if nf == 1:
                pkg.quant_device(frames[0], outs[0], k, max_iters=10, device=local, stream=stream)
            else:
                pkg.quant_batch_device(frames, outs, k, max_iters=10, device=local, stream=stream)
        px_per_step = n * nf * world
        workload = ("C4 per-GPU share: %d x %dx%d frames per rank per step, K=%d, quant_recurse "
                    "max_iters=10 (cluster + dedup + map), one batched call" % (nf, w, h, k)
                    if nf > 1 else "C3: one %dx%d frame per step, K=%d, quant_recurse" % (w, h, k))
        parallelism = "frames-per-rank x%d" % world
        scaling = "weak"
    else:
        if world > 1:
            pkg.comm_init_torch(device=local)
        r0, r1 = row_range(h, rank, world)
        g = torch.Generator(device=dev)
        g.manual_seed(frame_seed(0, 0))   # the same frame on every rank; each keeps its rows
        mine = torch.empty(((r1 - r0) * w,), dtype=torch.int32, device=dev)
        # generate the frame row-block by row-block (no full copy needed on any rank)
        for rb in range(0, h, 1024):
            blk = torch.randint(0, 1 << 24, (min(1024, h - rb) * w,), dtype=torch.int32, device=dev,
                                generator=g)
            lo, hi = max(rb, r0), min(rb + 1024, r1)
            if lo < hi:
                mine[(lo - r0) * w:(hi - r0) * w] = blk[(lo - rb) * w:(hi - rb) * w]
        out = torch.empty_like(mine)

        def step():
            pkg.quant_rows_device([mine], [out], k, widths=[w], n_globals=[n], nshard=1,
                                  max_iters=10, device=local, stream=stream)
        nf = 1
        px_per_step = n
        workload = ("%s: one %dx%d frame, K=%d, row-tile sharded over %d rank(s), RCCL allreduce "
                    "of the node totals per pass" % (a.config.upper(), w, h, k, world))
        parallelism = "row-tiles x%d" % world
        scaling = "strong"

    pkg.set_lanes(a.lanes)
    lanes = pkg.get_lanes()
    for _ in range(a.warmup):
        step()
    # --- timed region: no per-launch events (they would perturb the timing)
    pkg.set_timing(False, device=local)
    dt = timed_region(step, a.steps, world, lambda: torch.cuda.synchronize(dev))
    # --- roofline region: the same steps again with HIP events around every
    # launch (on the library's launch stream) for per-kernel durations
    stats = {}
    if not a.no_timing:
        # kernels measured un-overlapped: one engine lane, so an event pair
        # around a launch times that kernel alone on the GPU
        pkg.set_lanes(1)
        step()
        pkg.reset_stats(device=local)
        pkg.set_timing(True, device=local)
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize(dev)
        pkg.set_timing(False, device=local)
        stats = pkg.get_stats(device=local)
        pkg.set_lanes(a.lanes)
    rounds = pkg.last_rounds(device=local)
    swept = pkg.last_points_swept(device=local)
    full = pkg.last_points_full(device=local)

    # --- C3 single-frame latency (same frame shape, one frame per call)
    c3 = None
    if a.mode == "frames" and not a.no_c3 and nf > 1:
        def one():
            pkg.quant_device(frames[0], outs[0], k, max_iters=10, device=local, stream=stream)
        for _ in range(2):
            one()
        dt1 = timed_region(one, a.steps, world, lambda: torch.cuda.synchronize(dev))
        dt1 = max_over_ranks(dt1, world, dev)
        c3 = {"ms_per_frame": round(dt1 * 1e3 / a.steps, 3),
              "Mpix_per_s": round(n * world * a.steps / dt1 / 1e6, 2),
              "workload": "one %dx%d frame per call (C3), %d rank(s)" % (w, h, world)}

    dt = max_over_ranks(dt, world, dev)
    value = px_per_step * a.steps / dt / 1e6

    if rank == 0:
        pmc_key = "%s_%s_f%d_n%d" % (a.mode, a.config, nf, world)
        roof = pick_roofline(stats, pmc_key) if stats else None
        # whole-pipeline algorithmic bytes (B_alg = 4N + 44*sum|C_j| + 8N;
        # sum|C_j| = log2(K) N for uniform inputs)
        lk = int(round(np.log2(k)))
        b_alg = (4 + 44 * lk + 8) * px_per_step * a.steps
        res = {
            "metric": "Mpixels/sec DivQuant K=%d on %dx%d RGB" % (k, w, h),
            "value": round(value, 2),
            "unit": "Mpix/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt * 1e3 / a.steps, 3),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u8x3 pixels in u32, u32/u64 integer sums, f64 updates",
            "data": "synthetic uniform-random 24-bit RGB frames (torch.randint on device)",
            "config": {"workload": workload, "frames_per_rank_per_step": nf if a.mode == "frames" else None,
                       "engine_lanes": lanes if a.mode == "frames" else 1,
                       "width": w, "height": h, "k": k, "max_iters": 10, "parallelism": parallelism},
            "roofline": roof,
            "detail": {"ms_per_frame": round(dt * 1e3 / a.steps / (nf * world if a.mode == "frames" else 1), 3),
                       "pipeline_alg_GBps": round(b_alg / dt / 1e9, 1),
                       "pipeline_alg_frac_per_gpu": round(b_alg / dt / 1e9 / (HBM_PEAK_GBS * world), 4),
                       "rounds_last_frame": rounds, "points_swept_last_call": swept,
                       "points_full_iterations_last_call": full,
                       "c3": c3,
                       "kernels": {kname: {"launches": v[0], "ms": round(v[1], 3),
                                           "GBps": round(v[2] / (v[1] / 1e3) / 1e9, 1) if v[1] > 0 and v[2] > 0 else None}
                                   for kname, v in stats.items() if v[0]}},
        }
        if world == 1 and not a.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(3840, 2160, 256)
        print(json.dumps(res), flush=True)
    if world > 1:
        import torch.distributed as dist
        if a.mode == "rows":
            pkg.comm_destroy(device=local)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
