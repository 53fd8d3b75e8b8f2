#!/usr/bin/env python3
"""bench.py -- DivQuant hot path (quant_recurse: cluster + dedup + map) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3]
                    [--mode frames|rows] [--frames F]

Workload (BASELINE.json metric "Mpixels/sec DivQuant K=256 on 4K RGB"):

* --mode frames (default): one step = quant_recurse (K=256, max_iters=10,
  cluster + colortable dedup + map) on each of the F synthetic 3840x2160
  frames this rank owns, already resident in HBM, in ONE batched call.
  Default F = 8: C4's per-GPU share (C4 = 64 4K frames over 8 GPUs, so
  --gpus 8 is exactly C4).  Frames are independent objects: no data-path
  collective, "scaling": "weak".  The same run also measures, each verified
  against the reference build's outputs:
    detail.c3         C3: one 4K frame per call;
    detail.c2         C2: one 1920x1080 frame per call, K=256;
    detail.c5         C5: the 16384x16384 K=1024 tile, its rows split over the
                      N ranks, one RCCL allreduce of the node totals per pass
                      (N=1: the whole tile on one GPU);
    detail.c4_rowtile C4's row-tile variant: all 64 frames, each row-sharded
                      over the N ranks, one allreduce of every frame's node
                      totals per pass;
    detail.bgr24_input the C3 frame and the rank's batch as BGR24 Mats;
    detail.weighted_c3 the C3 frame through the weighted path
                      (allPixelsUnique=0, the app's live call);
    detail.weighted_regions that call at the app's region sizes (10^3 -
                      10^6 pixels, K=4) beside the reference build.
* --mode rows: F frames of the config (default 1; --config c5: the
  16384x16384 K=1024 gigapixel tile) row-tile sharded over the N ranks
  ("scaling": "strong": the total work is fixed).

--gpus N > 1 without a torchrun environment launches N ranks itself
(torch.distributed.run, one process per GPU, RCCL over xGMI) before any GPU
call in this process; every rank asserts the world size is N.

Frames are the SURVEY 8c/8d generator (xorshift64, frame f = seed + f); the
outputs of the timed work are checked against the reference build's golden
fixtures (tests/golden/c4.json, big.json) after the timed region and the run
FAILS on a mismatch ("verified" fields).  Prints ONE JSON line on rank 0.
`roofline` is the kernel with the largest measured time in the step, timed
live on the library's stream with HIP events around every launch, against
the 8 TB/s HBM peak, with its bytes from the engine work model
and SURVEY 8(d)'s model beside it; `traffic` comes from the committed
rocprofv3 PMC counters (profiles/pmc_traffic.json).  `cpu_baseline` times the
reference DivQuant (oracle/_ref, built from the unmodified reference sources)
-- or, if that build is absent, the oracle's restatement -- on one 4K frame,
one host core, rank 0 at N=1 only.
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

# HIP's hardware queues per process (its default is 4): one per engine lane
# plus the caller's stream, set before anything initialises HIP -- the
# library then runs 4 lanes per batch (dq_engine.cpp batch_lanes)
# (GPU_MAX_HW_QUEUES is read once, when HIP initialises: it must be set
# before any HIP call of the process; the bench line records it)
_HWQ = int(os.environ.get("DQ_BENCH_HW_QUEUES", "8"))   # (A/B: the queue count to run with)
_HWQ_CALLER = os.environ.get("GPU_MAX_HW_QUEUES")
if int(_HWQ_CALLER or 4) != _HWQ:
    os.environ["GPU_MAX_HW_QUEUES"] = str(_HWQ)

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")

CONFIGS = {   # BASELINE.json configs (C4 = 64 x c3 frames; C5 = c5 row-sharded)
    "c1": (256, 256, 16),
    "c2": (1920, 1080, 256),
    "c3": (3840, 2160, 256),
    "c5": (16384, 16384, 1024),
}
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# kernel kinds the roofline may name -> (kernel symbol, engine-model bytes per
# point as stated in DESIGN.md 5, SURVEY 8(d)-model bytes per point).  Engine
# model: a pass reads 4 B per point of the caller's packed frame (the roots)
# and 3 B per point of the planar working buffers; the fused partition +
# split pass reads 4 or 3 B and writes 3 B per parent point; the map reads
# 4 B and writes 4 B per pixel.  The engine counts these bytes per launch
# (dq_hip_get_stat); SURVEY 8(d) counts 4 B per point read and classes the
# partition's write as overhead.
ROOF_KERNELS = {"pass_kmeans": ("kpass_kernel<PASS_KMEANS>", "3 B read per swept point", 4),
                "partition": ("partsplit_kernel", "3 B read (4 B from a root's packed frame) + 3 B written "
                              "per parent point", 4),
                "pass_split": ("pass_kernel<PASS_SPLIT>", "4 B read per root point, 3 B per other point", 4),
                "pass_init": ("pass_kernel<PASS_INIT>", "4 B read per point (packed frames)", 4),
                "map": ("map_lds_kernel", "4 B read + 4 B written per pixel", 8)}
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default=None, choices=sorted(CONFIGS),
                    help="default: c3 (frames mode), c5 (rows mode)")
    ap.add_argument("--mode", default="frames", choices=["frames", "rows"])
    ap.add_argument("--frames", type=int, default=None,
                    help="frames per rank per step (frames mode, default 8) / frames per step (rows, default 1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="skip the HIP-event roofline region")
    ap.add_argument("--no-c3", action="store_true", help="skip the single-frame C3 measurement")
    ap.add_argument("--no-weighted", action="store_true", help="skip the weighted-path (allPixelsUnique=0) C3 leg")
    ap.add_argument("--no-c2", action="store_true", help="skip the C2 (1080p K=256) measurement")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 (16384^2 K=1024) measurement")
    ap.add_argument("--no-rowtile", action="store_true", help="skip the C4 row-tile measurement")
    ap.add_argument("--no-bgr", action="store_true", help="skip the BGR24-input measurements")
    ap.add_argument("--no-verify", action="store_true", help="skip the golden-fixture check")
    ap.add_argument("--lanes", type=int, default=0,
                    help="engine lanes per batch (0: library default); the roofline region always uses 1")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher and timing harness only (no GPU work; the CPU tests use it)")
    a = ap.parse_args(argv)
    if a.config is None:
        a.config = "c5" if a.mode == "rows" else "c3"
    if a.frames is None:
        a.frames = 8 if a.mode == "frames" else 1
    return a


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(a):
    """--gpus N > 1 without a torchrun environment: run this script as N
    ranks under torch.distributed.run (one process per GPU) and return their
    exit code.  Nothing here touches the GPU (the ranks do)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(a.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "1"))
    return subprocess.call(cmd, env=env)


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
            "sample": "one %dx%d frame (synthetic frame 0), K=%d, quant_recurse(allPixelsUnique=1), "
                      "%.2f s, single thread (host has %d cores)" % (w, h, k, dt, os.cpu_count() or 0)}


class _Quiet:
    """fd 1 to /dev/null around the reference's calls (it prints two timer
    lines per quant_recurse on stdout: the bench keeps stdout one JSON line)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        self.null = os.open(os.devnull, os.O_WRONLY)
        os.dup2(self.null, 1)

    def __exit__(self, *exc):
        ctypes.CDLL(None).fflush(None)
        os.dup2(self.saved, 1)
        os.close(self.saved)
        os.close(self.null)


def cpu_baseline_regions(regions, k, min_s=0.25):
    """cpu_baseline for the weighted regions leg: the reference build
    (oracle/_ref, one core) on each region, quant_recurse(K, allPixelsUnique=0)
    -- ClusteringSegmentation.cpp:1779-1803's call -- timed over repeated calls
    (at least min_s of CPU time per region), and its outputs, which the GPU's
    are checked against.  None when the reference build is absent."""
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libdqref.so")
    if not os.path.exists(ref_so):
        return None
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import dq_fixtures as fx
    lib = ctypes.CDLL(ref_so)
    res = []
    for px in regions:
        n = px.size
        out = np.zeros(n, np.uint32)
        ct = np.zeros(k, np.uint32)
        calls, t = 0, 0.0
        with _Quiet():
            while t < min_s or calls < 1:
                kk = ctypes.c_uint32(k)
                t0 = time.perf_counter()
                lib.quant_recurse(ctypes.c_uint32(n), fx.vp(px), fx.vp(out), ctypes.byref(kk), fx.vp(ct),
                                  ctypes.c_int(0))
                t += time.perf_counter() - t0
                calls += 1
        res.append({"us": t / calls * 1e6, "calls": calls, "out": out.copy(), "ct": ct[:kk.value].copy()})
    return res


def weighted_regions(pkg, torch, dev, stream, k, sides, image="batman", calls=0, cpu=True):
    """The app's live weighted call at region sizes: square crops side x side
    of the reference's sample image (tests/golden/png), quant_recurse(K,
    allPixelsUnique=0) per call on device-resident pixels (one region per
    call, synchronised like the app's loop over regions), beside the reference
    build on the same crops; GPU outputs checked against the reference's."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import dq_fixtures as fx
    img, w, h = fx.load_png_u32(os.path.join(GOLDEN, "png", image + ".png"))
    img = img.reshape(h, w)
    regions = []
    for s in sides:
        s = min(s, w, h)
        y0, x0 = (h - s) // 2, (w - s) // 2
        regions.append(np.ascontiguousarray(img[y0:y0 + s, x0:x0 + s]).reshape(-1))
    refs = cpu_baseline_regions(regions, k) if cpu else None
    rows = []
    for i, px in enumerate(regions):
        n = px.size
        t_in = torch.from_numpy(px.view(np.int32)).to(dev)
        t_out = torch.empty_like(t_in)
        nc = calls or max(20, min(400, int(2e6 / max(n, 1))))
        last = {}

        def one():
            last["ct"], _ = pkg.quant_device(t_in, t_out, k, max_iters=10, stream=stream, all_pixels_unique=0)
        for _ in range(3):
            one()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(nc):
            one()
            torch.cuda.synchronize(dev)   # (the app's loop uses each region's result before the next)
        gpu_us = (time.perf_counter() - t0) / nc * 1e6
        row = {"n": int(n), "side": int(round(n ** 0.5)), "unique_colours": int(len(np.unique(px))),
               "gpu_us_per_call": round(gpu_us, 1), "gpu_calls": nc}
        prof = pkg.last_wsmall_profile() if hasattr(pkg, "last_wsmall_profile") else {}
        row["path"] = "one launch (dq_wsmall.hip)" if prof else "multi-kernel rounds (dq_weighted.hip)"
        if prof:
            row["kernel_phases_us"] = {k: (round(v, 1) if isinstance(v, float) else v) for k, v in prof.items()}
        if refs is not None:
            r = refs[i]
            out = t_out.cpu().numpy().view(np.uint32)
            row["ref_cpu_us_per_call"] = round(r["us"], 1)
            row["ref_cpu_calls"] = r["calls"]
            row["gpu_over_cpu_speedup"] = round(r["us"] / gpu_us, 2)
            row["verified"] = bool(np.array_equal(last["ct"], r["ct"]) and np.array_equal(out, r["out"]))
        rows.append(row)
        del t_in, t_out
    return rows


def weighted_regions_batch(pkg, torch, dev, stream, k, side, image="batman", reps=5, cpu=True):
    """The same call for EVERY side x side tile of the sample image at once
    (dq_hip_quant_weighted_regions_dev: one launch, one workgroup per
    region), beside the reference build running the tiles one after another
    (the app's loop); every tile's output checked against the reference's."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import dq_fixtures as fx
    img, w, h = fx.load_png_u32(os.path.join(GOLDEN, "png", image + ".png"))
    img = img.reshape(h, w)
    regions = [np.ascontiguousarray(img[y:y + side, x:x + side]).reshape(-1)
               for y in range(0, h - side + 1, side) for x in range(0, w - side + 1, side)]
    ts = [torch.from_numpy(p.view(np.int32)).to(dev) for p in regions]
    outs = [torch.empty_like(t) for t in ts]
    wr = pkg.WeightedRegions(ts, outs, k)   # (argument arrays built once: the library call is timed)
    last = {}

    def one():
        wr.run(max_iters=10, stream=stream)
        last["cts"] = [wr.colortable(i) for i in range(wr.nr)]
    for _ in range(2):
        one()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        wr.run(max_iters=10, stream=stream)
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / reps
    one()
    row = {"side": side, "regions": len(regions), "pixels": int(sum(p.size for p in regions)),
           "gpu_ms_per_call": round(dt * 1e3, 3), "gpu_us_per_region": round(dt * 1e6 / len(regions), 2)}
    if cpu:
        ref_so = os.path.join(ROOT, "oracle", "_ref", "libdqref.so")
        if os.path.exists(ref_so):
            lib = ctypes.CDLL(ref_so)
            ok, t = True, 0.0
            with _Quiet():
                for i, px in enumerate(regions):
                    out = np.zeros(px.size, np.uint32)
                    ct = np.zeros(k, np.uint32)
                    kk = ctypes.c_uint32(k)
                    t0 = time.perf_counter()
                    lib.quant_recurse(ctypes.c_uint32(px.size), fx.vp(px), fx.vp(out), ctypes.byref(kk), fx.vp(ct),
                                      ctypes.c_int(0))
                    t += time.perf_counter() - t0
                    ok = ok and np.array_equal(last["cts"][i], ct[:kk.value]) and \
                        np.array_equal(outs[i].cpu().numpy().view(np.uint32), out)
            row["ref_cpu_ms_all_regions"] = round(t * 1e3, 2)
            row["ref_cpu_us_per_region"] = round(t * 1e6 / len(regions), 2)
            row["gpu_over_cpu_speedup"] = round(t / dt, 2)
            row["verified"] = bool(ok)
    del ts, outs
    return row


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


def frame_id(rank, i, nf):
    """Weak scaling: rank r owns frames [r*nf, (r+1)*nf) of the global batch
    (at N=8, nf=8: C4's 64 frames, each rank a distinct eighth)."""
    return rank * nf + i


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


def all_ranks_ok(ok, world, device):
    import torch
    import torch.distributed as dist
    if world == 1:
        return ok
    t = torch.tensor([0 if ok else 1], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item()) == 0


# ---------------------------------------------------------------------------
# Golden-fixture checks (the reference build's outputs, tests/golden/).
_fix_cache = {}


def fixture(name):
    if name not in _fix_cache:
        path = os.path.join(GOLDEN, name)
        _fix_cache[name] = json.load(open(path)) if os.path.exists(path) else {}
    return _fix_cache[name]


def frame_fixture(w, h, k, f):
    """The reference's (out_fnv, ct, band_fnv) of synthetic frame f, or None."""
    if (w, h, k) == (3840, 2160, 256):
        return fixture("c4.json").get("f%02d" % f)
    if f == 0:
        return fixture("big.json").get("%dx%d_k%d" % (w, h, k))
    return None


MISMATCH = []   # details of failed frame checks (reported with the error line)


def check_frame(pkg, out_t, ct, fix, rows=None, h=None, world=1, rank=0):
    """Compare one frame's output (whole frame, or this rank's row band) and
    colortable with the fixture.  Returns True / False / None (no fixture)."""
    if fix is None:
        return None
    if [int(v) for v in ct] != fix["ct"]:
        got = [int(v) for v in ct]
        MISMATCH.append({"what": "ct", "k_out": len(got), "k_ref": len(fix["ct"]),
                         "first_diff": next((i for i, (x, y) in enumerate(zip(got, fix["ct"])) if x != y), None)})
        return False
    out = out_t.cpu().numpy().view(np.uint32)
    if rows is None or world == 1:
        ok = "%016x" % pkg.fnv1a64(out) == fix["out_fnv"]
        if not ok:
            MISMATCH.append({"what": "out"})
        return ok
    bands = fix.get("band_fnv")
    if not bands or 8 % world != 0:
        return None
    per = 8 // world   # this rank's rows = bands [rank*per, (rank+1)*per)
    bh = h // 8
    w = out.size // (rows[1] - rows[0])
    for j in range(per):
        b = rank * per + j
        lo = (b * bh - rows[0]) * w
        if "%016x" % pkg.fnv1a64(out[lo:lo + bh * w]) != bands[b]:
            MISMATCH.append({"what": "band", "band": b})
            return False
    return True


def fail(msg, rank, **kw):
    print(json.dumps(dict({"error": msg, "rank": rank, "mismatch": MISMATCH}, **kw)), flush=True)
    sys.exit(3)


def pick_roofline(stats, pmc_key):
    """The roofline object of the kernel kind with the largest measured time."""
    cand = {k: v for k, v in stats.items() if k in ROOF_KERNELS and v[0] > 0 and v[1] > 0 and v[2] > 0}
    if not cand:
        return None
    kind = max(cand, key=lambda k: cand[k][1])
    launches, ms, alg, units = cand[kind]
    sym, b_eng, b_survey = ROOF_KERNELS[kind]
    gbs = alg / (ms / 1e3) / 1e9
    gbs_survey = b_survey * units / (ms / 1e3) / 1e9
    roof = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None,
            "kernel": sym, "launches": launches,
            "avg_launch_us": round(ms * 1e3 / launches, 2),
            "alg_bytes_per_launch": round(alg / launches),
            "points_per_launch": round(units / launches),
            "alg_model": "engine work model (DESIGN.md 5): %s" % b_eng,
            "frac_survey_model": round(gbs_survey / HBM_PEAK_GBS, 4),
            "survey_model": "SURVEY 8(d): %d B per point (a partition's write is overhead)" % b_survey,
            "share_of_step_kernel_time": round(ms / sum(v[1] for v in stats.values() if v[1] > 0), 3),
            "measured": "HIP events around every launch on the engine's stream, one engine lane "
                        "(kernels not overlapped), same workload as the timed region"}
    if os.path.exists(PMC_FILE):
        try:
            pmc = json.load(open(PMC_FILE)).get(pmc_key, {}).get(sym)
        except ValueError:
            pmc = None
        if pmc:
            roof["traffic"] = round(pmc["hbm_bytes_per_launch"])
            roof["traffic_source"] = pmc["source"]
    return roof


def copy_rate_gbs(torch, dev, mib=1024, reps=10):
    """Context for the roofline: the device-to-device copy rate of a buffer
    four times the 256-MB Infinity Cache (bytes read + written per second)
    -- the practical ceiling of a kernel that reads and writes its bytes
    once, measured live on this box."""
    a = torch.empty(mib << 18, dtype=torch.int32, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    del a, b
    return 2.0 * (mib << 20) / (ms / 1e3) / 1e9


def upload_frames(torch, pkg, dev, w, h, ids, rows=None):
    """Synthetic frames `ids` on the device (whole, or rows [r0, r1) of each)."""
    ts = []
    for f in ids:
        px = pkg.synth_frame(w * h, f)
        if rows is not None:
            px = px[rows[0] * w:rows[1] * w]
        ts.append(torch.from_numpy(px.view(np.int32)).to(dev))
    return ts


def rows_leg(ctx, cfg, nf, steps, warmup, verify):
    """nf frames of config `cfg`, each row-sharded over the ranks (one RCCL
    allreduce of all frames' node totals per pass); returns (dt, verified,
    comm ranks).  The communicator exists only inside the leg."""
    torch, pkg, dev, local, rank, world, stream = (ctx[k] for k in
                                                   ("torch", "pkg", "dev", "local", "rank", "world", "stream"))
    w, h, k = CONFIGS[cfg]
    n = w * h
    if world > 1:
        pkg.comm_init_torch(device=local)
    comm = pkg.comm_size(device=local)
    r0, r1 = row_range(h, rank, world)
    fr = upload_frames(torch, pkg, dev, w, h, range(nf), rows=(r0, r1))
    out = [torch.empty_like(f) for f in fr]
    last = {}

    def step():
        last["cts"], _ = pkg.quant_rows_device(fr, out, k, widths=[w] * nf, n_globals=[n] * nf, nshard=1,
                                               max_iters=10, device=local, stream=stream)
    for _ in range(warmup):
        step()
    dt = max_over_ranks(timed_region(step, steps, world, ctx["sync"]), world, dev)
    ok = None
    if verify:
        ctx["sync"]()
        rr = [check_frame(pkg, out[i], last["cts"][i], frame_fixture(w, h, k, i), rows=(r0, r1), h=h,
                          world=world, rank=rank) for i in range(nf)]
        checked = [r for r in rr if r is not None]
        ok = all_ranks_ok(all(checked), world, dev) if checked else None
        if ok is False:
            fail("%s row-tile outputs differ from the reference fixtures" % cfg.upper(), rank,
                 per_frame=rr)
    if world > 1:
        pkg.comm_destroy(device=local)
    del fr, out
    torch.cuda.empty_cache()
    return dt, ok, comm


def frame_leg(ctx, cfg, steps, verify, uniq=1):
    """One frame of config `cfg` per call (this rank's frame 0 of the config:
    the fixture's frame at N=1); returns (dt, verified).  uniq=0: the weighted
    path (allPixelsUnique=0, calc_color_table + ordered FP64 folds), checked
    against the same uniform-weight fixture (the two paths' outputs
    are identical on 4K noise, from the reference build itself)."""
    torch, pkg, dev, local, rank, world, stream = (ctx[k] for k in
                                                   ("torch", "pkg", "dev", "local", "rank", "world", "stream"))
    w, h, k = CONFIGS[cfg]
    # C3: this rank's first frame (C4's fixtures hold all 64); C2: frame 0 on
    # every rank (replicas: the one frame with a fixture)
    fid = frame_id(rank, 0, ctx["nf"]) if cfg == "c3" else 0
    t_in = upload_frames(torch, pkg, dev, w, h, [fid])[0]
    t_out = torch.empty_like(t_in)
    last = {}

    def one():
        last["ct"], _ = pkg.quant_device(t_in, t_out, k, max_iters=10, device=local, stream=stream,
                                         all_pixels_unique=uniq)
    for _ in range(3):
        one()
    dt = max_over_ranks(timed_region(one, steps, world, ctx["sync"]), world, dev)
    ok = None
    if verify:
        ctx["sync"]()
        r = check_frame(pkg, t_out, last["ct"], frame_fixture(w, h, k, fid))
        ok = all_ranks_ok(r is not False, world, dev)
        if r is None and world == 1:
            ok = None
        if ok is False:
            fail("%s output differs from the reference fixture" % cfg.upper(), rank)
    return dt, ok


def dry_run(a, rank, world):
    """--dry-run: the launcher and the timing harness without GPU work."""
    if world != a.gpus:
        raise SystemExit("bench: --gpus %d but the launcher started %d rank(s)" % (a.gpus, world))
    dt = max_over_ranks(timed_region(lambda: time.sleep(0.01 * (rank + 1)), a.steps, world, lambda: None), world)
    if rank == 0:
        print(json.dumps({"metric": "dry run", "value": 0.0, "n_gpus": world, "steps": a.steps,
                          "ms_per_step": round(dt * 1e3 / a.steps, 3), "dry_run": True}), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    rank, world, local = init_dist()
    if world != a.gpus:
        raise SystemExit("bench: --gpus %d but %d rank(s) in the torchrun environment" % (a.gpus, world))
    if a.dry_run:
        dry_run(a, rank, world)
        return
    import torch
    from __graft_entry__ import load_package

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pkg = load_package()
    stream = torch.cuda.current_stream(dev)
    sync = lambda: torch.cuda.synchronize(dev)  # noqa: E731
    ctx = {"torch": torch, "pkg": pkg, "dev": dev, "local": local, "rank": rank, "world": world,
           "stream": stream, "sync": sync, "nf": a.frames}
    verify = not a.no_verify

    w, h, k = CONFIGS[a.config]
    n = w * h
    nf = a.frames
    comm_ranks = None
    if a.mode == "frames":
        ids = [frame_id(rank, i, nf) for i in range(nf)]
        frames = upload_frames(torch, pkg, dev, w, h, ids)
        outs = [torch.empty_like(f) for f in frames]
        last = {}

        def step():   # one batched call: every pass of a round covers all frames
            if nf == 1:
                ct, _ = pkg.quant_device(frames[0], outs[0], k, max_iters=10, device=local, stream=stream)
                last["cts"] = [ct]
            else:
                last["cts"], _ = pkg.quant_batch_device(frames, outs, k, max_iters=10, device=local,
                                                        stream=stream)
        px_per_step = n * nf * world
        workload = ("C4 per-GPU share: %d x %dx%d frames per rank per step, K=%d, quant_recurse "
                    "max_iters=10 (cluster + dedup + map), one batched call" % (nf, w, h, k)
                    if nf > 1 else "one %dx%d frame per step, K=%d, quant_recurse" % (w, h, k))
        parallelism = "frames-per-rank x%d" % world
        scaling = "weak"
    else:
        if world > 1:
            pkg.comm_init_torch(device=local)
        comm_ranks = pkg.comm_size(device=local)
        r0, r1 = row_range(h, rank, world)
        frames = upload_frames(torch, pkg, dev, w, h, range(nf), rows=(r0, r1))
        outs = [torch.empty_like(f) for f in frames]
        last = {}

        def step():
            last["cts"], _ = pkg.quant_rows_device(frames, outs, k, widths=[w] * nf, n_globals=[n] * nf,
                                                   nshard=1, max_iters=10, device=local, stream=stream)
        px_per_step = n * nf
        workload = ("%s: %d x %dx%d frame(s), K=%d, row-tile sharded over %d rank(s), one RCCL "
                    "allreduce of all frames' node totals per pass" % (a.config.upper(), nf, w, h, k, world))
        parallelism = "row-tiles x%d" % world
        scaling = "strong"

    pkg.set_lanes(a.lanes)
    lanes = pkg.get_lanes()
    for _ in range(a.warmup):
        step()
    # --- timed region: no per-launch events (they would perturb the timing)
    pkg.set_timing(False, device=local)
    dt = timed_region(step, a.steps, world, sync)
    # --- correctness of the timed work: the last step's outputs vs the reference
    verified = None
    if verify:
        sync()
        res = []
        for i in range(nf):
            if a.mode == "frames":
                res.append(check_frame(pkg, outs[i], last["cts"][i], frame_fixture(w, h, k, ids[i])))
            else:
                res.append(check_frame(pkg, outs[i], last["cts"][i], frame_fixture(w, h, k, i), rows=(r0, r1),
                                       h=h, world=world, rank=rank))
        checked = [r for r in res if r is not None]
        ok = all_ranks_ok(all(checked), world, dev)
        verified = {"ok": ok, "frames_checked_rank0": len(checked), "frames_rank0": nf,
                    "against": "reference build outputs (tests/golden/%s): colortable + out FNV-1a-64%s"
                               % ("c4.json" if (w, h, k) == (3840, 2160, 256) else "big.json",
                                  " of this rank's row bands" if a.mode == "rows" and world > 1 else "")}
        if not ok:
            fail("bench outputs differ from the reference fixtures", rank, verified=verified, per_frame=res)
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
        sync()
        pkg.set_timing(False, device=local)
        stats = pkg.get_stats(device=local)
        pkg.set_lanes(a.lanes)
    rounds = pkg.last_rounds(device=local)
    swept = pkg.last_points_swept(device=local)
    full = pkg.last_points_full(device=local)
    dt = max_over_ranks(dt, world, dev)
    value = px_per_step * a.steps / dt / 1e6

    detail = {}
    big4k = a.mode == "frames" and (w, h, k) == (3840, 2160, 256)
    # --- C3: one 4K frame per call (this rank's first frame)
    if big4k and not a.no_c3 and nf > 1:
        dt1, ok1 = frame_leg(ctx, "c3", a.steps, verify)
        detail["c3"] = {"ms_per_frame": round(dt1 * 1e3 / a.steps, 3),
                        "Mpix_per_s": round(n * world * a.steps / dt1 / 1e6, 2),
                        "workload": "one 3840x2160 frame per call (C3), K=256, %d rank(s)" % world,
                        "verified": ok1}
    # --- C2: one 1920x1080 frame per call, K=256
    if a.mode == "frames" and not a.no_c2:
        w2, h2, _ = CONFIGS["c2"]
        dt2, ok2 = frame_leg(ctx, "c2", a.steps, verify)
        detail["c2"] = {"ms_per_frame": round(dt2 * 1e3 / a.steps, 3),
                        "Mpix_per_s": round(w2 * h2 * world * a.steps / dt2 / 1e6, 2),
                        "workload": "one 1920x1080 frame per call (C2), K=256, %d rank(s) (replicas)" % world,
                        "verified": ok2}

    # --- the weighted path (allPixelsUnique=0: every live app call site,
    # ClusteringSegmentation.cpp:1803) on one 4K frame per call
    if big4k and not a.no_weighted:
        sw_ = max(1, min(10, a.steps))
        dtw, okw = frame_leg(ctx, "c3", sw_, verify, uniq=0)
        detail["weighted_c3"] = {"ms_per_frame": round(dtw * 1e3 / sw_, 3),
                                 "Mpix_per_s": round(n * world * sw_ / dtw / 1e6, 2), "steps": sw_,
                                 "workload": "one 3840x2160 frame per call, K=256, quant_recurse(allPixelsUnique=0): "
                                             "GPU calc_color_table (hand-written: bucket-group runs + LDS tables) + exact ordered FP64 folds, %d "
                                             "rank(s)" % world,
                                 "verified": okw}
        if okw is False:
            fail("weighted-path output differs from the reference fixture", rank)
        # the app's own call size: quant_recurse(N_region, .., K=4,
        # allPixelsUnique=0) per superpixel region (ClusteringSegmentation.cpp:
        # 1779-1803), square crops of the reference's sample image at 10^3 -
        # 10^6 pixels, one region per call; the reference build on the same
        # crops beside it (rank 0, N=1: the cpu_baseline's kind), the GPU's
        # outputs checked against the reference's
        rows = weighted_regions(pkg, torch, dev, stream, 4, [32, 100, 316, 1000],
                                cpu=(rank == 0 and world == 1 and not a.no_cpu_baseline))
        detail["weighted_regions"] = {
            "workload": "quant_recurse(N, K=4, allPixelsUnique=0) on square crops of tests/golden/png/batman.png, "
                        "one region per call, device-resident pixels; ref_cpu = the reference build "
                        "(oracle/_ref, unmodified DivQuant sources), one core",
            "regions": rows}
        if any(r.get("verified") is False for r in rows):
            fail("weighted-region outputs differ from the reference build's", rank, regions=rows)
        # every tile of the image at once: the app's loop over its regions as
        # one batched call (dq_hip_quant_weighted_regions_dev), the reference
        # running the same tiles one by one
        cpu_b = rank == 0 and world == 1 and not a.no_cpu_baseline
        brows = [weighted_regions_batch(pkg, torch, dev, stream, 4, sd, cpu=cpu_b) for sd in (32, 100)]
        detail["weighted_regions_batched"] = {
            "workload": "quant_recurse(N, K=4, allPixelsUnique=0) for every side x side tile of "
                        "tests/golden/png/batman.png in ONE call (one workgroup per region), device-resident "
                        "pixels; ref_cpu = the reference build running the tiles one after another, one core",
            "batches": brows}
        if any(r.get("verified") is False for r in brows):
            fail("batched weighted-region outputs differ from the reference build's", rank, batches=brows)
    # --- the same frames as OpenCV BGR24 Mats: read directly by
    # the root's passes, partition and map (3 B per pixel, no packing pass);
    # one frame per call (C3 shape) and the rank's batch in one call
    if big4k and not a.no_bgr and nf > 1:
        bf = []
        for t in frames:
            p = t.view(torch.int32)
            bf.append(torch.stack([p & 0xFF, (p >> 8) & 0xFF, (p >> 16) & 0xFF], -1).to(torch.uint8).reshape(-1))
        lastb = {}

        def bone():
            lastb["ct"], _ = pkg.quant_bgr24_device(bf[0], w, h, outs[0], k, device=local, stream=stream)

        def bbatch():
            lastb["cts"], _ = pkg.quant_bgr24_batch_device(bf, w, h, outs, k, device=local, stream=stream)
        for _ in range(2):
            bone()
        dtb1 = max_over_ranks(timed_region(bone, a.steps, world, sync), world, dev)
        okb1 = None
        if verify:
            sync()
            okb1 = all_ranks_ok(check_frame(pkg, outs[0], lastb["ct"], frame_fixture(w, h, k, ids[0])) is not False,
                                world, dev)
        for _ in range(2):
            bbatch()
        dtb = max_over_ranks(timed_region(bbatch, a.steps, world, sync), world, dev)
        okb = None
        if verify:
            sync()
            okb = all_ranks_ok(all(check_frame(pkg, outs[i], lastb["cts"][i], frame_fixture(w, h, k, ids[i]))
                                   is not False for i in range(nf)), world, dev)
        if okb1 is False or okb is False:
            fail("BGR24-input outputs differ from the reference fixtures", rank)
        detail["bgr24_input"] = {
            "c3_ms_per_frame": round(dtb1 * 1e3 / a.steps, 3),
            "c3_Mpix_per_s": round(n * world * a.steps / dtb1 / 1e6, 2),
            "batch_ms_per_step": round(dtb * 1e3 / a.steps, 3),
            "batch_Mpix_per_s": round(n * nf * world * a.steps / dtb / 1e6, 2),
            "workload": "the same frames as BGR24 (CV_8UC3) device buffers: one frame per call, and %d frames "
                        "per rank in one batched call (dq_hip_quant_bgr24[_batch]_dev)" % nf,
            "verified": None if okb is None else bool(okb1 and okb)}
        del bf

    if a.mode == "frames":
        del frames, outs
        torch.cuda.empty_cache()
    # --- C5: the gigapixel tile, rows over the ranks (N=1: whole on one GPU)
    if a.mode == "frames" and not a.no_c5:
        w5, h5, k5 = CONFIGS["c5"]
        s5 = max(1, min(5, a.steps))
        dt5, ok5, comm5 = rows_leg(ctx, "c5", 1, s5, 2, verify)
        comm_ranks = comm5
        detail["c5"] = {"ms_per_tile": round(dt5 * 1e3 / s5, 3),
                        "Mpix_per_s": round(w5 * h5 * s5 / dt5 / 1e6, 2), "steps": s5,
                        "workload": "C5: one 16384x16384 tile, K=1024, rows split over %d rank(s), one RCCL "
                                    "allreduce of the node totals per pass" % world,
                        "scaling": "strong", "verified": ok5}
    # --- C4 row-tile variant: all 64 frames, each row-sharded over the ranks
    if big4k and not a.no_rowtile:
        rsteps = max(1, min(3, a.steps))
        dtr, okr, commr = rows_leg(ctx, "c3", 64, rsteps, 1, verify)
        comm_ranks = commr
        detail["c4_rowtile"] = {
            "ms_per_step": round(dtr * 1e3 / rsteps, 3),
            "Mpix_per_s": round(n * 64 * rsteps / dtr / 1e6, 2), "steps": rsteps,
            "workload": "C4 row-tile variant: 64 x %dx%d frames, K=%d, each frame's rows split over "
                        "%d rank(s), one RCCL allreduce of all frames' node totals per pass" % (w, h, k, world),
            "scaling": "strong", "verified": okr}

    if rank == 0:
        pmc_key = "%s_%s_f%d_n%d" % (a.mode, a.config, nf, world)
        roof = pick_roofline(stats, pmc_key) if stats else None
        if roof:
            cgbs = copy_rate_gbs(torch, dev)
            roof["copy_GBps_measured"] = round(cgbs, 1)
            roof["frac_of_copy"] = round(roof["achieved"] / cgbs, 4)
            roof["copy_note"] = ("a 1-GiB device-to-device copy (read + write) timed on this box: the "
                                 "practical ceiling of a read+write kernel; frac stays against the nominal peak")
        # engine-model bytes of all kernels of the roofline region, per step,
        # over the timed step's wall time (<= 1: they are bytes the kernels move)
        eng_bytes = sum(v[2] for v in stats.values()) / max(1, a.steps)
        detail.update({
            "ms_per_frame": round(dt * 1e3 / a.steps / (nf * world if a.mode == "frames" else nf), 3),
            "pipeline_engine_GBps_per_gpu": round(eng_bytes / (dt / a.steps) / 1e9, 1) if stats else None,
            "pipeline_engine_frac_per_gpu": round(eng_bytes / (dt / a.steps) / 1e9 / HBM_PEAK_GBS, 4)
            if stats else None,
            "rounds_last_frame": rounds, "points_swept_last_call": swept,
            "points_full_iterations_last_call": full,
            "rccl_comm_ranks": comm_ranks,
            "kernels": {kname: {"launches": v[0], "ms": round(v[1], 3),
                                "GBps": round(v[2] / (v[1] / 1e3) / 1e9, 1) if v[1] > 0 and v[2] > 0 else None}
                        for kname, v in stats.items() if v[0]}})
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
            "dtype": "u8 RGB (packed u32 frames, planar u8 working buffers), u32/u64 integer sums, f64 updates",
            "data": "synthetic uniform-random 24-bit RGB frames (SURVEY 8c xorshift64, frame f = seed + f)",
            "config": {"workload": workload, "frames_per_rank_per_step": nf if a.mode == "frames" else None,
                       "frames_per_step": nf if a.mode == "rows" else None,
                       "engine_lanes": lanes if a.mode == "frames" else 1,
                       "gpu_max_hw_queues": int(os.environ["GPU_MAX_HW_QUEUES"]),
                       "gpu_max_hw_queues_set_by_bench": _HWQ_CALLER != os.environ["GPU_MAX_HW_QUEUES"],
                       "width": w, "height": h, "k": k, "max_iters": 10, "parallelism": parallelism},
            "verified": verified,
            "roofline": roof,
            "detail": detail,
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
