"""GPU parity of the cross-process row-tile path with N > 1 ranks.

The multi-process path (DivQuantCluster.cpp:438-559 split-pass sums and
:613-811 2-means sums of each rank's rows, one allreduce of the integer node
totals per pass, every rank running the same FP64 update) is exercised here
with N engines of ONE process on one GPU, each with its own stream and host
thread, joined by an in-process loopback collective in place of RCCL
(dq_hip_loopback_rows_dev).  This runs the TOT_ALLREDUCE code that exists only
for N > 1 -- kpass writing this rank's node totals, the epilogue's FP64
update on the global totals while cursors and record sizes come from the
local counts, the per-rank plan mirror -- with local != global, as the 8-GPU
node will.  The bar is the unsharded one: every rank's colortable equal to the
reference's, the frame assembled from every rank's rows bit-exact, the split
trace and centroid doubles exact, and every rank enqueueing the identical
collective sequence (count and sizes).
"""
import ctypes

import numpy as np
import pytest

import dq_fixtures as fx

pytestmark = pytest.mark.gpu

W4, H4 = 3840, 2160


def _oracle(px, k, max_iters=10):
    orc = fx.oracle()
    n = len(px)
    out = np.zeros(n, np.uint32)
    ct = np.zeros(k, np.uint32)
    kk = ctypes.c_uint32(k)
    orc.dqo_quant_recurse(ctypes.c_uint32(n), fx.vp(px), fx.vp(out), ctypes.byref(kk), fx.vp(ct))
    means = np.zeros((k, 3), np.float64)
    sizes = np.zeros(k, np.int64)
    trace = np.zeros((max(k - 1, 1), 4), np.int64)
    ct2 = np.zeros(k, np.uint32)
    kk2 = ctypes.c_uint32(k)
    orc.dqo_cluster(ctypes.c_uint32(n), fx.vp(px), ctypes.byref(kk2), fx.vp(ct2),
                    ctypes.c_int(max_iters), fx.vp(means), fx.vp(sizes), fx.vp(trace))
    return out, ct[:kk.value], means, sizes, trace[:k - 1]


def _run(gpu, frames, w, h, k, nranks):
    """frames: host uint32 arrays (w*h) -> (outs, cts per rank, logs)."""
    import torch
    t_in = [torch.from_numpy(np.ascontiguousarray(p, np.uint32).view(np.int32)).to("cuda:0") for p in frames]
    t_out = [torch.full_like(t, -1) for t in t_in]
    cts, logs, _ = gpu.loopback_rows_device(t_in, t_out, w, h, k, nranks)
    torch.cuda.synchronize()
    return [t.cpu().numpy().view(np.uint32) for t in t_out], cts, logs


def _check_collectives(logs, nranks):
    assert len(logs) == nranks
    assert len(logs[0]) > 0, "no collective ran: the TOT_ALLREDUCE path was not taken"
    for r in range(1, nranks):
        assert logs[r] == logs[0], "rank %d enqueued a different collective sequence" % r
    assert all(c % 8 == 0 and c > 0 for c in logs[0])   # 8 u64 per logical node


def _check_vs_oracle(gpu, px, k, out, cts_frame, nranks):
    r_out, r_ct, r_means, r_sizes, r_trace = _oracle(px, k)
    for r in range(nranks):
        assert np.array_equal(cts_frame[r], r_ct), "rank %d colortable" % r
    assert np.array_equal(out, r_out)
    if k > 1:   # rank 0's diagnostics (identical on every rank: same totals, same FP64)
        assert np.array_equal(gpu.last_trace(k), r_trace)
        means, sizes = gpu.last_centroids(k)
        filled = r_sizes > 0
        assert np.array_equal(sizes, r_sizes)
        assert np.array_equal(means[filled].view(np.uint64), r_means[filled].view(np.uint64))


@pytest.mark.parametrize("nranks", [2, 3, 4, 8])
def test_loopback_uniform(gpu, nranks):
    w, h, k = 640, 480, 256
    px = fx.xorshift(w * h, seed=1700 + nranks)
    (out,), cts, logs = _run(gpu, [px], w, h, k, nranks)
    _check_collectives(logs, nranks)
    _check_vs_oracle(gpu, px, k, out, [c[0] for c in cts], nranks)


@pytest.mark.parametrize("name,k", [("batman", 16), ("cookie", 125), ("batman", 256)])
def test_loopback_images(gpu, name, k):
    """Structured images: a rank may hold no point of a cluster at all (its
    local count 0 while the global total is not)."""
    px, w, h = fx.load_png_u32(fx.os.path.join(fx.GOLDEN, "png", name + ".png"))
    for nranks in (2, 5, 8):
        (out,), cts, logs = _run(gpu, [px], w, h, k, nranks)
        _check_collectives(logs, nranks)
        _check_vs_oracle(gpu, px, k, out, [c[0] for c in cts], nranks)


def test_loopback_ragged_and_tiny(gpu):
    """Heights not divisible by N, ranks of one row, K > n (empty clusters),
    grey / tie-heavy frames."""
    rng = np.random.default_rng(77)
    cases = [(fx.xorshift(37 * 29, seed=5), 37, 29, 64),
             (fx.xorshift(101 * 9, seed=6), 101, 9, 32),
             ((rng.integers(0, 6, 333 * 151, dtype=np.uint32) * 0x2A2A2A), 333, 151, 32),
             (rng.integers(0, 256, 200 * 100, dtype=np.uint32) * 0x010101, 200, 100, 16),
             (fx.xorshift(64 * 8, seed=7), 64, 8, 1024)]
    for px, w, h, k in cases:
        for nranks in (2, 7, 8):
            if h < nranks:
                continue
            (out,), cts, logs = _run(gpu, [px], w, h, k, nranks)
            _check_collectives(logs, nranks)
            _check_vs_oracle(gpu, px, k, out, [c[0] for c in cts], nranks)


def test_loopback_batch(gpu):
    """Several frames per call (C4's row-tile variant shape): every pass's
    allreduce carries all frames' node totals."""
    w, h, k = 320, 200, 64
    frames = [fx.xorshift(w * h, seed=1800 + i) for i in range(3)]
    frames[1] &= 0xF0F0F0
    outs, cts, logs = _run(gpu, frames, w, h, k, 4)
    _check_collectives(logs, 4)
    for i, (px, out) in enumerate(zip(frames, outs)):
        r_out, r_ct = _oracle(px, k)[:2]
        assert np.array_equal(out, r_out), i
        for r in range(4):
            assert np.array_equal(cts[r][i], r_ct), (i, r)


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_loopback_c4_frames(gpu, nranks):
    """C4 frames 0-7 (the row-tile variant's per-GPU share at 8 GPUs) row-
    sharded over N ranks, against the reference build's per-frame hashes and
    the 8 row-band hashes each of 8 ranks would hold."""
    import torch
    fix = fx.load_json("c4.json")
    ids = list(range(8))
    t_in = [torch.from_numpy(fx.xorshift(W4 * H4, seed=fx.SEED + f).view(np.int32)).to("cuda:0") for f in ids]
    t_out = [torch.full_like(t, -1) for t in t_in]
    cts, logs, _ = gpu.loopback_rows_device(t_in, t_out, W4, H4, 256, nranks)
    torch.cuda.synchronize()
    _check_collectives(logs, nranks)
    for i, f in enumerate(ids):
        c = fix["f%02d" % f]
        for r in range(nranks):
            assert [int(v) for v in cts[r][i]] == c["ct"], (f, r)
        out = t_out[i].cpu().numpy().view(np.uint32)
        for b in range(8):
            band = out[b * 270 * W4:(b + 1) * 270 * W4]
            assert "%016x" % fx.fnv(band) == c["band_fnv"][b], (f, b)
        assert "%016x" % fx.fnv(out) == c["out_fnv"], f


def test_loopback_c5_8_ranks(gpu):
    """C5 (16384^2, K=1024) row-sharded over 8 ranks: the 8-GPU run's exact
    collective path, against the reference build's row-band hashes."""
    import torch
    big = fx.load_json("big.json")
    key = "16384x16384_k1024"
    if key not in big:
        pytest.skip("C5 fixture not generated")
    c = big[key]
    arrs = fx.load_npz("big.npz")
    t = torch.from_numpy(fx.xorshift(16384 * 16384).view(np.int32)).to("cuda:0")
    o = torch.full_like(t, -1)
    cts, logs, _ = gpu.loopback_rows_device([t], [o], 16384, 16384, 1024, 8)
    torch.cuda.synchronize()
    _check_collectives(logs, 8)
    for r in range(8):
        assert [int(v) for v in cts[r][0]] == c["ct"], r
    out = o.cpu().numpy().view(np.uint32)
    del t, o
    for b in range(8):
        assert "%016x" % fx.fnv(out[b * 2048 * 16384:(b + 1) * 2048 * 16384]) == c["band_fnv"][b], b
    assert "%016x" % fx.fnv(out) == c["out_fnv"]
    assert np.array_equal(gpu.last_trace(1024), arrs["trace_" + key])
    means, sizes = gpu.last_centroids(1024)
    ref_means = arrs["means_" + key]
    filled = ~np.isnan(ref_means[:, 0])
    assert np.array_equal(filled, sizes > 0)
    assert np.array_equal(means[filled].view(np.uint64), ref_means[filled].view(np.uint64))


def test_arena_zero_after_sharded_runs(gpu):
    """The planned rounds' invariant (the round arena is all zero when a run
    starts, restored only by the end-of-run clear) checked at the entry of
    every run (kDebugArenaCheck) over the order that aborted in round 3:
    virtual-shard runs, then an unsharded batch over the default lanes."""
    import torch
    w, h, k = 640, 480, 256
    try:
        gpu.set_debug(16)
        for nshard in (2, 8, 3):
            px = fx.xorshift(w * h, seed=900 + nshard)
            t = torch.from_numpy(px.view(np.int32)).to("cuda:0")
            o = torch.empty_like(t)
            (ct,), _ = gpu.quant_rows_device([t], [o], k, widths=[w], nshard=nshard)
            torch.cuda.synchronize()
            r_out, r_ct = _oracle(px, k)[:2]
            assert np.array_equal(ct, r_ct) and np.array_equal(o.cpu().numpy().view(np.uint32), r_out)
        fix = fx.load_json("c4.json")
        t_in = [torch.from_numpy(fx.xorshift(W4 * H4, seed=fx.SEED + f).view(np.int32)).to("cuda:0")
                for f in range(4)]
        t_out = [torch.empty_like(t) for t in t_in]
        for _ in range(2):
            cts, _ = gpu.quant_batch_device(t_in, t_out, 256)
            torch.cuda.synchronize()
            for f in range(4):
                assert [int(v) for v in cts[f]] == fix["f%02d" % f]["ct"], f
                assert "%016x" % fx.fnv(t_out[f].cpu().numpy().view(np.uint32)) == fix["f%02d" % f]["out_fnv"]
    finally:
        gpu.set_debug(0)


def test_fresh_arena_chunks_under_concurrent_lanes(gpu):
    """Regression for the round-4 abort (DESIGN.md 3c''): a new arena chunk
    was cleared by a null-stream hipMemset that nothing ordered before the
    round's kernels.  With kDebugFreshArena every run of every lane
    allocates (and clears) new chunks while the other lanes run, each call
    entered with the caller's stream busy; 4-frame batches over the default
    lanes, checked against the reference's hashes.  (The buggy build did not
    fail this test on three tries: the race needs the clear to queue behind
    other work -- a guard, not a deterministic reproducer.)"""
    import torch
    fix = fx.load_json("c4.json")
    t_in = [torch.from_numpy(fx.xorshift(W4 * H4, seed=fx.SEED + f).view(np.int32)).to("cuda:0")
            for f in range(4)]
    t_out = [torch.empty_like(t) for t in t_in]
    busy = torch.empty(1 << 28, dtype=torch.int32, device="cuda:0")
    try:
        gpu.set_debug(32 | 16)
        for _ in range(3):
            # the caller's (null) stream busy when the call starts: the lanes
            # join it, and so would a null-stream clear
            busy.fill_(7)
            cts, _ = gpu.quant_batch_device(t_in, t_out, 256)
            torch.cuda.synchronize()
            for f in range(4):
                assert [int(v) for v in cts[f]] == fix["f%02d" % f]["ct"], f
                assert "%016x" % fx.fnv(t_out[f].cpu().numpy().view(np.uint32)) == fix["f%02d" % f]["out_fnv"]
    finally:
        gpu.set_debug(0)
