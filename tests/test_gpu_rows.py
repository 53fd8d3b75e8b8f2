"""GPU parity of row-tile sharding (dq_hip_quant_rows_dev).

A frame's rows split into shards: every pass sums each shard's points
separately and the FP64 update runs on the node totals over all shards
(nodesum kernel; across processes an RCCL allreduce of those integer totals).
The bar is the unsharded one: colortable, label map, split trace and the
centroid doubles bit-exact against the reference-pinned oracle, for every
shard count.  Virtual shards (several row ranges on this GPU) exercise the
exact arithmetic of multi-GPU sharding; a 1-rank RCCL communicator exercises
the allreduce path itself (this box has one GPU).
"""
import ctypes

import numpy as np
import pytest

import dq_fixtures as fx

pytestmark = pytest.mark.gpu


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


def _rows(gpu, frames, k, nshard, widths=None, n_globals=None):
    import torch
    t_in = [torch.from_numpy(np.ascontiguousarray(p, np.uint32).view(np.int32)).to("cuda:0") for p in frames]
    t_out = [torch.empty_like(t) for t in t_in]
    cts, _ = gpu.quant_rows_device(t_in, t_out, k, widths=widths, n_globals=n_globals, nshard=nshard)
    torch.cuda.synchronize()
    return [t.cpu().numpy().view(np.uint32) for t in t_out], cts


def _check(gpu, px, k, out, ct):
    r_out, r_ct, r_means, r_sizes, r_trace = _oracle(px, k)
    assert np.array_equal(ct, r_ct)
    assert np.array_equal(out, r_out)
    if k > 1:
        assert np.array_equal(gpu.last_trace(k), r_trace)
        means, sizes = gpu.last_centroids(k)
        filled = r_sizes > 0
        assert np.array_equal(sizes, r_sizes)
        assert np.array_equal(means[filled].view(np.uint64), r_means[filled].view(np.uint64))


@pytest.mark.parametrize("nshard", [2, 3, 8])
def test_virtual_shards_uniform(gpu, nshard):
    w, h, k = 640, 480, 256
    px = fx.xorshift(w * h, seed=700 + nshard)
    (out,), (ct,) = _rows(gpu, [px], k, nshard, widths=[w])
    _check(gpu, px, k, out, ct)


@pytest.mark.parametrize("name,k", [("batman", 16), ("cookie", 125), ("batman", 256)])
def test_virtual_shards_images(gpu, name, k):
    """Structured images: shards see very different colour mixes (a shard may
    hold no point of a cluster at all)."""
    px, w, h = fx.load_png_u32(fx.os.path.join(fx.GOLDEN, "png", name + ".png"))
    for nshard in (2, 5, 8):
        (out,), (ct,) = _rows(gpu, [px], k, nshard, widths=[w])
        _check(gpu, px, k, out, ct)


def test_virtual_shards_ragged_and_tiny(gpu):
    """No width (4-point shard boundaries), n not a multiple of anything,
    shards smaller than one sweep, K > n (empty clusters), grey / tie-heavy."""
    rng = np.random.default_rng(4242)
    cases = [(fx.xorshift(1001, seed=3), 64), (fx.xorshift(37, seed=4), 64),
             ((rng.integers(0, 6, 50003, dtype=np.uint32) * 0x2A2A2A), 32),
             (rng.integers(0, 256, 20000, dtype=np.uint32) * 0x010101, 16)]
    for px, k in cases:
        for nshard in (2, 7):
            (out,), (ct,) = _rows(gpu, [px], k, nshard)
            _check(gpu, px, k, out, ct)


def test_virtual_shards_batch(gpu):
    """Several sharded frames in one call (C4's row-tile variant: every pass
    of a round covers all frames' shards)."""
    frames = [fx.xorshift(320 * 200, seed=800 + i) for i in range(3)]
    frames[1] &= 0xF0F0F0
    outs, cts = _rows(gpu, frames, 64, 4, widths=[320] * 3)
    for px, out, ct in zip(frames, outs, cts):
        r_out, r_ct = _oracle(px, 64)[:2]
        assert np.array_equal(ct, r_ct) and np.array_equal(out, r_out)


def test_rccl_single_rank(gpu):
    """The cross-process path (nodesum -> ncclAllReduce -> epilogue from the
    totals) on a 1-rank RCCL communicator, with and without virtual shards."""
    uid = gpu.comm_unique_id()
    gpu.comm_init(1, 0, uid, device=0)
    try:
        w, h, k = 512, 384, 128
        px = fx.xorshift(w * h, seed=901)
        for nshard in (1, 3):
            (out,), (ct,) = _rows(gpu, [px], k, nshard, widths=[w], n_globals=[w * h])
            _check(gpu, px, k, out, ct)
    finally:
        gpu.comm_destroy(device=0)


def test_rows_n_global_needs_comm(gpu):
    import torch
    t = torch.zeros(4096, dtype=torch.int32, device="cuda:0")
    with pytest.raises(gpu.DivQuantError):
        gpu.quant_rows_device([t], [torch.empty_like(t)], 16, n_globals=[8192])


def test_dq_hip_quant_ngpus(gpu):
    """dq_hip_quant's ngpus (in-process multi-GPU over ncclCommInitAll): the
    result equals the oracle's for every ngpus (clamped to the devices here);
    DQ_HIP_MULTI_1=1 drives the in-process communicator path on one device."""
    import os
    import subprocess
    import sys
    px = fx.xorshift(300001, seed=4321)
    r_out, r_ct = _oracle(px, 128)[:2]
    for ng in (1, 2, 8):
        out, ct = gpu.quant_host(px, 128, 1, ng)
        assert np.array_equal(ct, r_ct) and np.array_equal(out, r_out), ng
    code = ("import sys, numpy as np; sys.path.insert(0, %r); sys.path.insert(0, %r)\n"
            "import dq_fixtures as fx\nfrom __graft_entry__ import load_package\n"
            "p = load_package(); px = fx.xorshift(300001, seed=4321)\n"
            "out, ct = p.quant_host(px, 128, 1, 1)\n"
            "print(fx.fnv(out), ' '.join(str(int(c)) for c in ct))\n") % (fx.TESTS, fx.ROOT)
    env = dict(os.environ, DQ_HIP_MULTI_1="1")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=200)
    assert r.returncode == 0, r.stderr[-2000:]
    h, cts = r.stdout.strip().splitlines()[-1].split(" ", 1)
    assert int(h) == fx.fnv(r_out) and [int(c) for c in cts.split()] == [int(c) for c in r_ct]
