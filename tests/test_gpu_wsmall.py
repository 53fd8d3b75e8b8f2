"""The one-launch weighted path for small inputs (dq_wsmall.hip): the app's
quant_recurse(N_region, .., K=4, allPixelsUnique=0) per superpixel region
(ClusteringSegmentation.cpp:1779-1803).  Besides the fixtures it shares
with the multi-kernel path (test_gpu_parity.py, `wpath`), these cases aim
at what is particular to it: the exact integer runs of its sequential folds
around rounding ties (power-of-two pixel counts make weights with few
significant bits), its size limits and the fall-back above them, the
in-kernel map up to 16 colours and the host map above."""
import ctypes

import numpy as np
import pytest

import dq_fixtures as fx

pytestmark = pytest.mark.gpu


def _oracle(px, k):
    n = len(px)
    out = np.zeros(n, np.uint32)
    ct = np.zeros(k, np.uint32)
    kk = ctypes.c_uint32(k)
    fx.oracle().dqo_quant_recurse_weighted(ctypes.c_uint32(n), fx.vp(px), fx.vp(out), ctypes.byref(kk), fx.vp(ct))
    return out, ct[:kk.value]


def _check(gpu, px, k):
    out, ct = gpu.quant_recurse(px, k, 0)
    ref_out, ref_ct = _oracle(px, k)
    assert np.array_equal(ct, ref_ct), (len(px), k, ct, ref_ct)
    assert np.array_equal(out, ref_out), (len(px), k)


@pytest.mark.parametrize("n", [1, 2, 3, 64, 1024, 4096, 65536, 131071])
def test_small_sizes_and_ties(gpu, n):
    """Power-of-two pixel counts (norm = 2^-j: weights and summands with few
    significant bits, so the runs meet exact rounding ties) and odd ones,
    few and many colours, K from 1 to 64, against the oracle's sequential
    folds; each call took the one-launch path (one 'round')."""
    rng = np.random.default_rng(n)
    for trial, (ncol, k) in enumerate([(1, 4), (3, 4), (17, 4), (300, 16), (2000, 64), (40, 2), (5, 7)]):
        if ncol > n and trial > 1:
            continue
        pal = rng.integers(0, 1 << 24, ncol, dtype=np.uint32)
        if trial % 2:
            pal &= 0xF0F0F0
        px = pal[rng.integers(0, ncol, n)]
        _check(gpu, px, k)
        if k >= 3 and len(np.unique(px)) >= 3:
            assert gpu.last_rounds() == 1, (n, k)


def test_small_region_crops(gpu):
    """Square crops of the reference's sample images (the app's regions) at
    10^3 - 10^5 pixels, K = 4 (the app's) and 16, against the oracle."""
    for name in ("batman", "cookie"):
        img, w, h = fx.load_png_u32(fx.GOLDEN + "/png/%s.png" % name)
        img = img.reshape(h, w)
        for side in (32, 100, 200, 316):
            y0, x0 = (h - side) // 3, (w - side) // 2
            px = np.ascontiguousarray(img[y0:y0 + side, x0:x0 + side]).reshape(-1)
            for k in (4, 16):
                _check(gpu, px, k)


def test_small_limits_fall_back(gpu):
    """More than 6144 colours (the kernel's buffers) or more than 131071
    pixels: the multi-kernel rounds take the call, same outputs."""
    rng = np.random.default_rng(7)
    px = rng.integers(0, 1 << 24, 20000, dtype=np.uint32)   # ~20000 colours
    _check(gpu, px, 4)
    assert gpu.last_rounds() > 1
    px = (rng.integers(0, 1 << 24, 131072, dtype=np.uint32) & 0xE0E0E0)   # 131072 pixels, 512 colours
    _check(gpu, px, 4)
    assert gpu.last_rounds() > 1
    px = rng.integers(0, 1 << 24, 6144, dtype=np.uint32)    # at most 6144 colours: the kernel
    _check(gpu, px, 4)
    assert gpu.last_rounds() == 1


def test_small_device_pointers_and_no_map(gpu):
    """The device-pointer entry on a stream, and quant_varpart_fast's cluster-
    only call (no dedup, no map) against the oracle's colour table + folds."""
    import torch
    rng = np.random.default_rng(11)
    pal = rng.integers(0, 1 << 24, 900, dtype=np.uint32)
    px = pal[rng.integers(0, 900, 30000)]
    t = torch.from_numpy(px.view(np.int32)).to("cuda:0")
    o = torch.empty_like(t)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        ct, _ = gpu.quant_device(t, o, 4, all_pixels_unique=0, stream=s)
    s.synchronize()
    ref_out, ref_ct = _oracle(px, 4)
    assert np.array_equal(ct, ref_ct)
    assert np.array_equal(o.cpu().numpy().view(np.uint32), ref_out)
    ct = gpu.quant_varpart_fast(px, 8, all_pixels_unique=0)
    col = np.zeros(len(px), np.uint32)
    w = np.zeros(len(px), np.float64)
    u = fx.oracle().dqo_color_table(ctypes.c_uint32(len(px)), fx.vp(px), fx.vp(col), fx.vp(w))
    rct = np.zeros(8, np.uint32)
    kk = ctypes.c_uint32(8)
    fx.oracle().dqo_cluster_weighted(ctypes.c_uint32(u), fx.vp(col), fx.vp(w), ctypes.byref(kk), fx.vp(rct),
                                     ctypes.c_int(10), None, None, None)
    assert np.array_equal(ct, rct[:kk.value])


def test_regions_batch_equals_single_calls(gpu):
    """The app's per-region calls batched (dq_hip_quant_weighted_regions_dev):
    one launch for every region the kernel holds -- crops of the sample
    images from 1 to ~10^5 pixels at K 1-64 -- plus regions it does not
    (more than 6144 colours, more than 131071 pixels, K above 64) taken one
    by one; every region equals its own single call, and a subset the
    oracle's sequential folds."""
    import torch
    rng = np.random.default_rng(21)
    regions = []
    for name in ("batman", "cookie"):
        img, w, h = fx.load_png_u32(fx.GOLDEN + "/png/%s.png" % name)
        img = img.reshape(h, w)
        for side in (1, 3, 16, 32, 64, 100, 128, 200, 316):
            y0, x0 = int(rng.integers(0, h - side + 1)), int(rng.integers(0, w - side + 1))
            regions.append(np.ascontiguousarray(img[y0:y0 + side, x0:x0 + side]).reshape(-1))
    regions.append(rng.integers(0, 1 << 24, 20000, dtype=np.uint32))                    # > 6144 colours
    regions.append(rng.integers(0, 1 << 24, 140000, dtype=np.uint32) & 0xE0E0E0)        # > 131071 px
    ks = [int(k) for k in rng.choice([1, 2, 4, 7, 16, 64], len(regions))]
    ks[-3] = 100                                                                          # K > 64
    ts = [torch.from_numpy(p.view(np.int32)).to("cuda:0") for p in regions]
    outs = [torch.empty_like(t) for t in ts]
    cts, _ = gpu.quant_weighted_regions_device(ts, outs, ks)
    torch.cuda.synchronize()
    for i, (t, k) in enumerate(zip(ts, ks)):
        o = torch.empty_like(t)
        ct, _ = gpu.quant_device(t, o, k, all_pixels_unique=0)
        torch.cuda.synchronize()
        assert np.array_equal(cts[i], ct), (i, len(regions[i]), k)
        assert torch.equal(outs[i], o), (i, len(regions[i]), k)
    for i in (2, 5, 8, 12):
        ref_out, ref_ct = _oracle(regions[i], ks[i])
        assert np.array_equal(cts[i], ref_ct), i
        assert np.array_equal(outs[i].cpu().numpy().view(np.uint32), ref_out), i
