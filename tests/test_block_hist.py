"""Full-frame fixed-palette map + 4x4 block histograms (SURVEY 8f.1,
genHistogramsForBlocks, ClusteringSegmentation.cpp:365-576).

Oracle: oracle/dq_oracle.cpp dqo_block_hist restates the block loop with the
reference's own container (std::unordered_map<uint32_t,uint32_t>), so its
tie-break is the reference's iteration order on this toolchain; the mapped
frame comes from dqo_map (pinned to the reference by test_oracle_golden.py).
The reference function itself needs OpenCV (not in this image): its block
loop is not run here, so the pin is the container plus the map's golden pin.

CPU tests: the closed form of that iteration order used by the kernel
(csrc/stl_order.h) against the real container; palette and block grid.
GPU tests: the HIP path bit-exact against the oracle (mode, histogram tables)
on tie-heavy frames, ragged edges, every supported block size, and the
reference's sample images.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import dq_fixtures as fx

NATIVE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")


def _oracle_block_hist(frame, dim, palette):
    orc = fx.oracle()
    h, w = frame.shape
    px = np.ascontiguousarray(frame, np.uint32).reshape(-1)
    quant = np.zeros(px.size, np.uint32)
    orc.dqo_map(fx.vp(px), ctypes.c_uint32(px.size), fx.vp(quant), fx.vp(palette),
                ctypes.c_int(palette.size))
    bw, bh = -(-w // dim), -(-h // dim)
    mode = np.zeros(bw * bh, np.uint32)
    nd = np.zeros(bw * bh, np.uint32)
    keys = np.zeros(bw * bh * dim * dim, np.uint32)
    counts = np.zeros(bw * bh * dim * dim, np.uint32)
    orc.dqo_block_hist(fx.vp(quant), ctypes.c_uint32(w), ctypes.c_uint32(h), ctypes.c_uint32(bw),
                       ctypes.c_uint32(bh), ctypes.c_uint32(dim), fx.vp(mode), fx.vp(nd),
                       fx.vp(keys), fx.vp(counts))
    cap = dim * dim
    return (quant.reshape(h, w), mode.reshape(bh, bw), nd.reshape(bh, bw),
            keys.reshape(bh, bw, cap), counts.reshape(bh, bw, cap))


def _tie_frame(h, w, seed, ncolors=6):
    """Blocks of a few palette-mapped colours: 8/8, 4/4/4/4 ... ties everywhere."""
    r = fx.xorshift(h * w + ncolors, seed=seed)
    base = r[:ncolors] & 0xFFFFFF
    return base[r[ncolors:] % ncolors].reshape(h, w).astype(np.uint32)


# ---------------------------------------------------------------------------
# CPU
def test_stl_order_closed_form_matches_libstdcxx(tmp_path):
    exe = str(tmp_path / "stl_order_check")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-o", exe,
                           os.path.join(NATIVE, "stl_order_check.cpp")], timeout=120)
    res = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stdout + res.stderr
    assert "mismatches 0" in res.stdout


def test_subdivided_colors(pkg):
    ours = pkg.get_subdivided_colors()
    ref = np.zeros(125, np.uint32)
    fx.oracle().dqo_subdivided_colors(fx.vp(ref))
    assert np.array_equal(ours, ref)
    assert np.array_equal(ours, fx.subdivided_colors())
    assert len(set(ours.tolist())) == 125


def test_subdivided_colors_reference_test(pkg):
    """The reference's own test of this palette, testSegmentColorCube
    (Test/CoordTest.mm:2101-2170), restated on the library's table: 125
    entries; the entries with R = G = 0 are exactly five, B = 0, 63, 127, 191,
    255 in table order, and they are colortable[0..4] = 0xFF000000,
    0xFF00003F, 0xFF00007F, 0xFF0000BF, 0xFF0000FF (the comment block at
    :2116-2120); every value 0..255 has a nearest of those five bins (first
    on ties), 256 in all."""
    vec = pkg.get_subdivided_colors()
    assert vec.size == 125
    filtered = [int(p) & 0xFF for p in vec.tolist() if (int(p) & 0x00FFFF00) == 0]
    assert filtered == [0, 63, 127, 191, 255]
    assert vec[:5].tolist() == [0xFF000000, 0xFF00003F, 0xFF00007F, 0xFF0000BF, 0xFF0000FF]
    counts = {}
    for i in range(256):
        best, bi = 256, None
        for j, f in enumerate(filtered):
            if abs(i - f) < best:
                best, bi = abs(i - f), j
        counts[bi] = counts.get(bi, 0) + 1
    assert sum(counts.values()) == 256 and sorted(counts) == [0, 1, 2, 3, 4]


def test_block_grid(pkg):
    # clusteringCombine (ClusteringSegmentationMain.cpp:138-149)
    assert pkg.block_grid(1778, 1000, 4) == (445, 250)
    assert pkg.block_grid(1000, 1000, 4) == (250, 250)
    assert pkg.block_grid(3840, 2160, 4) == (960, 540)
    assert pkg.block_grid(5, 3, 4) == (2, 1)


def test_oracle_block_hist_invariants():
    frame = _tie_frame(13, 18, seed=5)
    pal = fx.subdivided_colors()
    quant, mode, nd, keys, counts = _oracle_block_hist(frame, 4, pal)
    bh, bw = mode.shape
    for by in range(bh):
        for bx in range(bw):
            blk = quant[by * 4:by * 4 + 4, bx * 4:bx * 4 + 4].reshape(-1)
            n = int(nd[by, bx])
            k, c = keys[by, bx, :n], counts[by, bx, :n]
            assert sorted(k.tolist()) == sorted(set(blk.tolist()))
            assert int(c.sum()) == blk.size
            # mode = first key with the largest count, in the table's order
            assert mode[by, bx] == k[int(np.argmax(c))]


# ---------------------------------------------------------------------------
# GPU
def _check(gpu, frame, dim, palette=None):
    pal = fx.subdivided_colors() if palette is None else palette
    bgr, mode, quant, (nd, keys, counts) = gpu.gen_histograms_for_blocks(
        frame, superpixel_dim=dim, palette=pal, tables=True)
    rq, rmode, rnd, rkeys, rcounts = _oracle_block_hist(frame, dim, pal)
    assert np.array_equal(quant, rq)
    assert np.array_equal(nd, rnd)
    assert np.array_equal(keys, rkeys)
    assert np.array_equal(counts, rcounts)
    assert np.array_equal(mode, rmode)
    assert np.array_equal(bgr[..., 0], rmode & 0xFF)
    assert np.array_equal(bgr[..., 2], (rmode >> 16) & 0xFF)
    # without tables only tie blocks take the ranking kernel
    _, mode2, _ = gpu.gen_histograms_for_blocks(frame, superpixel_dim=dim, palette=pal)
    assert np.array_equal(mode2, rmode)
    return mode


@pytest.mark.gpu
@pytest.mark.parametrize("ncolors", [2, 3, 6, 40])
def test_block_hist_ties(gpu, ncolors):
    mode = _check(gpu, _tie_frame(64, 96, seed=11 + ncolors, ncolors=ncolors), 4)
    assert mode.shape == (16, 24)


@pytest.mark.gpu
@pytest.mark.parametrize("dim", [1, 2, 3, 4])
def test_block_hist_dims_ragged(gpu, dim):
    # random colours (up to dim^2 distinct keys per block: 14..16 exercise the
    # 13 -> 29 bucket rehash) and ragged right / bottom edges
    h, w = 3 * dim + 2, 5 * dim + 3
    frame = (fx.xorshift(h * w, seed=100 + dim) & 0xFFFFFF).reshape(h, w)
    _check(gpu, frame, dim)
    _check(gpu, _tie_frame(h, w, seed=200 + dim, ncolors=5), dim)


@pytest.mark.gpu
def test_block_hist_other_palette(gpu):
    pal = fx.make_palette({"k": 64, "kind": "dups", "seed": 2})
    _check(gpu, _tie_frame(40, 44, seed=7, ncolors=30), 4, palette=pal)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["batman", "cookie"])
def test_block_hist_sample_images(gpu, name):
    """The app's own call: genHistogramsForBlocks on the reference's sample
    images (clusteringCombine, ClusteringSegmentationMain.cpp:268)."""
    px, w, h = fx.load_png_u32(os.path.join(fx.GOLDEN, "png", name + ".png"))
    _check(gpu, px.reshape(h, w), 4)


@pytest.mark.gpu
def test_block_hist_device(gpu):
    import torch
    h, w, dim = 1080, 1920, 4
    frame = _tie_frame(h, w, seed=3, ncolors=12)
    t_in = torch.from_numpy(frame.reshape(-1).view(np.int32)).to("cuda:0")
    t_q = torch.empty_like(t_in)
    bw, bh = gpu.block_grid(w, h, dim)
    t_mode = torch.empty(bw * bh, dtype=torch.int32, device="cuda:0")
    gpu.block_hist_device(t_in, w, h, t_q, t_mode, superpixel_dim=dim)
    torch.cuda.synchronize()
    _, rmode, _, _, _ = _oracle_block_hist(frame, dim, fx.subdivided_colors())
    assert np.array_equal(t_mode.cpu().numpy().view(np.uint32).reshape(bh, bw), rmode)


@pytest.mark.gpu
def test_block_hist_bad_args(gpu):
    with pytest.raises(gpu.DivQuantError):
        gpu.gen_histograms_for_blocks(np.zeros((8, 8), np.uint32), superpixel_dim=5)


@pytest.mark.gpu
def test_block_hist_device_two_streams(gpu):
    """Two asynchronous calls on two streams back to back: each call's tie
    queues are its own, so both results are exact."""
    import torch
    h, w, dim = 1080, 1920, 4
    frames = [_tie_frame(h, w, seed=11 + i, ncolors=4 + 4 * i) for i in range(2)]
    bw, bh = gpu.block_grid(w, h, dim)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    ins = [torch.from_numpy(f.reshape(-1).view(np.int32)).to("cuda:0") for f in frames]
    torch.cuda.synchronize()
    qs = [torch.empty_like(t) for t in ins]
    modes = [torch.empty(bw * bh, dtype=torch.int32, device="cuda:0") for _ in ins]
    for _ in range(3):
        for i in range(2):
            gpu.block_hist_device(ins[i], w, h, qs[i], modes[i], superpixel_dim=dim, stream=streams[i])
    torch.cuda.synchronize()
    for i in range(2):
        _, rmode, _, _, _ = _oracle_block_hist(frames[i], dim, fx.subdivided_colors())
        assert np.array_equal(modes[i].cpu().numpy().view(np.uint32).reshape(bh, bw), rmode), i
