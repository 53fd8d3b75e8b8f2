"""BGR24 ingestion / output on the GPU.

The app converts its OpenCV CV_8UC3 frame pixel by pixel on the CPU with
Vec3BToUID (superpixels/OpenCVUtil.h:19-27; ClusteringSegmentation.cpp:381-395,
the region gather at :1795-1800) and writes results back with PixelToVec3b
(OpenCVUtil.h:53-59; :1812-1817).  dq_hip_{pack,unpack,gather}_bgr24_dev do
that on HBM-resident frames.

Oracle: dqo_pack_bgr24 / dqo_unpack_bgr24 / dqo_gather_bgr24
(oracle/dq_oracle.cpp).  Pin: packing the reference's sample PNGs (decoded to
BGR as imread(IMREAD_COLOR) returns them) reproduces the committed input
hashes `px_fnv` of tests/golden/png.json, which the reference build was run
on.  CPU tests: the oracle against that pin and against numpy.  GPU tests:
the HIP kernels bit-exact against the oracle on aligned (fast) and ragged /
padded / misaligned (per-pixel) layouts, untouched row padding, and the
PNGs end to end (pack -> quant_recurse -> unpack) against the golden tables.
"""
import ctypes

import numpy as np
import pytest

import dq_fixtures as fx


def _png_bgr(name):
    from PIL import Image
    im = Image.open(fx.os.path.join(fx.GOLDEN, "png", name + ".png")).convert("RGB")
    rgb = np.asarray(im, dtype=np.uint8)
    return np.ascontiguousarray(rgb[:, :, ::-1]), im.width, im.height   # OpenCV order: B, G, R


def _frame(w, h, stride, seed, fill=0xAB):
    """A CV_8UC3-like buffer: h rows of `stride` bytes, padding bytes = fill."""
    buf = np.full(h * stride, fill, np.uint8)
    r = fx.xorshift(max(1, (3 * w * h + 3) // 4), seed).view(np.uint8)[:3 * w * h]
    rows = buf.reshape(h, stride)
    rows[:, :3 * w] = r.reshape(h, 3 * w)
    return buf


def _orc_pack(buf, w, h, stride):
    out = np.zeros(w * h, np.uint32)
    fx.oracle().dqo_pack_bgr24(fx.vp(buf), ctypes.c_uint32(w), ctypes.c_uint32(h),
                               ctypes.c_uint32(stride), fx.vp(out))
    return out


def _orc_unpack(px, w, h, stride, fill=0xAB):
    buf = np.full(h * stride, fill, np.uint8)
    fx.oracle().dqo_unpack_bgr24(fx.vp(px), ctypes.c_uint32(w), ctypes.c_uint32(h),
                                 ctypes.c_uint32(stride), fx.vp(buf))
    return buf


def _orc_gather(buf, stride, coords):
    out = np.zeros(coords.size, np.uint32)
    fx.oracle().dqo_gather_bgr24(fx.vp(buf), ctypes.c_uint32(stride), fx.vp(coords),
                                 ctypes.c_uint32(coords.size), fx.vp(out))
    return out


# ---------------------------------------------------------------- CPU ------
@pytest.mark.parametrize("name", ["batman", "cookie"])
def test_oracle_pack_pinned_by_png_fixture(name):
    bgr, w, h = _png_bgr(name)
    px = _orc_pack(bgr.reshape(-1), w, h, 3 * w)
    fix = fx.load_json("png.json")[name]
    assert (w, h) == (fix["w"], fix["h"])
    assert "%016x" % fx.fnv(px) == fix["px_fnv"]


def test_oracle_matches_numpy_and_round_trips():
    w, h, stride = 37, 5, 3 * 37 + 7
    buf = _frame(w, h, stride, 11)
    px = _orc_pack(buf, w, h, stride)
    rows = buf.reshape(h, stride)[:, :3 * w].reshape(h, w, 3).astype(np.uint32)
    want = (rows[:, :, 2] << 16) | (rows[:, :, 1] << 8) | rows[:, :, 0]
    assert np.array_equal(px, want.reshape(-1))
    # unpack ignores bits 24-31 and leaves the row padding alone
    back = _orc_unpack(px | np.uint32(0x5A000000), w, h, stride)
    assert np.array_equal(back, buf)
    coords = np.array([0, 36, (4 << 16) | 36, (2 << 16) | 17], np.uint32)
    got = _orc_gather(buf, stride, coords)
    assert list(got) == [px[0], px[36], px[4 * w + 36], px[2 * w + 17]]


# ---------------------------------------------------------------- GPU ------
LAYOUTS = [
    # (width, height, extra stride bytes, base offset): fast path needs
    # width % 4 == 0, stride % 4 == 0 and a 4-B aligned base
    (3840, 2160, 0, 0),     # 4K continuous Mat (fast)
    (64, 3, 4, 0),          # padded rows, still fast
    (1001, 7, 5, 0),        # ragged width and stride (per pixel)
    (256, 9, 0, 1),         # misaligned base pointer (per pixel)
    (1, 1, 0, 0),
    (4, 70000, 0, 0),       # more rows than one grid dimension holds
]


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,pad,off", LAYOUTS)
def test_pack_unpack_bit_exact(gpu, w, h, pad, off):
    import torch
    stride = 3 * w + pad
    buf = _frame(w, h, stride, 3 + w + h)
    d_raw = torch.zeros(buf.size + 16, dtype=torch.uint8, device="cuda:0")
    d_raw[off:off + buf.size] = torch.from_numpy(buf).to("cuda:0")
    d_bgr = d_raw[off:off + buf.size]
    d_px = torch.empty(w * h, dtype=torch.int32, device="cuda:0")
    gpu.pack_bgr24_device(d_bgr, w, h, d_px, stride=stride)
    torch.cuda.synchronize()
    want = _orc_pack(buf, w, h, stride)
    got = d_px.cpu().numpy().view(np.uint32)
    assert np.array_equal(got, want)

    # unpack: set bits 24-31 (dropped), padding bytes must stay 0xAB
    d_px |= 0x3C000000
    d_out_raw = torch.full((buf.size + 16,), 0xAB, dtype=torch.uint8, device="cuda:0")
    d_out = d_out_raw[off:off + buf.size]
    gpu.unpack_bgr24_device(d_px, w, h, d_out, stride=stride)
    torch.cuda.synchronize()
    assert np.array_equal(d_out.cpu().numpy(), buf)
    raw = d_out_raw.cpu().numpy()
    assert (raw[:off] == 0xAB).all() and (raw[off + buf.size:] == 0xAB).all()


@pytest.mark.gpu
def test_gather_bit_exact(gpu):
    import torch
    w, h = 3840, 2160
    stride = 3 * w
    buf = _frame(w, h, stride, 99)
    r = fx.xorshift(200001, 7)
    coords = (((r >> 16) % h) << 16 | (r & 0xFFFF) % w).astype(np.uint32)
    coords[:2] = [0, ((h - 1) << 16) | (w - 1)]
    d_bgr = torch.from_numpy(buf).to("cuda:0")
    d_c = torch.from_numpy(coords.view(np.int32)).to("cuda:0")
    d_out = torch.empty(coords.size, dtype=torch.int32, device="cuda:0")
    gpu.gather_bgr24_device(d_bgr, stride, d_c, coords.size, d_out)
    torch.cuda.synchronize()
    assert np.array_equal(d_out.cpu().numpy().view(np.uint32), _orc_gather(buf, stride, coords))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["batman", "cookie"])
def test_png_bgr_end_to_end(gpu, name):
    """BGR Mat on the device -> pack -> quant_recurse (K=16) -> unpack: the
    colortable the reference produced on this image, and the output Mat equal
    to the oracle's map unpacked."""
    import torch
    fix = fx.load_json("png.json")[name]
    bgr, w, h = _png_bgr(name)
    n = w * h
    d_bgr = torch.from_numpy(bgr.reshape(-1)).to("cuda:0")
    d_px = torch.empty(n, dtype=torch.int32, device="cuda:0")
    d_q = torch.empty(n, dtype=torch.int32, device="cuda:0")
    gpu.pack_bgr24_device(d_bgr, w, h, d_px)
    torch.cuda.synchronize()
    ct, _ = gpu.quant_device(d_px, d_q, 16)
    assert list(ct) == fix["k16"]["ct"]
    d_out = torch.empty(3 * n, dtype=torch.uint8, device="cuda:0")
    gpu.unpack_bgr24_device(d_q, w, h, d_out)
    torch.cuda.synchronize()
    px = _orc_pack(bgr.reshape(-1), w, h, 3 * w)
    mapped = np.zeros(n, np.uint32)
    ct_u32 = np.asarray(ct, np.uint32)   # (alive across the call)
    fx.oracle().dqo_map(fx.vp(px), ctypes.c_uint32(n), fx.vp(mapped), fx.vp(ct_u32),
                        ctypes.c_int(len(ct)))
    assert "%016x" % fx.fnv(mapped) == fix["k16"]["out_fnv"]
    assert np.array_equal(d_out.cpu().numpy(), _orc_unpack(mapped, w, h, 3 * w))


# ------------------------------------------- fused BGR24 reads (GPU) -------
def _bgr_of(px):
    """Packed 0x00RRGGBB -> BGR24 bytes (PixelToVec3b order)."""
    px = np.asarray(px, np.uint32)
    return np.stack([px & 0xFF, (px >> 8) & 0xFF, (px >> 16) & 0xFF], -1).astype(np.uint8).reshape(-1)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["batman", "cookie"])
def test_fused_bgr24_png(gpu, name):
    """quant_recurse straight from the Mat's BGR24 bytes (the root's passes,
    its partition and the map read 3-B pixels): the reference's
    colortables and output hashes for the sample images, uniform-weight K in
    {4, 16, 125, 256} and weighted K in {4, 16}."""
    import torch
    fix = fx.load_json("png.json")[name]
    bgr, w, h = _png_bgr(name)
    d_bgr = torch.from_numpy(bgr.reshape(-1)).to("cuda:0")
    d_out = torch.empty(w * h, dtype=torch.int32, device="cuda:0")
    for k in (4, 16, 125, 256):
        ct, _ = gpu.quant_bgr24_device(d_bgr, w, h, d_out, k)
        torch.cuda.synchronize()
        assert [int(v) for v in ct] == fix["k%d" % k]["ct"], (name, k)
        assert "%016x" % fx.fnv(d_out.cpu().numpy().view(np.uint32)) == fix["k%d" % k]["out_fnv"], (name, k)
    for k in (4, 16):
        ct, _ = gpu.quant_bgr24_device(d_bgr, w, h, d_out, k, all_pixels_unique=0)
        torch.cuda.synchronize()
        assert [int(v) for v in ct] == fix["k%d_weighted" % k]["ct"], (name, k)
        assert "%016x" % fx.fnv(d_out.cpu().numpy().view(np.uint32)) == fix["k%d_weighted" % k]["out_fnv"]


@pytest.mark.gpu
def test_fused_bgr24_c4_frames(gpu):
    """Two of C4's 4K frames (seed + f) as BGR24, one batched call
    over the engine lanes: every frame's colortable and output hash equal the
    reference's (tests/golden/c4.json)."""
    import torch
    fix = fx.load_json("c4.json")
    w, h = 3840, 2160
    frames = [torch.from_numpy(_bgr_of(fx.xorshift(w * h, seed=fx.SEED + f))).to("cuda:0") for f in range(2)]
    outs = [torch.empty(w * h, dtype=torch.int32, device="cuda:0") for _ in range(2)]
    cts, _ = gpu.quant_bgr24_batch_device(frames, w, h, outs, 256)
    torch.cuda.synchronize()
    for f in range(2):
        r = fix["f%02d" % f]
        assert [int(v) for v in cts[f]] == r["ct"], f
        assert "%016x" % fx.fnv(outs[f].cpu().numpy().view(np.uint32)) == r["out_fnv"], f


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,pad,off", [(333, 77, 0, 0), (256, 64, 0, 1), (320, 50, 0, 0), (100, 40, 5, 0),
                                         (1, 1, 0, 0), (17, 3, 0, 3)])
def test_fused_bgr24_layouts(gpu, w, h, pad, off):
    """Ragged pixel counts (not a multiple of 16), misaligned frames and padded
    rows take the staged / packed forms: results equal the packed path's on
    the same pixels (colortable, output), uniform and weighted."""
    import torch
    stride = 3 * w + pad
    buf = _frame(w, h, stride, seed=1000 + w + h)
    px = _orc_pack(buf, w, h, stride)
    raw = torch.zeros(len(buf) + 64, dtype=torch.uint8, device="cuda:0")
    raw[off:off + len(buf)] = torch.from_numpy(buf).to("cuda:0")
    d_bgr = raw[off:off + len(buf)]
    d_px = torch.from_numpy(px.view(np.int32)).to("cuda:0")
    d_a = torch.empty(w * h, dtype=torch.int32, device="cuda:0")
    d_b = torch.empty(w * h, dtype=torch.int32, device="cuda:0")
    for k, uniq in ((16, 1), (5, 1), (8, 0)):
        ct_a, _ = gpu.quant_bgr24_device(d_bgr, w, h, d_a, k, stride=stride, all_pixels_unique=uniq)
        ct_b, _ = gpu.quant_device(d_px, d_b, k, all_pixels_unique=uniq)
        torch.cuda.synchronize()
        assert list(ct_a) == list(ct_b), (k, uniq)
        assert torch.equal(d_a, d_b), (k, uniq)


@pytest.mark.gpu
def test_map_bgr24(gpu):
    """map_colors_mps from BGR24 bytes (direct for K <= 1024, packed first
    above) equals the oracle's map of the packed pixels."""
    import torch
    w, h = 640, 360
    px = fx.xorshift(w * h, seed=4242) & np.uint32(0xFFFFFF)
    d_bgr = torch.from_numpy(_bgr_of(px)).to("cuda:0")
    d_out = torch.empty(w * h, dtype=torch.int32, device="cuda:0")
    for k in (1, 16, 300, 1024, 2000):
        pal = fx.xorshift(k, seed=77 + k) & np.uint32(0xFFFFFF)
        gpu.map_bgr24_device(d_bgr, w, h, d_out, pal)
        torch.cuda.synchronize()
        want = np.zeros(w * h, np.uint32)
        fx.oracle().dqo_map(fx.vp(px), ctypes.c_uint32(len(px)), fx.vp(want), fx.vp(pal), ctypes.c_int(k))
        assert np.array_equal(d_out.cpu().numpy().view(np.uint32), want), k
