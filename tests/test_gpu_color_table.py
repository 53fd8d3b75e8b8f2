"""The device colour table (dq_weighted.hip launch_color_table: runs of equal
pixels partitioned by hash-bucket group, an LDS hash table per group, ranks
by first occurrence inside each bucket) through the reference's host
signature calc_color_table (DivQuantMapColors.cpp:82-203), against the
oracle's restatement (dqo_color_table) on the cases that stress its parts:
one colour everywhere (one hot slot), long stripes (runs across the 256-pixel
run limit and the 1024-pixel wave steps), every colour of the fullest hash
bucket (844 colours ranked in one bucket), one group filled to its limit
(4 buckets, 3376 colours), ragged sizes, 2-D decimated walks, and an input
that is not 16-B aligned.  Colours and weight bits must be identical."""
import ctypes

import numpy as np
import pytest

import dq_fixtures as fx

pytestmark = pytest.mark.gpu

_BUCKETS = None


def _buckets():
    global _BUCKETS
    if _BUCKETS is None:
        c = np.arange(1 << 24, dtype=np.int64)
        _BUCKETS = (((c >> 16) & 255) * 33023 + ((c >> 8) & 255) * 30013 + (c & 255) * 27011) % 20023
    return _BUCKETS


def _cct(lib):
    f = getattr(lib, "_Z16calc_color_tablePKjjPjjjiPi")
    f.restype = ctypes.POINTER(ctypes.c_double)
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                  ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    return f


def _oracle(pts):
    n = len(pts)
    col = np.zeros(max(n, 1), np.uint32)
    w = np.zeros(max(n, 1), np.float64)
    u = fx.oracle().dqo_color_table(ctypes.c_uint32(n), fx.vp(pts), fx.vp(col), fx.vp(w))
    return col[:u], w[:u]


def _check(lib, px, rows=1, cols=None, dec=1):
    cols = len(px) if cols is None else cols
    cct = _cct(lib)
    m = ((rows + dec - 1) // dec) * ((cols + dec - 1) // dec)
    out = np.zeros(max(m, 1), np.uint32)
    nc = ctypes.c_int(0)
    w = cct(fx.vp(px), len(px), fx.vp(out), rows, cols, dec, ctypes.byref(nc))
    # the reference's walk: inPixels[ic + ir*numRows] (:120-125)
    idx = np.array([ic + ir * rows for ir in range(0, rows, dec) for ic in range(0, cols, dec)], np.int64) \
        if (rows != 1 or dec != 1) else np.arange(cols)
    pts = np.ascontiguousarray(px[idx] & 0xFFFFFF)
    rc, rw = _oracle(pts)
    got_w = np.ctypeslib.as_array(w, shape=(max(nc.value, 1),))[:nc.value].copy()
    assert nc.value == len(rc), (len(px), nc.value, len(rc))
    assert np.array_equal(out[:nc.value], rc)
    assert np.array_equal(got_w.view(np.uint64), rw.view(np.uint64))


@pytest.fixture(scope="module")
def lib(gpu):
    return ctypes.CDLL(gpu.LIB_PATH)


def test_hot_slot_and_stripes(lib):
    n = 300001
    _check(lib, np.full(n, 0x123456, np.uint32))                      # one colour
    px = np.repeat(np.array([0xFF0000, 0x00FF00, 0x0000FF, 0xFF0000], np.uint32), [70000, 90001, 1, 139999])
    px[::9973] = 0xABCDEF                                               # singletons inside the runs
    _check(lib, px)
    rng = np.random.default_rng(3)
    runs = rng.integers(1, 3000, 400)
    px = np.repeat(rng.integers(0, 1 << 24, 400, dtype=np.uint32), runs)
    _check(lib, px)


def test_fullest_bucket_and_full_group(lib):
    b = _buckets()
    cnt = np.bincount(b, minlength=20023)
    h = int(np.argmax(cnt))
    full = np.nonzero(b == h)[0].astype(np.uint32)                    # 844 colours, one bucket
    rng = np.random.default_rng(5)
    _check(lib, full[rng.integers(0, len(full), 200000)])
    g = h // 4                                                        # its group of 4 buckets
    grp = np.nonzero((b >= 4 * g) & (b < 4 * g + 4))[0].astype(np.uint32)
    assert len(grp) >= 3300
    px = np.concatenate([rng.permutation(grp), grp[rng.integers(0, len(grp), 150000)]])
    _check(lib, px)


@pytest.mark.parametrize("n", [1, 2, 15, 17, 1023, 1025, 131073, 1000003])
def test_ragged_sizes(lib, n):
    rng = np.random.default_rng(n)
    _check(lib, rng.integers(0, 1 << 24, n, dtype=np.uint32) & (0xFFFFFF if n % 2 else 0xF0E0F0))


def test_decimated_and_2d_walks(lib):
    rng = np.random.default_rng(9)
    img = rng.integers(0, 1 << 24, 600 * 600, dtype=np.uint32) & 0xFCFCFC
    for rows, cols, dec in ((600, 600, 1), (600, 600, 2), (600, 600, 3), (500, 600, 4), (1, 360000, 5)):
        _check(lib, img, rows, cols, dec)


def test_unaligned_device_input(gpu):
    """quant_device on a tensor view one pixel in (4-B aligned, not 16):
    the weighted path's colour table reads it unvectorised, same result."""
    import torch
    rng = np.random.default_rng(13)
    n = 200000
    px = rng.integers(0, 1 << 24, n + 1, dtype=np.uint32) & 0xF8F8F8
    t = torch.from_numpy(px.view(np.int32)).to("cuda:0")[1:]
    o = torch.empty_like(t)
    gpu.set_wsmall(False)
    try:
        ct, _ = gpu.quant_device(t, o, 16, all_pixels_unique=0)
    finally:
        gpu.set_wsmall(True)
    ref_out = np.zeros(n, np.uint32)
    ref_ct = np.zeros(16, np.uint32)
    kk = ctypes.c_uint32(16)
    p = np.ascontiguousarray(px[1:])
    fx.oracle().dqo_quant_recurse_weighted(ctypes.c_uint32(n), fx.vp(p), fx.vp(ref_out), ctypes.byref(kk),
                                           fx.vp(ref_ct))
    assert np.array_equal(ct, ref_ct[:kk.value])
    assert np.array_equal(o.cpu().numpy().view(np.uint32), ref_out)
