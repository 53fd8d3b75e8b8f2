"""Shared fixture helpers for tests/, tests/golden/make_golden.py and bench.py.

Test infrastructure: the input generators, the hash and the golden-file I/O.
The xorshift generator and the FNV hash run in C (oracle/_build/libdqoracle.so,
``dqo_xorshift_fill`` / ``dqo_fnv1a64``) because the big configs have 10^7-10^8
pixels.  Nothing here reads /root/reference at run time (the GPU box has none).
"""
import ctypes
import json
import os

import numpy as np

TESTS = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(TESTS)
GOLDEN = os.path.join(TESTS, "golden")
ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "libdqoracle.so")
SEED = 0x9E3779B97F4A7C15

_orc = None


def vp(a):
    return ctypes.c_void_p(a.ctypes.data)


def oracle():
    """Load (building if needed) the CPU restatement -- the checker."""
    global _orc
    if _orc is None:
        if not os.path.exists(ORACLE_SO):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "port"])
        lib = ctypes.CDLL(ORACLE_SO)
        lib.dqo_fnv1a64.restype = ctypes.c_uint64
        lib.dqo_cluster.restype = ctypes.c_int
        lib.dqo_quant_recurse.restype = ctypes.c_int
        _orc = lib
    return _orc


def xorshift(n, seed=SEED):
    out = np.empty(n, np.uint32)
    oracle().dqo_xorshift_fill(vp(out), ctypes.c_uint64(n), ctypes.c_uint64(seed))
    return out


def fnv(a):
    a = np.ascontiguousarray(a, np.uint32)
    return int(oracle().dqo_fnv1a64(vp(a), ctypes.c_uint64(a.size)))


def labels_of(out, ct):
    """Index of each output colour in the colortable (colours are unique after dedup)."""
    lut = {int(c): i for i, c in enumerate(ct)}
    return np.array([lut[int(v)] for v in out], np.int32)


def dump_json(name, obj):
    with open(os.path.join(GOLDEN, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def load_npz(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


# --------------------------------------------------------------------------
# Test/DivQuantTest.m inputs, restated (the 7 known-answer tests).
def kat_inputs():
    gray10 = np.array([(i * 25) * 0x010101 for i in range(10)], np.uint32)  # :33-46 step=(255-0)/10
    umbrella = np.array([0xEBC58B, 0xDAD4E7, 0xD7779D, 0x7E393D, 0xABA4BA, 0xCF4B53,
                         0xC49AC7, 0xAC7292, 0xECEFE7, 0xDC789D, 0xA8ABC4, 0x906E9E,
                         0xB54748, 0xA24F44, 0x857E77, 0x7F654B], np.uint32)  # :219-235
    return {
        "testQuantN1": (gray10, 1),                                   # :31-64
        "testQuantN2": (gray10, 2),                                   # :66-101
        "testQuantN3": (gray10, 3),                                   # :103-142
        "testQuantN3N2": (np.array([0x8DC63F, 0xF26522], np.uint32), 3),  # :147-178
        "testQuantGray2": (np.array([0x0A0A0A, 0xF5F5F5], np.uint32), 2),  # :182-213
        "testQuant_4x4_N4": (umbrella, 4),                            # :218-258
        "testQuant_4x4_N16": (umbrella, 16),                          # :263-319
    }


# Colortables the XCTest asserts literally (Test/DivQuantTest.m line cited).
KAT_EXPECTED = {
    "testQuantN1": [0x000000],                                        # :60-61
    "testQuantN2": [0x323232, 0xAFAFAF],                              # :95-98
    "testQuantN3": [0x191919, 0xAFAFAF, 0x585858],                    # :135-139
    "testQuantN3N2": [0xF26522, 0x8DC63F],                            # :172-175
    "testQuantGray2": [0x0A0A0A, 0xF5F5F5],                           # :207-210
    "testQuant_4x4_N4": [0xA14D48, 0xC292B3, 0xE6D8C8, 0x96758D],      # :251-255
    "testQuant_4x4_N16": [0x7E393D, 0xD7779D, 0xEBC58B, 0x857E77, 0xDAD4E7, 0xABA4BA,
                          0xA24F44, 0xAC7292, 0xCF4B53, 0x7F654B, 0x906E9E, 0xC49AC7,
                          0xECEFE7, 0xB54748, 0xA8ABC4, 0xDC789D],    # :296-316
}


# --------------------------------------------------------------------------
# Small synthetic cases: (n, k, kind, seed).  Inputs are regenerated from the
# spec so only the spec and the expected outputs are committed.
def small_case_specs():
    specs = []
    sizes_k = [(1, 1), (1, 4), (2, 2), (3, 16), (10, 3), (50, 7), (257, 16), (1000, 16),
               (1000, 64), (4099, 256), (4099, 300), (777, 1024), (20000, 256),
               (70001, 32), (65536, 16)]
    kinds = ["uniform", "ties", "gray", "clustered", "coarse", "topbyte"]
    for i, (n, k) in enumerate(sizes_k):
        for j, kind in enumerate(kinds):
            if n > 20000 and kind not in ("uniform", "clustered", "coarse"):
                continue
            specs.append({"n": n, "k": k, "kind": kind, "seed": 1000 + 17 * i + j})
    return specs


def make_case(spec):
    n, kind, seed = spec["n"], spec["kind"], spec["seed"]
    r = xorshift(n, seed=SEED ^ (seed * 0x100000001B3))
    if kind == "uniform":
        return r
    if kind == "topbyte":            # bits 24-31 must be ignored everywhere
        return r | ((xorshift(n, seed=seed) & 0xFF) << 24).astype(np.uint32)
    if kind == "ties":               # 4 colours, many exact duplicates
        pal = np.array([0x3F3F3F, 0x7E7E7E, 0x123456, 0x563412], np.uint32)
        return pal[r % 4]
    if kind == "gray":
        return ((r & 0xFF) * 0x010101).astype(np.uint32)
    if kind == "clustered":          # 5 centres +- 8 noise per channel
        cen = np.array([[20, 30, 40], [200, 10, 90], [128, 128, 128], [250, 240, 230], [60, 200, 60]])
        c = cen[r % 5]
        noise = np.stack([(r >> 8) & 15, (r >> 12) & 15, (r >> 16) & 15], 1).astype(np.int64) - 8
        v = np.clip(c + noise, 0, 255).astype(np.uint32)
        return (v[:, 0] << 16) | (v[:, 1] << 8) | v[:, 2]
    if kind == "coarse":             # 3 bits per channel: heavy ties on every axis
        return (r & 0xE0E0E0).astype(np.uint32)
    raise ValueError(kind)


# --------------------------------------------------------------------------
# Palettes for the map_colors_mps-only fixtures.
def map_palette_specs():
    specs = []
    for k in (1, 2, 3, 5, 16, 64, 255, 256, 1024):
        specs.append({"k": k, "kind": "random", "seed": 77 + k})
    for k in (2, 7, 33, 256, 1000):
        specs.append({"k": k, "kind": "sametsum", "seed": 91 + k})
    for k in (4, 40, 300):
        specs.append({"k": k, "kind": "dups", "seed": 5 + k})
    specs.append({"k": 125, "kind": "subdivided", "seed": 0})
    specs.append({"k": 64, "kind": "gray", "seed": 3})
    return specs


def subdivided_colors():
    """getSubdividedColors (superpixels/OpenCVUtil.cpp:853-897): 5^3 colours, alpha 0xFF."""
    vals = [0, 63, 127, 191, 255]
    return np.array([(0xFF << 24) | (r << 16) | (g << 8) | b
                     for r in vals for g in vals for b in vals], np.uint32)


def make_palette(spec):
    k, kind = spec["k"], spec["kind"]
    r = xorshift(max(k, 1) * 4, seed=SEED + 1 + spec["seed"])
    if kind == "random":
        return r[:k].copy()
    if kind == "sametsum":           # many entries share R+G+B -> std::sort tie order matters
        s = (r[:k] % 5) * 60 + 90
        a = np.minimum(r[k:2 * k] % 256, s)
        b = np.minimum((r[2 * k:3 * k] % 256), s - a)
        c = s - a - b
        ok = c <= 255
        c = np.where(ok, c, 255)
        return ((a << 16) | (b << 8) | c).astype(np.uint32)
    if kind == "dups":
        base = r[:max(1, k // 4)]
        return base[r[k:2 * k] % len(base)].astype(np.uint32)
    if kind == "subdivided":
        return subdivided_colors()
    if kind == "gray":
        return (((r[:k] & 0xFF)) * 0x010101).astype(np.uint32)
    raise ValueError(kind)


# --------------------------------------------------------------------------
def load_png_u32(path):
    """Decode like OpenCV imread(IMREAD_COLOR) + Vec3BToUID (OpenCVUtil.h:19-27):
    alpha dropped, pixel = R<<16 | G<<8 | B."""
    from PIL import Image
    im = Image.open(path).convert("RGB")
    a = np.asarray(im, dtype=np.uint32)
    px = (a[:, :, 0] << 16) | (a[:, :, 1] << 8) | a[:, :, 2]
    return np.ascontiguousarray(px.reshape(-1), np.uint32), im.width, im.height


# --------------------------------------------------------------------------
# Weighted-path (allPixelsUnique=0) cases: duplicate-heavy inputs where the
# reference's weighted FP64 folds and the uniform-weight integer sums often
# decide differently (near-tie TSEs, cuts, 2-means planes), and image regions
# like the app's per-region calls (ClusteringSegmentation.cpp:1779-1803, K=4).
def weighted_case_specs():
    specs = []
    kinds = ["fewcolours", "greyramp", "tight", "coarse"]
    ks = [1, 2, 3, 4, 5, 8, 16, 64]
    for i in range(320):
        n = 1 + (int(xorshift(1, seed=0xA5A5 + i)[0]) % 3000)
        specs.append({"n": n, "k": ks[i % len(ks)], "kind": kinds[i % 4], "seed": 5000 + i})
    for i, (name, k) in enumerate([(nm, k) for nm in ("batman", "cookie") for k in (2, 4, 8, 16)]):
        for j in range(4):
            specs.append({"n": 0, "k": k, "kind": "crop_" + name, "seed": 7000 + 10 * i + j})
    return specs


def make_weighted_case(spec):
    n, kind, seed = spec["n"], spec["kind"], spec["seed"]
    if kind.startswith("crop_"):   # a rectangle of a sample image, 1K..40K pixels
        px, w, h = load_png_u32(os.path.join(GOLDEN, "png", kind[5:] + ".png"))
        r = xorshift(4, seed=seed)
        cw, ch = 16 + int(r[0]) % 200, 16 + int(r[1]) % 200
        x0, y0 = int(r[2]) % (w - cw), int(r[3]) % (h - ch)
        return np.ascontiguousarray(px.reshape(h, w)[y0:y0 + ch, x0:x0 + cw].reshape(-1))
    r = xorshift(4 * n + 64, seed=seed)
    if kind == "fewcolours":   # a small palette, skewed counts (geometric-like)
        ncol = 2 + int(r[0]) % 38
        pal = r[1:1 + ncol]
        sel = np.minimum(np.log2(1 + (r[64:64 + n] & 0xFFFF)).astype(np.int64), ncol - 1)
        return pal[sel].astype(np.uint32)
    if kind == "greyramp":
        return (((r[64:64 + n] % 32) * 8) * 0x010101).astype(np.uint32)
    if kind == "tight":        # one cluster, +-3 per channel
        base = np.array([60 + int(r[0]) % 140, 60 + int(r[1]) % 140, 60 + int(r[2]) % 140], np.int64)
        d = np.stack([r[64:64 + n] % 7, (r[64:64 + n] >> 8) % 7, (r[64:64 + n] >> 16) % 7], 1).astype(np.int64) - 3
        c = np.clip(base + d, 0, 255).astype(np.uint32)
        return (c[:, 0] << 16) | (c[:, 1] << 8) | c[:, 2]
    if kind == "coarse":
        return (r[64:64 + n] & 0xC0C0C0).astype(np.uint32)
    raise ValueError(kind)


# --------------------------------------------------------------------------
# quant_varpart_fast's cut_bits / decimation paths (DivQuantCluster.cpp:1130-
# 1146): num_bits < 8 and/or dec_factor > 1, either flag value.
# Frame shapes keep the reference's numRows-stride index (calc_color_table
# :124) inside the buffer: rows == 1, or rows <= cols.
def varpart_case_specs():
    specs = []
    shapes = [(1, 4096), (64, 64), (48, 80), (1, 3001), (33, 57), (128, 128)]
    kinds = ["uniform", "crop_batman", "crop_cookie", "fewcolours", "tight", "greyramp"]
    ks = [1, 2, 4, 16, 64, 256]
    i = 0
    for nb in range(1, 9):
        for dec in (1, 2, 3, 5):
            for uniq in (0, 1):
                if nb == 8 and dec == 1:
                    continue   # the plain paths (cases / weighted fixtures)
                rows, cols = shapes[i % len(shapes)]
                specs.append({"rows": rows, "cols": cols, "num_bits": nb, "dec": dec, "uniq": uniq,
                              "k": ks[(i * 7) % len(ks)], "kind": kinds[i % len(kinds)], "seed": 9000 + i,
                              "max_iters": 10 if i % 5 else 3})
                i += 1
    return specs


def make_varpart_case(spec):
    n = spec["rows"] * spec["cols"]
    kind = spec["kind"]
    if kind == "uniform":
        return xorshift(n, seed=spec["seed"])
    if kind.startswith("crop_"):
        px, w, h = load_png_u32(os.path.join(GOLDEN, "png", kind[5:] + ".png"))
        r = xorshift(2, seed=spec["seed"])
        x0, y0 = int(r[0]) % (w - 128), int(r[1]) % (h - 128)
        crop = px.reshape(h, w)[y0:y0 + 128, x0:x0 + 128].reshape(-1)
        return np.ascontiguousarray(crop[:n])
    return make_weighted_case({"n": n, "kind": kind, "seed": spec["seed"]})
