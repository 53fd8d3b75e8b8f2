"""CPU: pin the oracle (oracle/dq_oracle.cpp, the CPU restatement used as the
checker) against the reference's own known answers (Test/DivQuantTest.m) and
against outputs of the unmodified reference compiled here
(tests/golden/, made by tests/golden/make_golden.py)."""
import ctypes

import numpy as np
import pytest

import dq_fixtures as fx


def oracle_quant(px, k):
    orc = fx.oracle()
    px = np.ascontiguousarray(px, np.uint32)
    out = np.zeros(len(px), np.uint32)
    ct = np.zeros(k, np.uint32)
    kk = ctypes.c_uint32(k)
    orc.dqo_quant_recurse(ctypes.c_uint32(len(px)), fx.vp(px), fx.vp(out), ctypes.byref(kk), fx.vp(ct))
    return out, ct[:kk.value]


def oracle_cluster(px, k, max_iters=10):
    orc = fx.oracle()
    px = np.ascontiguousarray(px, np.uint32)
    ct = np.zeros(k, np.uint32)
    kk = ctypes.c_uint32(k)
    means = np.zeros((k, 3), np.float64)
    sizes = np.zeros(k, np.int64)
    trace = np.zeros((max(k - 1, 1), 4), np.int64)
    orc.dqo_cluster(ctypes.c_uint32(len(px)), fx.vp(px), ctypes.byref(kk), fx.vp(ct),
                    ctypes.c_int(max_iters), fx.vp(means), fx.vp(sizes), fx.vp(trace))
    return ct[:kk.value], means, sizes, trace[:k - 1]


def oracle_map(px, pal):
    px = np.ascontiguousarray(px, np.uint32)
    pal = np.ascontiguousarray(pal, np.uint32)
    out = np.zeros(len(px), np.uint32)
    fx.oracle().dqo_map(fx.vp(px), ctypes.c_uint32(len(px)), fx.vp(out), fx.vp(pal), ctypes.c_int(len(pal)))
    return out


def check_means(means, sizes, ref_means):
    filled = ~np.isnan(ref_means[:, 0])
    assert np.array_equal(filled, sizes > 0)
    assert np.array_equal(means[filled].view(np.uint64), ref_means[filled].view(np.uint64))


@pytest.mark.parametrize("name", sorted(fx.KAT_EXPECTED))
def test_kat_literal(name):
    """The colortables Test/DivQuantTest.m asserts."""
    px, k = fx.kat_inputs()[name]
    out, ct = oracle_quant(px, k)
    assert [int(v) for v in ct] == fx.KAT_EXPECTED[name]


@pytest.mark.parametrize("name", sorted(fx.KAT_EXPECTED))
def test_kat_reference_outputs(name):
    """Label map, split trace and centroid doubles of the reference run."""
    px, k = fx.kat_inputs()[name]
    fix = fx.load_json("kats.json")[name]
    out, ct = oracle_quant(px, k)
    assert [int(v) for v in out] == fix["out"]
    if k > 1:
        _, means, sizes, trace = oracle_cluster(px, k)
        assert trace.tolist() == fix["trace"]
        check_means(means, sizes, np.array([[float.fromhex(v) for v in m] for m in fix["means"]]))


def test_fixture_kats_agree_with_xctest():
    kats = fx.load_json("kats.json")
    for name, exp in fx.KAT_EXPECTED.items():
        assert kats[name]["ct"] == exp


def test_cases():
    cases = fx.load_json("cases.json")
    arrs = fx.load_npz("cases.npz")
    assert len(cases) > 50
    for i, c in enumerate(cases):
        spec = c["spec"]
        px = fx.make_case(spec)
        out, ct = oracle_quant(px, spec["k"])
        assert "%016x" % fx.fnv(out) == c["out_fnv"], spec
        assert [int(v) for v in ct] == c["ct"], spec
        if spec["k"] > 1:
            _, means, sizes, trace = oracle_cluster(px, spec["k"])
            assert np.array_equal(trace, arrs["trace_%d" % i]), spec
            check_means(means, sizes, arrs["means_%d" % i])


def test_c1_label_map():
    z = fx.load_npz("c1.npz")
    out, ct = oracle_quant(fx.xorshift(256 * 256), 16)
    assert np.array_equal(ct, z["ct"])
    assert np.array_equal(z["ct"][z["labels"]], out)


@pytest.mark.parametrize("key", ["512x512_k64", "1920x1080_k256"])
def test_big(key):
    c = fx.load_json("big.json")[key]
    arrs = fx.load_npz("big.npz")
    px = fx.xorshift(c["w"] * c["h"])
    out, ct = oracle_quant(px, c["k"])
    assert [int(v) for v in ct] == c["ct"]
    assert "%016x" % fx.fnv(out) == c["out_fnv"]
    _, means, sizes, trace = oracle_cluster(px, c["k"])
    assert np.array_equal(trace, arrs["trace_" + key])
    check_means(means, sizes, arrs["means_" + key])


def test_big_split_sizes_uniform():
    """uniform inputs split log2(K)*N points in total."""
    big = fx.load_json("big.json")
    for key, c in big.items():
        n = c["w"] * c["h"]
        assert c["sum_split_sizes"] == int(np.log2(c["k"])) * n, key


@pytest.mark.parametrize("name", ["batman", "cookie"])
def test_sample_images(name):
    fix = fx.load_json("png.json")[name]
    px, w, h = fx.load_png_u32(fx.os.path.join(fx.GOLDEN, "png", name + ".png"))
    assert (w, h) == (fix["w"], fix["h"])
    assert "%016x" % fx.fnv(px) == fix["px_fnv"]
    assert len(np.unique(px)) == fix["unique"]
    for k in (4, 16):
        out, ct = oracle_quant(px, k)
        assert [int(v) for v in ct] == fix["k%d" % k]["ct"]
        assert "%016x" % fx.fnv(out) == fix["k%d" % k]["out_fnv"]


def test_map_palettes():
    px = fx.xorshift(1 << 16, seed=fx.SEED + 7)
    for c in fx.load_json("map.json"):
        pal = fx.make_palette(c["spec"])
        out = oracle_map(px, pal)
        assert "%016x" % fx.fnv(out) == c["out_fnv"], c["spec"]
        assert [int(v) for v in out[:64]] == c["first"]


def test_map_equals_argmin_distance_rank():
    """The identity the GPU map kernel relies on: map_colors_mps (the walk) ==
    argmin over palette entries of (squared distance, MPS visit rank), on
    random, equal-sum (sort-tie) and duplicate-heavy palettes."""
    rng = np.random.default_rng(7)
    px = np.concatenate([fx.xorshift(20000, seed=3),
                         (fx.xorshift(5000, seed=4) & 0xC0C0C0)])   # tie-heavy pixels
    for trial in range(15):
        k = int(rng.integers(1, 300))
        if trial % 3 == 0:
            pal = rng.integers(0, 1 << 24, k, dtype=np.uint32)
        elif trial % 3 == 1:
            pal = (rng.integers(0, 6, k, dtype=np.uint32) * 0x333333) ^ rng.integers(0, 3, k, dtype=np.uint32)
        else:
            pal = fx.make_palette({"k": k, "kind": "sametsum", "seed": trial})
        want = oracle_map(px, pal)
        got = np.zeros(len(px), np.uint32)
        fx.oracle().dqo_map_argmin(fx.vp(px), ctypes.c_uint32(len(px)), fx.vp(got), fx.vp(pal),
                                   ctypes.c_int(len(pal)))
        assert np.array_equal(got, want), trial


def oracle_quant_weighted(px, k):
    orc = fx.oracle()
    px = np.ascontiguousarray(px, np.uint32)
    out = np.zeros(len(px), np.uint32)
    ct = np.zeros(k, np.uint32)
    kk = ctypes.c_uint32(k)
    orc.dqo_quant_recurse_weighted(ctypes.c_uint32(len(px)), fx.vp(px), fx.vp(out), ctypes.byref(kk),
                                   fx.vp(ct))
    return out, ct[:kk.value]


def oracle_cluster_weighted(px, k, max_iters=10):
    orc = fx.oracle()
    px = np.ascontiguousarray(px, np.uint32)
    col = np.zeros(len(px), np.uint32)
    w = np.zeros(len(px), np.float64)
    u = orc.dqo_color_table(ctypes.c_uint32(len(px)), fx.vp(px), fx.vp(col), fx.vp(w))
    ct = np.zeros(k, np.uint32)
    kk = ctypes.c_uint32(k)
    means = np.zeros((k, 3), np.float64)
    sizes = np.zeros(k, np.int64)
    trace = np.zeros((max(k - 1, 1), 4), np.int64)
    orc.dqo_cluster_weighted(ctypes.c_uint32(u), fx.vp(col), fx.vp(w), ctypes.byref(kk), fx.vp(ct),
                             ctypes.c_int(max_iters), fx.vp(means), fx.vp(sizes), fx.vp(trace))
    return ct[:kk.value], means, sizes, trace[:k - 1]


def test_weighted_fixtures():
    """allPixelsUnique=0 (every live app call site): the oracle's weighted
    restatement (calc_color_table order + ordered FP64 folds) against the
    reference's outputs -- the synthetic fixtures, the sample images, and the
    duplicate-heavy / image-region cases of weighted2.json."""
    for c in fx.load_json("weighted.json"):
        s = c["spec"]
        px = fx.xorshift(s["w"] * s["h"]) if s.get("kind") == "xorshift" else fx.make_case(s)
        out, ct = oracle_quant_weighted(px, s["k"])
        assert [int(v) for v in ct] == c["ct"], s
        assert "%016x" % fx.fnv(out) == c["out_fnv"], s
    for name, fix in fx.load_json("png.json").items():
        px = fx.load_png_u32(fx.os.path.join(fx.GOLDEN, "png", name + ".png"))[0]
        for k in (4, 16):
            out, ct = oracle_quant_weighted(px, k)
            assert [int(v) for v in ct] == fix["k%d_weighted" % k]["ct"], (name, k)
            assert "%016x" % fx.fnv(out) == fix["k%d_weighted" % k]["out_fnv"], (name, k)


def test_weighted2_fixtures():
    cases = fx.load_json("weighted2.json")
    arrs = fx.load_npz("weighted2.npz")
    assert sum(c["uw_differs"] for c in cases) >= 20   # the fixture set exercises the difference
    for i, c in enumerate(cases):
        s = c["spec"]
        px = fx.make_weighted_case(s)
        assert len(px) == c["n_px"]
        out, ct = oracle_quant_weighted(px, s["k"])
        assert [int(v) for v in ct] == c["ct"], (i, s)
        assert "%016x" % fx.fnv(out) == c["out_fnv"], (i, s)
        if s["k"] > 1 and i % 4 == 0:
            _, means, sizes, trace = oracle_cluster_weighted(px, s["k"])
            assert np.array_equal(trace, arrs["trace_%d" % i]), (i, s)
            ref = arrs["means_%d" % i]
            filled = ~np.isnan(ref[:, 0])
            assert np.array_equal(filled, sizes > 0)
            assert np.array_equal(means[filled].view(np.uint64), ref[filled].view(np.uint64)), (i, s)


def test_color_table_matches_reference():
    """dqo_color_table against the reference's calc_color_table outputs."""
    for c in fx.load_json("utils.json")["calc_color_table"]:
        px = fx.make_case(c["spec"])
        col = np.zeros(len(px), np.uint32)
        w = np.zeros(len(px), np.float64)
        u = fx.oracle().dqo_color_table(ctypes.c_uint32(len(px)), fx.vp(px), fx.vp(col), fx.vp(w))
        assert u == c["num_colors"]
        assert [int(v) for v in col[:u]] == c["colors"]
        assert [float(x).hex() for x in w[:u]] == c["weights"]


def oracle_varpart(px, spec):
    """dqo_quant_varpart: quant_varpart_fast restated for any (num_bits, dec_factor)."""
    k = spec["k"]
    px = np.ascontiguousarray(px, np.uint32)
    ct = np.zeros(k, np.uint32)
    kk = ctypes.c_uint32(k)
    means = np.zeros((k, 3), np.float64)
    sizes = np.zeros(k, np.int64)
    trace = np.zeros((max(k - 1, 1), 4), np.int64)
    rc = fx.oracle().dqo_quant_varpart(
        ctypes.c_uint32(len(px)), fx.vp(px), ctypes.c_uint32(spec["rows"]), ctypes.c_uint32(spec["cols"]),
        ctypes.byref(kk), fx.vp(ct), ctypes.c_int(spec["num_bits"]), ctypes.c_int(spec["dec"]),
        ctypes.c_int(spec["max_iters"]), ctypes.c_int(spec["uniq"]), fx.vp(means), fx.vp(sizes), fx.vp(trace))
    assert rc >= 0, rc
    return ct[:kk.value], means, sizes, trace[:k - 1]


def test_varpart_fixtures():
    """cut_bits / decimation: the oracle's quant_varpart_fast
    restatement against the reference's colortables, split traces and double
    centroids for num_bits 1..8 x dec_factor {1,2,3,5} x allPixelsUnique."""
    cases = fx.load_json("varpart.json")
    arrs = fx.load_npz("varpart.npz")
    assert len(cases) == 62
    for i, c in enumerate(cases):
        s = c["spec"]
        px = fx.make_varpart_case(s)
        assert len(px) == c["n_px"]
        ct, means, sizes, trace = oracle_varpart(px, s)
        assert [int(v) for v in ct] == c["ct"], (i, s)
        if s["k"] > 1:
            assert np.array_equal(trace, arrs["trace_%d" % i]), (i, s)
        ref = arrs["means_%d" % i]
        filled = ~np.isnan(ref[:, 0])
        if s["k"] > 1:
            assert np.array_equal(filled, sizes > 0), (i, s)
            assert np.array_equal(means[filled].view(np.uint64), ref[filled].view(np.uint64)), (i, s)


def test_cut_bits_restatement():
    """dqo_cut_bits against the reference's whole-word form (DivQuantUni.cpp:63-77)
    and per-channel form (:78-93), restated in numpy."""
    px = fx.xorshift(5000, seed=77) | np.uint32(0xAB000000)
    for nb in range(1, 9):
        sh = 8 - nb
        bm = (0xFF >> sh) << sh
        want = ((px & np.uint32((bm << 16) | (bm << 8) | bm)) >> np.uint32(sh)).astype(np.uint32)
        got = np.zeros_like(px)
        fx.oracle().dqo_cut_bits(fx.vp(px), ctypes.c_uint32(len(px)), fx.vp(got), nb, nb, nb)
        assert np.array_equal(got, want), nb
    got = np.zeros_like(px)
    fx.oracle().dqo_cut_bits(fx.vp(px), ctypes.c_uint32(len(px)), fx.vp(got), 3, 5, 7)
    want = (((px >> 16) & 0xFF) >> 5) << 16 | (((px >> 8) & 0xFF) >> 3) << 8 | ((px & 0xFF) >> 1)
    assert np.array_equal(got, want.astype(np.uint32))
