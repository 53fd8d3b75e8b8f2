"""GPU parity tests: the HIP path (through the C ABI of libdivquant_hip.so)
against the reference's own outputs (tests/golden/, generated from the
unmodified reference by tests/golden/make_golden.py) and against the CPU
oracle on seeded inputs.

Bar (BASELINE.json north star): output colours (the label map) and the
colortable bit-exact; the double centroids mean[ic] within 1e-5 -- they are
in fact asserted bit-exact here.
"""
import ctypes

import numpy as np
import pytest

import dq_fixtures as fx

pytestmark = pytest.mark.gpu


def _oracle_cluster(px, k, max_iters=10):
    orc = fx.oracle()
    ct = np.zeros(k, np.uint32)
    kk = ctypes.c_uint32(k)
    means = np.zeros((k, 3), np.float64)
    sizes = np.zeros(k, np.int64)
    trace = np.zeros((max(k - 1, 1), 4), np.int64)
    orc.dqo_cluster(ctypes.c_uint32(len(px)), fx.vp(px), ctypes.byref(kk), fx.vp(ct),
                    ctypes.c_int(max_iters), fx.vp(means), fx.vp(sizes), fx.vp(trace))
    return ct[:kk.value], means, sizes, trace[:k - 1]


def _quant_dev(gpu, px, k):
    import torch
    t_in = torch.from_numpy(np.ascontiguousarray(px, np.uint32).view(np.int32)).to("cuda:0")
    t_out = torch.empty_like(t_in)
    ct, empty = gpu.quant_device(t_in, t_out, k)
    torch.cuda.synchronize()
    return t_out.cpu().numpy().view(np.uint32), ct


def _check_centroids(gpu, k, ref_means):
    """Reference mean[ic] is recorded only for non-empty clusters (NaN elsewhere)."""
    means, sizes = gpu.last_centroids(k)
    filled = ~np.isnan(ref_means[:, 0])
    assert np.array_equal(filled, sizes > 0)
    assert np.array_equal(means[filled].view(np.uint64), ref_means[filled].view(np.uint64)), \
        np.abs(means[filled] - ref_means[filled]).max()
    assert np.all(np.abs(means[filled] - ref_means[filled]) <= 1e-5)


# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name", sorted(fx.KAT_EXPECTED))
def test_kat_quant_recurse(gpu, name):
    """Test/DivQuantTest.m known answers through the reference-named C entry."""
    px, k = fx.kat_inputs()[name]
    out, ct = gpu.quant_recurse(px, k, 1)
    assert [int(v) for v in ct] == fx.KAT_EXPECTED[name]
    fix = fx.load_json("kats.json")[name]
    assert [int(v) for v in out] == fix["out"]


@pytest.mark.parametrize("name", sorted(fx.KAT_EXPECTED))
def test_kat_trace_and_centroids(gpu, name):
    px, k = fx.kat_inputs()[name]
    out, ct = _quant_dev(gpu, px, k)
    fix = fx.load_json("kats.json")[name]
    assert [int(v) for v in ct] == fix["ct"]
    if k > 1:
        assert gpu.last_trace(k).tolist() == fix["trace"]
        ref_means = np.array([[float.fromhex(v) for v in m] for m in fix["means"]])
        _check_centroids(gpu, k, ref_means)


def test_cases(gpu):
    """Small seeded inputs: uniform, tie-heavy, grey, clustered, coarse, top-byte garbage;
    N from 1 to 70001, K from 1 to 1024 (K > N gives empty clusters)."""
    cases = fx.load_json("cases.json")
    arrs = fx.load_npz("cases.npz")
    bad = []
    for i, c in enumerate(cases):
        spec = c["spec"]
        px = fx.make_case(spec)
        out, ct = _quant_dev(gpu, px, spec["k"])
        if "%016x" % fx.fnv(out) != c["out_fnv"] or [int(v) for v in ct] != c["ct"]:
            bad.append((i, spec))
            continue
        if spec["k"] > 1:
            tr = gpu.last_trace(spec["k"])
            if not np.array_equal(tr, arrs["trace_%d" % i]):
                bad.append((i, spec, "trace"))
            _check_centroids(gpu, spec["k"], arrs["means_%d" % i])
    assert not bad, bad


def test_c1_full_label_map(gpu):
    """C1 256x256 K=16: the whole label map against the reference's."""
    z = fx.load_npz("c1.npz")
    px = fx.xorshift(256 * 256)
    out, ct = _quant_dev(gpu, px, 16)
    assert np.array_equal(ct, z["ct"])
    assert np.array_equal(z["ct"][z["labels"]], out)
    assert np.array_equal(gpu.last_trace(16), z["trace"])
    _check_centroids(gpu, 16, z["means"])


@pytest.mark.parametrize("key", ["512x512_k64", "1920x1080_k256", "1920x1080_k1024",
                                 "3840x2160_k256", "4096x4096_k1024"])
def test_big_configs(gpu, key):
    big = fx.load_json("big.json")
    if key not in big:
        pytest.skip("fixture not generated")
    c = big[key]
    arrs = fx.load_npz("big.npz")
    px = fx.xorshift(c["w"] * c["h"])
    out, ct = _quant_dev(gpu, px, c["k"])
    assert [int(v) for v in ct] == c["ct"]
    assert "%016x" % fx.fnv(out) == c["out_fnv"]
    assert np.array_equal(gpu.last_trace(c["k"]), arrs["trace_" + key])
    _check_centroids(gpu, c["k"], arrs["means_" + key])


@pytest.mark.parametrize("name", ["batman", "cookie"])
@pytest.mark.parametrize("k", [4, 16, 125, 256])
def test_sample_images(gpu, name, k):
    """The reference's own sample images (tests/*/...png), both allPixelsUnique values."""
    fix = fx.load_json("png.json")[name]
    px, w, h = fx.load_png_u32(fx.os.path.join(fx.GOLDEN, "png", name + ".png"))
    assert "%016x" % fx.fnv(px) == fix["px_fnv"]
    for uniq, key in ((1, "k%d" % k), (0, "k%d_weighted" % k)):
        out, ct = gpu.quant_recurse(px, k, uniq)
        assert [int(v) for v in ct] == fix[key]["ct"], key
        assert "%016x" % fx.fnv(out) == fix[key]["out_fnv"], key
    arrs = fx.load_npz("png.npz")
    _quant_dev(gpu, px, k)
    assert np.array_equal(gpu.last_trace(k), arrs["trace_%s_k%d" % (name, k)])
    _check_centroids(gpu, k, arrs["means_%s_k%d" % (name, k)])


def test_map_colors_mps(gpu):
    """map_colors_mps alone: random, equal-sum (sort-tie), duplicate, grey and the
    125-colour getSubdividedColors palettes."""
    px = fx.xorshift(1 << 16, seed=fx.SEED + 7)
    bad = []
    for c in fx.load_json("map.json"):
        pal = fx.make_palette(c["spec"])
        out = gpu.map_colors_mps(px, pal)
        if "%016x" % fx.fnv(out) != c["out_fnv"]:
            bad.append(c["spec"])
    assert not bad, bad


@pytest.fixture(params=[True, False], ids=["wsmall", "rounds"])
def wpath(gpu, request):
    """Both weighted paths: small inputs in one launch (dq_wsmall.hip) and the
    multi-kernel rounds (dq_weighted.hip) they would otherwise take."""
    gpu.set_wsmall(request.param)
    yield request.param
    gpu.set_wsmall(True)


def test_weighted_path(gpu, wpath):
    """allPixelsUnique=0 (every live app call site, ClusteringSegmentation.cpp:1803):
    the reference's weighted outputs -- calc_color_table order + ordered FP64
    folds -- on the synthetic fixtures and on the 352 duplicate-heavy /
    image-region cases of weighted2.json (55 of which the uniform-weight
    algorithm gets wrong)."""
    bad = []
    for c in fx.load_json("weighted.json"):
        s = c["spec"]
        px = fx.xorshift(s["w"] * s["h"]) if s.get("kind") == "xorshift" else fx.make_case(s)
        out, ct = gpu.quant_recurse(px, s["k"], 0)
        if [int(v) for v in ct] != c["ct"] or "%016x" % fx.fnv(out) != c["out_fnv"]:
            bad.append(s)
    cases = fx.load_json("weighted2.json")
    for i, c in enumerate(cases):
        s = c["spec"]
        px = fx.make_weighted_case(s)
        out, ct = gpu.quant_recurse(px, s["k"], 0)
        if [int(v) for v in ct] != c["ct"] or "%016x" % fx.fnv(out) != c["out_fnv"]:
            bad.append((i, s, c["uw_differs"]))
    assert not bad, bad


def test_weighted_trace_and_centroids(gpu, wpath):
    """The weighted path's split trace (sizes in unique colours) and centroid
    doubles against the reference's (instrumented build, weighted2.npz)."""
    import torch
    cases = fx.load_json("weighted2.json")
    arrs = fx.load_npz("weighted2.npz")
    for i, c in enumerate(cases):
        s = c["spec"]
        if s["k"] == 1 or i % 3:
            continue
        px = fx.make_weighted_case(s)
        t = torch.from_numpy(px.view(np.int32)).to("cuda:0")
        o = torch.empty_like(t)
        ct, _ = gpu.quant_device(t, o, s["k"], all_pixels_unique=0)
        torch.cuda.synchronize()
        assert [int(v) for v in ct] == c["ct"], (i, s)
        assert "%016x" % fx.fnv(o.cpu().numpy().view(np.uint32)) == c["out_fnv"], (i, s)
        assert np.array_equal(gpu.last_trace(s["k"]), arrs["trace_%d" % i]), (i, s)
        _check_centroids(gpu, s["k"], arrs["means_%d" % i])


def test_weighted_vs_oracle_sweep(gpu, wpath):
    """Fresh seeded duplicate-heavy inputs against the oracle's weighted restatement."""
    rng = np.random.default_rng(777)
    for trial in range(40):
        n = int(rng.integers(1, 60000))
        k = int(rng.choice([1, 2, 3, 4, 7, 16, 64, 256]))
        ncol = int(rng.integers(1, 3000))
        pal = rng.integers(0, 1 << 24, ncol, dtype=np.uint32)
        px = pal[rng.integers(0, ncol, n)]
        if trial % 3 == 0:
            px &= 0xE0E0E0
        out, ct = gpu.quant_recurse(px, k, 0)
        ref_out = np.zeros(n, np.uint32)
        ref_ct = np.zeros(k, np.uint32)
        kk = ctypes.c_uint32(k)
        fx.oracle().dqo_quant_recurse_weighted(ctypes.c_uint32(n), fx.vp(px), fx.vp(ref_out), ctypes.byref(kk),
                                               fx.vp(ref_ct))
        assert np.array_equal(ct, ref_ct[:kk.value]), (trial, n, k)
        assert np.array_equal(out, ref_out), (trial, n, k)
    # quant_varpart_fast(allPixelsUnique=0): the table before the dedup
    px = fx.make_weighted_case(fx.weighted_case_specs()[5])
    ct = gpu.quant_varpart_fast(px, 8, all_pixels_unique=0)
    col = np.zeros(len(px), np.uint32)
    w = np.zeros(len(px), np.float64)
    u = fx.oracle().dqo_color_table(ctypes.c_uint32(len(px)), fx.vp(px), fx.vp(col), fx.vp(w))
    rct = np.zeros(8, np.uint32)
    kk = ctypes.c_uint32(8)
    fx.oracle().dqo_cluster_weighted(ctypes.c_uint32(u), fx.vp(col), fx.vp(w), ctypes.byref(kk), fx.vp(rct),
                                     ctypes.c_int(10), None, None, None)
    assert np.array_equal(ct, rct[:kk.value])


@pytest.mark.parametrize("n,mask,k", [(300000, 0xFFFFFF, 4), (600000, 0xFEFEFE, 16), (1 << 20, 0xFCFCFC, 64)])
def test_weighted_multi_tile_vs_oracle(gpu, n, mask, k):
    """The weighted path's exact parallel folds on nodes of many tiles (10^5 -
    10^6 unique colours: every pass's folds run over hundreds of 4096-point
    tiles, with binade crossings inside tiles and across them) against the
    oracle's sequential folds: colortable, output and centroid doubles."""
    px = fx.xorshift(n, seed=fx.SEED + n) & mask
    out, ct = gpu.quant_recurse(px, k, 0)
    ref_out = np.zeros(n, np.uint32)
    ref_ct = np.zeros(k, np.uint32)
    kk = ctypes.c_uint32(k)
    fx.oracle().dqo_quant_recurse_weighted(ctypes.c_uint32(n), fx.vp(px), fx.vp(ref_out), ctypes.byref(kk),
                                           fx.vp(ref_ct))
    assert np.array_equal(ct, ref_ct[:kk.value]), (n, k)
    assert np.array_equal(out, ref_out), (n, k)
    # (tiles folded summand by summand: the fallback, not the rule -- none
    # on these frames in the CPU model, tests/test_exact_fold.py)
    assert gpu.last_seq_tiles() <= gpu.last_rounds(), gpu.last_seq_tiles()


def test_oracle_random_sweep(gpu):
    """Fresh seeded inputs (not in any fixture) against the CPU oracle."""
    rng = np.random.default_rng(12345)
    for trial in range(24):
        n = int(rng.integers(1, 300000))
        k = int(rng.choice([2, 3, 8, 16, 64, 100, 256, 512, 1024]))
        mode = trial % 3
        if mode == 0:
            px = rng.integers(0, 1 << 24, n, dtype=np.uint32)
        elif mode == 1:
            px = (rng.integers(0, 6, n, dtype=np.uint32) * 0x2A2A2A) ^ rng.integers(0, 4, n, dtype=np.uint32)
        else:
            px = rng.integers(0, 1 << 24, n, dtype=np.uint32) & 0xF0C0F0
        out, ct = _quant_dev(gpu, px, k)
        ref_ct, ref_means, ref_sizes, ref_trace = _oracle_cluster(px, k)
        orc_out = np.zeros(n, np.uint32)
        kk = ctypes.c_uint32(k)
        ct2 = np.zeros(k, np.uint32)
        fx.oracle().dqo_quant_recurse(ctypes.c_uint32(n), fx.vp(px), fx.vp(orc_out), ctypes.byref(kk), fx.vp(ct2))
        assert np.array_equal(ct, ct2[:kk.value]), (trial, n, k)
        assert np.array_equal(out, orc_out), (trial, n, k)
        assert np.array_equal(gpu.last_trace(k), ref_trace), (trial, n, k)


def test_host_and_device_entry_points_agree(gpu):
    px = fx.xorshift(200003, seed=99)
    a_out, a_ct = gpu.quant_recurse(px, 128, 1)
    b_out, b_ct = _quant_dev(gpu, px, 128)
    assert np.array_equal(a_ct, b_ct) and np.array_equal(a_out, b_out)
    c_out = gpu.map_colors_mps(px, a_ct)
    assert np.array_equal(c_out, a_out)


def test_repeatable(gpu):
    px = fx.xorshift(1 << 20, seed=5)
    r = [_quant_dev(gpu, px, 256) for _ in range(3)]
    for out, ct in r[1:]:
        assert np.array_equal(out, r[0][0]) and np.array_equal(ct, r[0][1])


@pytest.mark.parametrize("max_iters", [1, 2, 3, 5, 10, 17])
def test_max_iters_vs_oracle(gpu, max_iters):
    """The iteration count is part of the algorithm (:613): every max_iters,
    with fixed-point finalisation on, against the oracle's full loop."""
    import torch
    for seed, (n, k) in enumerate([(70001, 16), (250000, 256), (9000, 1024)]):
        px = fx.xorshift(n, seed=1000 + seed)
        if seed == 2:
            px &= 0xE0E0E0
        t = torch.from_numpy(px.view(np.int32)).to("cuda:0")
        ct, _ = gpu.cluster_device(t, k, max_iters=max_iters)
        ref_ct, ref_means, ref_sizes, ref_trace = _oracle_cluster(px, k, max_iters=max_iters)
        assert np.array_equal(ct, ref_ct), (max_iters, n, k)
        assert np.array_equal(gpu.last_trace(k), ref_trace), (max_iters, n, k)
        means, sizes = gpu.last_centroids(k)
        filled = sizes > 0
        assert np.array_equal(means[filled].view(np.uint64), ref_means[filled].view(np.uint64))


def test_fixed_point_finalisation_is_exact(gpu):
    """Finalising a split when its 2-means pass reproduces the previous pass's
    exact sums gives the same outputs as running every iteration, and sweeps
    fewer points (uniform data: the axis-mean cut is already the bisector)."""
    cases = [fx.xorshift(1 << 20, seed=21), fx.xorshift(300000, seed=22) & 0xF8FCF8]
    for name in ("batman", "cookie"):
        cases.append(fx.load_png_u32(fx.os.path.join(fx.GOLDEN, "png", name + ".png"))[0])
    try:
        for px in cases:
            for k in (16, 256):
                gpu.set_fixed_point(False)
                a_out, a_ct = _quant_dev(gpu, px, k)
                a_trace = gpu.last_trace(k)
                a_means, _ = gpu.last_centroids(k)
                full_swept, full = gpu.last_points_swept(), gpu.last_points_full()
                assert full_swept == full
                gpu.set_fixed_point(True)
                for plan in (False, True):   # host-planned rounds only: the same nodes
                    gpu.set_planned_rounds(plan)
                    b_out, b_ct = _quant_dev(gpu, px, k)
                    assert np.array_equal(a_out, b_out) and np.array_equal(a_ct, b_ct)
                    assert np.array_equal(gpu.last_trace(k), a_trace)
                    b_means, _ = gpu.last_centroids(k)
                    assert np.array_equal(np.nan_to_num(a_means).view(np.uint64),
                                          np.nan_to_num(b_means).view(np.uint64))
                    if not plan:
                        assert gpu.last_points_full() == full
                        assert gpu.last_points_swept() < full
    finally:
        gpu.set_fixed_point(True)
        gpu.set_planned_rounds(True)


@pytest.mark.parametrize("key", ["1920x1080_k256", "512x512_k64"])
def test_one_launch_kmeans_loops(gpu, key):
    """Rounds of small records run every 2-means iteration in one
    kloop_kernel launch per round: same exact integer sums and
    the same FP64 update as the kpass_kernel chain, so the colortable, output,
    split trace, centroid doubles -- and the records, partition cursors and
    results later rounds read -- are the reference's either way.  C2's last
    rounds and the batman PNG (a later host round partitions nodes the loop
    finalised) must take the loop."""
    big = fx.load_json("big.json")
    if key not in big:
        pytest.skip("fixture not generated")
    c = big[key]
    arrs = fx.load_npz("big.npz")
    px = fx.xorshift(c["w"] * c["h"])
    bat = fx.load_png_u32(fx.os.path.join(fx.GOLDEN, "png", "batman.png"))[0]
    fix = fx.load_json("png.json")["batman"]
    try:
        gpu.set_persist(False)
        for lmax in (49152, 0):
            gpu.set_loop_max(lmax)
            out, ct = _quant_dev(gpu, px, c["k"])
            assert (gpu.last_loop_rounds() > 0) == (lmax > 0)
            assert gpu.last_persist_rounds() == 0
            assert [int(v) for v in ct] == c["ct"]
            assert "%016x" % fx.fnv(out) == c["out_fnv"]
            assert np.array_equal(gpu.last_trace(c["k"]), arrs["trace_" + key])
            _check_centroids(gpu, c["k"], arrs["means_" + key])
            for k in (16, 125, 256):
                out, ct = _quant_dev(gpu, bat, k)
                assert [int(v) for v in ct] == fix["k%d" % k]["ct"], (lmax, k)
                assert "%016x" % fx.fnv(out) == fix["k%d" % k]["out_fnv"], (lmax, k)
    finally:
        gpu.set_loop_max(49152)
        gpu.set_persist(True)


@pytest.mark.parametrize("key", ["3840x2160_k256", "1920x1080_k256", "4096x4096_k1024"])
def test_persistent_kmeans_rounds(gpu, key):
    """Rounds of larger records run every 2-means iteration in one
    kpersist_kernel launch: the records' workgroups meet per
    iteration on device counters, and the last arriver runs the same FP64
    update on the same exact sums as kpass_kernel.  With and without it (and
    with kloop off, so kpersist takes kloop's rounds too): the reference's
    colortable, output, split trace and centroid doubles; C3's frame must
    take it."""
    big = fx.load_json("big.json")
    if key not in big:
        pytest.skip("fixture not generated")
    c = big[key]
    arrs = fx.load_npz("big.npz")
    px = fx.xorshift(c["w"] * c["h"])
    try:
        for persist, lmax in ((True, 49152), (True, 0), (False, 49152)):
            gpu.set_persist(persist)
            gpu.set_loop_max(lmax)
            out, ct = _quant_dev(gpu, px, c["k"])
            if key == "3840x2160_k256" or not persist:
                assert (gpu.last_persist_rounds() > 0) == persist, (persist, lmax)
            assert [int(v) for v in ct] == c["ct"], (persist, lmax)
            assert "%016x" % fx.fnv(out) == c["out_fnv"], (persist, lmax)
            assert np.array_equal(gpu.last_trace(c["k"]), arrs["trace_" + key])
            _check_centroids(gpu, c["k"], arrs["means_" + key])
    finally:
        gpu.set_loop_max(49152)
        gpu.set_persist(True)


def test_kmeans_loop_at_max_len_near_white(gpu):
    """kloop_kernel at its largest record (kLoopMaxLen = 983008 points): a
    data wave then sums 65536 points, and near-white points (255^2-sized
    squares) bring its u32 sums of squares to within 5 % of 2^32.  The root
    splits this frame exactly in half (R < 248 | R >= 248), so the next round
    holds two records of exactly kLoopMaxLen points, unproven at their split
    (G, B and R-within-half spread alike), which the loop must run.  Parity
    against the oracle's exact sums."""
    import ctypes
    lmax = 61440 * 16 - 32
    rng = np.random.default_rng(2024)
    n2 = lmax
    lo = (rng.integers(240, 248, n2, dtype=np.uint32) << 16)
    hi = (rng.integers(248, 256, n2, dtype=np.uint32) << 16)
    r = np.concatenate([lo, hi])
    gb = (rng.integers(248, 256, 2 * n2, dtype=np.uint32) << 8) | rng.integers(248, 256, 2 * n2, dtype=np.uint32)
    px = r | gb
    px = px[rng.permutation(px.size)].astype(np.uint32)
    k = 8
    ref_out = np.zeros(px.size, np.uint32)
    ref_ct = np.zeros(k, np.uint32)
    kk = ctypes.c_uint32(k)
    fx.oracle().dqo_quant_recurse(ctypes.c_uint32(px.size), fx.vp(px), fx.vp(ref_out), ctypes.byref(kk),
                                  fx.vp(ref_ct))
    try:
        gpu.set_loop_max(lmax)
        out, ct = _quant_dev(gpu, px, k)
        loops = gpu.last_loop_rounds()
        assert np.array_equal(ct, ref_ct[:kk.value])
        assert np.array_equal(out, ref_out)
        assert loops > 0
        gpu.set_loop_max(lmax + 1000)   # (clamped to kLoopMaxLen)
        out, ct = _quant_dev(gpu, px, k)
        assert np.array_equal(ct, ref_ct[:kk.value]) and np.array_equal(out, ref_out)
    finally:
        gpu.set_loop_max(49152)


def test_repeated_runs_identical(gpu):
    """Run-to-run determinism under many fused 2-means launches (fixed points
    off: every node runs all its iterations through kpass_kernel's
    last-arriver epilogue).  A partial store still in flight when the record's
    last workgroup summed the partials once made repeated calls differ."""
    px = fx.load_png_u32(fx.os.path.join(fx.GOLDEN, "png", "batman.png"))[0]
    try:
        gpu.set_fixed_point(False)
        first = None
        for _ in range(4):
            out, ct = _quant_dev(gpu, px, 256)
            got = (out, np.asarray(ct), gpu.last_trace(256).copy())
            if first is None:
                first = got
                continue
            assert all(np.array_equal(x, y) for x, y in zip(got, first))
    finally:
        gpu.set_fixed_point(True)


def test_batch_over_lanes(gpu):
    """A batch of frames in one call is split over engine lanes (own stream,
    own host thread each): every frame bit-exact against the oracle, and the
    diagnostics report the batch's last frame."""
    import torch
    frames = [fx.xorshift(200000 + 1000 * i, seed=300 + i) for i in range(5)]
    frames[2] &= 0xF0F0F0
    t_in = [torch.from_numpy(p.view(np.int32)).to("cuda:0") for p in frames]
    t_out = [torch.empty_like(t) for t in t_in]
    cts, _ = gpu.quant_batch_device(t_in, t_out, 64)
    torch.cuda.synchronize()
    for px, t, ct in zip(frames, t_out, cts):
        orc_out = np.zeros(len(px), np.uint32)
        kk = ctypes.c_uint32(64)
        ct2 = np.zeros(64, np.uint32)
        fx.oracle().dqo_quant_recurse(ctypes.c_uint32(len(px)), fx.vp(px), fx.vp(orc_out),
                                      ctypes.byref(kk), fx.vp(ct2))
        assert np.array_equal(ct, ct2[:kk.value])
        assert np.array_equal(t.cpu().numpy().view(np.uint32), orc_out)
    ref_trace = _oracle_cluster(frames[-1], 64)[3]
    assert np.array_equal(gpu.last_trace(64), ref_trace)


@pytest.mark.parametrize("kind", ["cluster1024", "cluster256", "line512", "uniform1024"])
def test_map_dense_palettes(gpu, kind):
    """Palettes whose cells have many candidates (a tight cluster of entries:
    most cells overflow the inline slots or need the whole palette), against
    the oracle's literal map_colors_mps walk.  Exercises the map's overflow
    queue and its queue-full fallback."""
    rng = np.random.default_rng({"cluster1024": 1, "cluster256": 2, "line512": 3, "uniform1024": 4}[kind])
    if kind.startswith("cluster"):
        k = int(kind[7:])
        c = rng.integers(100, 116, (k, 3))
    elif kind == "line512":
        k = 512
        t = rng.integers(0, 256, k)
        c = np.stack([t, (t * 3) % 256, 255 - t], 1)
    else:
        k = 1024
        c = rng.integers(0, 256, (k, 3))
    pal = ((c[:, 0] << 16) | (c[:, 1] << 8) | c[:, 2]).astype(np.uint32)
    px = fx.xorshift(300007, seed=77)
    out = gpu.map_colors_mps(px, pal)
    ref = np.zeros_like(px)
    fx.oracle().dqo_map(fx.vp(px), ctypes.c_uint32(len(px)), fx.vp(ref), fx.vp(pal), ctypes.c_int(k))
    assert np.array_equal(out, ref)


def test_map_above_task_limit(gpu):
    """A map of more than 2^28 pixels (Engine::kMapTaskMax: map_lds_kernel's
    output buffer range) is split into tasks; every pixel, the ragged tail
    past the split included, is mapped (stores past the range were
    dropped).  Input: a 65536-pixel random block repeated, so the expected
    output is the oracle's map of the block, repeated."""
    import torch
    blk = fx.xorshift(1 << 16, seed=91)
    rng = np.random.default_rng(5)
    pal = rng.integers(0, 1 << 24, 200).astype(np.uint32)
    ref = np.zeros_like(blk)
    fx.oracle().dqo_map(fx.vp(blk), ctypes.c_uint32(len(blk)), fx.vp(ref), fx.vp(pal), ctypes.c_int(len(pal)))
    n = (1 << 28) + 1000
    reps = (n + len(blk) - 1) // len(blk)
    t_blk = torch.from_numpy(blk.view(np.int32)).to("cuda:0")
    t_in = t_blk.repeat(reps)[:n].contiguous()
    t_out = torch.full_like(t_in, -1)
    gpu.map_device(t_in, t_out, pal)
    torch.cuda.synchronize()
    t_ref = torch.from_numpy(ref.view(np.int32)).to("cuda:0")
    full = n // len(blk)
    assert bool((t_out[:full * len(blk)].view(full, -1) == t_ref).all())
    assert bool((t_out[full * len(blk):] == t_ref[:n - full * len(blk)]).all())
    del t_in, t_out
    torch.cuda.empty_cache()


def test_cpp_linkage_entry_points(gpu):
    """The C++-linkage symbols the reference's callers link against
    (DivQuantHeader.h:52-96): map_colors_mps (ClusteringSegmentation.cpp:408,
    :2434) and quant_varpart_fast (quant_util.cpp:60) called by their mangled
    names, against the reference's outputs."""
    L = gpu.lib()
    mcm = getattr(L, "_Z14map_colors_mpsPKjjPjS1_i")
    mcm.restype = None
    mcm.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    px = fx.xorshift(1 << 16, seed=fx.SEED + 7)
    for c in fx.load_json("map.json"):
        pal = fx.make_palette(c["spec"])
        out = np.zeros_like(px)
        mcm(fx.vp(px), len(px), fx.vp(out), fx.vp(pal), len(pal))
        assert "%016x" % fx.fnv(out) == c["out_fnv"], c["spec"]
    qvf = getattr(L, "_Z18quant_varpart_fastjPKjPjjjS1_S1_iiii")
    qvf.restype = None
    qvf.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    cases = fx.load_json("cases.json")
    for i, c in enumerate(cases[:40]):
        spec = c["spec"]
        px = fx.make_case(spec)
        tmp = np.zeros_like(px)
        k = ctypes.c_uint32(spec["k"])
        ct = np.zeros(spec["k"], np.uint32)
        qvf(len(px), fx.vp(px), fx.vp(tmp), 1, len(px), ctypes.cast(ctypes.pointer(k), ctypes.c_void_p),
            fx.vp(ct), 8, 1, 10, 1)
        # quant_varpart_fast's table is cluster-index order before the dedup of
        # quant_util.cpp:93-118: its first-occurrence dedup is the fixture's
        seen, dd = set(), []
        for v in ct[:k.value]:
            if int(v) not in seen:
                seen.add(int(v))
                dd.append(int(v))
        assert dd == c["ct"], (i, spec)


def test_varpart_cut_bits_decimation(gpu):
    """quant_varpart_fast's cut_bits / decimation paths (SURVEY 8f.4,
    DivQuantCluster.cpp:1130-1146) through the mangled C++ symbol, against
    the reference's colortables for num_bits 1..8 x dec_factor {1,2,3,5} x
    allPixelsUnique (62 cases, rows x cols frames with the numRows-stride
    walk); the device entry dq_hip_varpart_dev also against the reference's
    split traces and centroid doubles."""
    import torch
    L = gpu.lib()
    qvf = getattr(L, "_Z18quant_varpart_fastjPKjPjjjS1_S1_iiii")
    qvf.restype = None
    qvf.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    cases = fx.load_json("varpart.json")
    arrs = fx.load_npz("varpart.npz")
    for i, c in enumerate(cases):
        s = c["spec"]
        px = fx.make_varpart_case(s)
        tmp = np.zeros_like(px)
        k = ctypes.c_uint32(s["k"])
        ct = np.zeros(s["k"], np.uint32)
        qvf(len(px), fx.vp(px), fx.vp(tmp), s["rows"], s["cols"], ctypes.cast(ctypes.pointer(k), ctypes.c_void_p),
            fx.vp(ct), s["num_bits"], s["dec"], s["max_iters"], s["uniq"])
        assert [int(v) for v in ct[:k.value]] == c["ct"], (i, s)
        d = torch.from_numpy(px.view(np.int32)).cuda()
        k2 = ctypes.c_uint32(s["k"])
        ct2 = np.zeros(s["k"], np.uint32)
        rc = L.dq_hip_varpart_dev(0, d.data_ptr(), len(px), s["rows"], s["cols"],
                                  ctypes.byref(k2), fx.vp(ct2), s["num_bits"],
                                  s["dec"], s["max_iters"], s["uniq"], None)
        assert rc >= 0 and [int(v) for v in ct2[:k2.value]] == c["ct"], (i, s)
        if s["k"] > 1:
            means, sizes = gpu.last_centroids(s["k"])
            trace = gpu.last_trace(s["k"])
            assert np.array_equal(trace, arrs["trace_%d" % i]), (i, s)
            ref = arrs["means_%d" % i]
            filled = ~np.isnan(ref[:, 0])
            assert np.array_equal(filled, sizes > 0), (i, s)
            assert np.array_equal(means[filled].view(np.uint64), ref[filled].view(np.uint64)), (i, s)
    # a walk that would read past the input is refused (-2), not run
    d = torch.zeros(48 * 80, dtype=torch.int32, device="cuda")
    k3 = ctypes.c_uint32(4)
    ct3 = np.zeros(4, np.uint32)
    assert L.dq_hip_varpart_dev(0, d.data_ptr(), 48 * 80, 80, 48, ctypes.byref(k3),
                                fx.vp(ct3), 8, 1, 10, 0, None) == -2


def test_cut_bits_device(gpu):
    """dq_hip_cut_bits_dev against the oracle's cut_bits restatement (equal and
    per-channel bit counts, in place and out of place)."""
    import torch
    L = gpu.lib()
    px = fx.xorshift(1000003, seed=99) | np.uint32(0x5A000000)
    for nbr, nbg, nbb in [(8, 8, 8), (5, 5, 5), (1, 1, 1), (3, 6, 7), (8, 2, 4)]:
        want = np.zeros_like(px)
        fx.oracle().dqo_cut_bits(fx.vp(px), ctypes.c_uint32(len(px)), fx.vp(want), nbr, nbg, nbb)
        d = torch.from_numpy(px.view(np.int32)).cuda()
        o = torch.empty_like(d)
        assert L.dq_hip_cut_bits_dev(0, ctypes.c_void_p(d.data_ptr()), ctypes.c_uint32(len(px)),
                                     ctypes.c_void_p(o.data_ptr()), nbr, nbg, nbb, None) == 0
        torch.cuda.synchronize()
        assert np.array_equal(o.cpu().numpy().view(np.uint32), want), (nbr, nbg, nbb)
        assert L.dq_hip_cut_bits_dev(0, ctypes.c_void_p(d.data_ptr()), ctypes.c_uint32(len(px)),
                                     ctypes.c_void_p(d.data_ptr()), nbr, nbg, nbb, None) == 0
        torch.cuda.synchronize()
        assert np.array_equal(d.cpu().numpy().view(np.uint32), want), ("in place", nbr, nbg, nbb)


def test_planned_rounds_equal_host_rounds(gpu):
    """Device-planned (speculative) rounds against host-planned rounds only:
    identical colortables, label maps, traces and centroid doubles, on
    uniform, clustered, coarse and image inputs, single frames and a batch."""
    import torch
    cases = [(fx.xorshift(1 << 20, seed=31), 256), (fx.xorshift(500000, seed=32) & 0xF0E0F0, 64),
             (fx.make_case({"n": 70001, "k": 32, "kind": "clustered", "seed": 5}), 32),
             (fx.load_png_u32(fx.os.path.join(fx.GOLDEN, "png", "cookie.png"))[0], 125),
             (fx.xorshift(3000, seed=33), 1024)]
    try:
        for px, k in cases:
            res = []
            for plan in (False, True):
                gpu.set_planned_rounds(plan)
                out, ct = _quant_dev(gpu, px, k)
                m, _ = gpu.last_centroids(k)
                res.append((out, ct, gpu.last_trace(k), np.nan_to_num(m).view(np.uint64)))
            if len(px) == 1 << 20:
                assert gpu.last_planned_rounds() > 0
            for x, y in zip(res[0], res[1]):
                assert np.array_equal(x, y), (len(px), k)
        frames = [fx.xorshift(300000, seed=40 + i) for i in range(4)]
        frames[1] &= 0xF8F8F8
        t_in = [torch.from_numpy(p.view(np.int32)).to("cuda:0") for p in frames]
        outs = []
        for plan in (False, True):
            gpu.set_planned_rounds(plan)
            t_out = [torch.empty_like(t) for t in t_in]
            cts, _ = gpu.quant_batch_device(t_in, t_out, 128)
            torch.cuda.synchronize()
            outs.append(([t.cpu().numpy() for t in t_out], cts))
        for a, b in zip(outs[0][0], outs[1][0]):
            assert np.array_equal(a, b)
        for a, b in zip(outs[0][1], outs[1][1]):
            assert np.array_equal(a, b)
    finally:
        gpu.set_planned_rounds(True)
