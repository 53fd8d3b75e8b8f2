"""GPU parity at the BASELINE configs' full sizes (C4, C5).

The fixtures are the reference build's own outputs (tests/golden/make_golden.py
--only c4 / c5): C4's 64 distinct 4K frames (frame f = SURVEY 8c generator,
seed + f) and the 16384x16384 K=1024 tile.  Bar: colortable and the
whole-frame output hash bit-exact, split traces and centroid doubles exact.
"""
import numpy as np
import pytest

import dq_fixtures as fx

pytestmark = pytest.mark.gpu

W4, H4 = 3840, 2160


def _frames(ids):
    import torch
    return [torch.from_numpy(fx.xorshift(W4 * H4, seed=fx.SEED + f).view(np.int32)).to("cuda:0") for f in ids]


def _check_centroids(gpu, k, ref_means):
    means, sizes = gpu.last_centroids(k)
    filled = ~np.isnan(ref_means[:, 0])
    assert np.array_equal(filled, sizes > 0)
    assert np.array_equal(means[filled].view(np.uint64), ref_means[filled].view(np.uint64))


def test_c4_share_batch_default_lanes(gpu):
    """The bench's workload exactly: 8 distinct 4K frames, K=256, one batched
    call over the library's default engine lanes."""
    import torch
    fix = fx.load_json("c4.json")
    arrs = fx.load_npz("c4.npz")
    ids = list(range(8))
    t_in = _frames(ids)
    t_out = [torch.empty_like(t) for t in t_in]
    gpu.set_lanes(0)
    cts, _ = gpu.quant_batch_device(t_in, t_out, 256)
    torch.cuda.synchronize()
    for f, t, ct in zip(ids, t_out, cts):
        c = fix["f%02d" % f]
        assert [int(v) for v in ct] == c["ct"], f
        assert "%016x" % fx.fnv(t.cpu().numpy().view(np.uint32)) == c["out_fnv"], f
    # diagnostics: the batch's last frame
    assert np.array_equal(gpu.last_trace(256), arrs["trace_f07"])
    _check_centroids(gpu, 256, arrs["means_f07"])


def test_c4_share_repeatable(gpu):
    """The bench workload called 60 times over 1, 2 and 3 engine lanes: every
    call's colortables equal the reference's and every output equals the
    first (reference-checked) call's, bit for bit -- the device-planned
    rounds, lane overlap and fused 2-means epilogues leave no run-to-run
    differences."""
    import torch
    fix = fx.load_json("c4.json")
    t_in = _frames(range(8))
    t_out = [torch.empty_like(t) for t in t_in]
    ref = None
    try:
        for c in range(60):
            gpu.set_lanes(1 + c % 3)
            cts, _ = gpu.quant_batch_device(t_in, t_out, 256)
            torch.cuda.synchronize()
            for f in range(8):
                assert [int(v) for v in cts[f]] == fix["f%02d" % f]["ct"], (c, f)
            if ref is None:
                for f in range(8):
                    assert "%016x" % fx.fnv(t_out[f].cpu().numpy().view(np.uint32)) == fix["f%02d" % f]["out_fnv"]
                ref = [t.clone() for t in t_out]
            else:
                for f in range(8):
                    assert torch.equal(t_out[f], ref[f]), (c, f)
    finally:
        gpu.set_lanes(0)


def test_c4_frames_8_to_63_one_call(gpu):
    """The remaining 56 frames of C4 (the other ranks' shares) in one call."""
    import torch
    fix = fx.load_json("c4.json")
    ids = list(range(8, 64))
    bad = []
    for chunk in (ids[:28], ids[28:]):
        t_in = _frames(chunk)
        t_out = [torch.empty_like(t) for t in t_in]
        cts, _ = gpu.quant_batch_device(t_in, t_out, 256)
        torch.cuda.synchronize()
        for f, t, ct in zip(chunk, t_out, cts):
            c = fix["f%02d" % f]
            if [int(v) for v in ct] != c["ct"] or \
                    "%016x" % fx.fnv(t.cpu().numpy().view(np.uint32)) != c["out_fnv"]:
                bad.append(f)
        del t_in, t_out
    assert not bad, bad


def test_c4_rowtile_batch_8_shards(gpu):
    """C4's row-tile variant: 8 frames in one call, each split into 8 row
    shards (the exact arithmetic of 8-GPU row sharding, on one GPU)."""
    import torch
    fix = fx.load_json("c4.json")
    ids = list(range(8))
    t_in = _frames(ids)
    t_out = [torch.empty_like(t) for t in t_in]
    cts, _ = gpu.quant_rows_device(t_in, t_out, 256, widths=[W4] * 8, nshard=8)
    torch.cuda.synchronize()
    for f, t, ct in zip(ids, t_out, cts):
        c = fix["f%02d" % f]
        out = t.cpu().numpy().view(np.uint32)
        assert [int(v) for v in ct] == c["ct"], f
        assert "%016x" % fx.fnv(out) == c["out_fnv"], f
        for b in range(8):   # the row bands each of 8 ranks would hold
            band = out[b * 270 * W4:(b + 1) * 270 * W4]
            assert "%016x" % fx.fnv(band) == c["band_fnv"][b], (f, b)


def _c5(gpu, nshard):
    import torch
    big = fx.load_json("big.json")
    key = "16384x16384_k1024"
    if key not in big:
        pytest.skip("C5 fixture not generated")
    c = big[key]
    arrs = fx.load_npz("big.npz")
    t = torch.from_numpy(fx.xorshift(16384 * 16384).view(np.int32)).to("cuda:0")
    o = torch.empty_like(t)
    if nshard == 0:
        ct, _ = gpu.quant_device(t, o, 1024)
    else:
        (ct,), _ = gpu.quant_rows_device([t], [o], 1024, widths=[16384], nshard=nshard)
    torch.cuda.synchronize()
    assert [int(v) for v in ct] == c["ct"]
    out = o.cpu().numpy().view(np.uint32)
    del t, o
    assert "%016x" % fx.fnv(out) == c["out_fnv"]
    for b in range(8):
        assert "%016x" % fx.fnv(out[b * 2048 * 16384:(b + 1) * 2048 * 16384]) == c["band_fnv"][b], b
    assert np.array_equal(gpu.last_trace(1024), arrs["trace_" + key])
    _check_centroids(gpu, 1024, arrs["means_" + key])


def test_c5_gigapixel_one_gpu(gpu):
    """C5 16384x16384 K=1024 on one GPU (the bench's N=1 rows workload)."""
    _c5(gpu, 0)


def test_c5_gigapixel_8_row_shards(gpu):
    """C5 with its rows split into 8 shards: the arithmetic of the 8-GPU run."""
    _c5(gpu, 8)
