"""Records finalised at a frame's last planned round, whose partition (PS_STATS)
counts no partition cursors, and then partitioned by a later host round:
their cursors are counted when needed (Engine::fix_cursors).
Skewed frames (a half-masked gradient, power-law channels) at K=1000 make
the greedy replay split below the planned levels where such a record was
proven at its split (tools/cursor_fix_designs.py: 1-2 records per call;
most such parents were 2-means records, whose cursors their passes count).
A batch of two such 4K frames on one engine lane (rounds of > 12 M points:
the PS_STATS last round) must equal each frame run alone (one frame per
call: no PS_STATS round) -- the single-frame path is pinned to the
reference's fixtures -- and must have taken the fix-up path."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _frame(design, n, seed):
    """tools/cursor_fix_designs.py's frames that take the path (measured)."""
    rng = np.random.default_rng(seed)
    if design == "gradient":
        i = np.arange(n, dtype=np.uint64)
        px = ((i * 2654435761) >> 8).astype(np.uint32) & 0x00FFFFFF
        px[: n // 2] &= 0x0F0F0F
        return px
    r, g, b = ((rng.pareto(1.5, n) * 20).clip(0, 255).astype(np.uint32) for _ in range(3))
    return (r << 16) | (g << 8) | b


@pytest.mark.parametrize("design,k", [("gradient", 1000), ("powerlaw", 1000)])
def test_batch_stats_round_then_host_partition(gpu, design, k):
    import torch
    n = 3840 * 2160
    frames = [_frame(design, n, s) for s in (1, 2)]
    ts = [torch.from_numpy(f.view(np.int32)).to("cuda:0") for f in frames]
    lanes = gpu.get_lanes()
    gpu.set_lanes(1)
    try:
        outs = [torch.empty_like(t) for t in ts]
        cts, _ = gpu.quant_batch_device(ts, outs, k)
        torch.cuda.synchronize()
        fixes = gpu.last_cursor_fixes()
    finally:
        gpu.set_lanes(lanes)
    assert fixes > 0, "the fix-up path was not taken (%d)" % fixes
    for i, t in enumerate(ts):
        o = torch.empty_like(t)
        ct, _ = gpu.quant_device(t, o, k)
        torch.cuda.synchronize()
        assert np.array_equal(cts[i], ct), i
        assert torch.equal(outs[i], o), i
