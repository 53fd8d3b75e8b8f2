"""CPU: the weighted path's exact parallel fold, as a model.

The GPU path reproduces the reference's sequential FP64 folds s += x_i
(DivQuantCluster.cpp:73-85, :496-517, :719-770) by classifying every summand
from a prefix estimate: a summand whose running sum provably stays in one
binade [2^e, 2^(e+1)) adds u * RNE(x / u), u = 2^(e-52), exactly; the rest
("specials": the first summand, binade crossings, ties) are added in order.
This file restates that algorithm in numpy with the GPU's tile size, margin,
segment limit and chain rules, and checks it bit for bit against the
sequential fold on summand sequences shaped like the reference's (weights
count / N times channel values and their squares, zeros for points not
taken), including sequences built to land on binade boundaries and ties.
"""
import math

import numpy as np
import pytest

TILE = 4096
MARGIN = 2.0 ** -20
SEG_MAX = 128       # kWSeg


def seq_fold(x):
    s = 0.0
    for v in x.tolist():
        s += v
    return s


def binade(v):
    return math.frexp(v)[1] - 1   # 2^e <= v < 2^(e+1)


def classify_tile(x, p0):
    """One tile: the segments (('run', e, M) | ('sp', x)) in order, or None
    when the tile is not describable (the GPU folds it summand by summand).
    p0: the tile's prefix estimate (any summation order)."""
    # in-tile prefix estimate: per-lane sums of 16 then an exclusive scan
    # (any order is fine: only the bound matters)
    pre = np.concatenate([[0.0], np.cumsum(x)[:-1]]) + p0
    kinds, es, ms = [], [], []
    for xi, P in zip(x.tolist(), pre.tolist()):
        if xi == 0.0:
            kinds.append("zero"); es.append(None); ms.append(0)
            continue
        lo, hi = P * (1.0 - MARGIN), (P + xi) * (1.0 + MARGIN)
        if not lo > 0.0 or binade(lo) != binade(hi):
            kinds.append("sp"); es.append(None); ms.append(0)
            continue
        e = binade(lo)
        t = math.ldexp(xi, 52 - e)
        fl = math.floor(t)
        fr = t - fl
        if fr == 0.5:
            kinds.append("sp"); es.append(None); ms.append(0)
            continue
        kinds.append("run"); es.append(e); ms.append(int(fl) + (1 if fr > 0.5 else 0))
    # segments in sequence order: each special, and each maximal stretch of
    # run members (m != 0) with one (specials before, binade) key
    segs = []
    key = None
    nsp = 0
    for k, e, m, xi in zip(kinds, es, ms, x.tolist()):
        if k == "sp":
            segs.append(("sp", xi))
            nsp += 1
        elif k == "run" and m != 0:
            if (nsp, e) != key:
                key = (nsp, e)
                segs.append(["run", e, 0])
            segs[-1][2] += m
    if len(segs) > SEG_MAX:
        return None
    return [tuple(g) for g in segs]


def apply_run(s, e, m):
    if not s > 0.0 or binade(s) != e:
        return None
    si = int(math.ldexp(s, 52 - e)) + m
    if si > 2 ** 53:
        return None
    return math.ldexp(float(si), e - 52)


def parallel_fold(x):
    """The GPU's fold: tiles, prefix estimates, descriptions, the chain."""
    tiles = [x[i:i + TILE] for i in range(0, max(len(x), 1), TILE)]
    est = [float(np.sum(t)) for t in tiles]           # wk_tilesum (any order)
    pre = np.concatenate([[0.0], np.cumsum(est)[:-1]]) # wk_prefix (any order)
    s = 0.0
    seq_tiles = 0
    for t, p0 in zip(tiles, pre.tolist()):
        segs = classify_tile(t, p0)
        v = s
        ok = segs is not None
        if ok:
            for g in segs:
                if g[0] == "sp":
                    v += g[1]
                else:
                    v = apply_run(v, g[1], g[2])
                    if v is None:
                        ok = False
                        break
        if ok:
            s = v
        else:   # summand by summand
            seq_tiles += 1
            for xi in t.tolist():
                s += xi
    return s, seq_tiles


def summands(n, seed, kind):
    """Sequences like the reference's: w = count / N over unique colours,
    times a channel value, its square, or 1, zero where a point is not taken."""
    rng = np.random.default_rng(seed)
    counts = rng.integers(1, 4, n)
    N = float(counts.sum())
    w = (1.0 / N) * counts.astype(np.float64)
    v = rng.integers(0, 256, n).astype(np.uint32)
    if kind == "sum":
        x = w * v.astype(np.float64)
    elif kind == "sq":
        x = w * (v * v).astype(np.float64)
    else:
        x = w.copy()
    take = rng.random(n) < 0.5
    x[~take] = 0.0
    return x


@pytest.mark.parametrize("n", [1, 7, 4095, 4096, 4097, 30000, 200000])
@pytest.mark.parametrize("kind", ["sum", "sq", "w"])
def test_parallel_fold_equals_sequential(n, kind):
    x = summands(n, n * 7 + len(kind), kind)
    got, _ = parallel_fold(x)
    assert got.hex() == seq_fold(x).hex()


def test_binade_boundaries_and_ties():
    """Summands that put the running sum exactly on binade boundaries and
    halfway between grid points (ties, decided by the sum's parity)."""
    rng = np.random.default_rng(3)
    for trial in range(40):
        n = int(rng.integers(100, 20000))
        x = np.full(n, 2.0 ** -int(rng.integers(3, 12)))            # exact powers of two
        x[rng.integers(0, n, n // 7)] *= 3.0                          # odd multiples
        x[rng.integers(0, n, n // 11)] = 2.0 ** -60 * 3               # tiny: ties at coarse grids
        x[rng.integers(0, n, n // 13)] = 0.0
        got, _ = parallel_fold(x)
        assert got.hex() == seq_fold(x).hex(), trial


@pytest.mark.parametrize("kind", ["sum", "sq", "w"])
def test_every_tile_is_described(kind):
    """No tile needs the summand-by-summand fold on reference-like sequences,
    the node's first tile included (its sum crosses a binade every few
    summands from s = 0: 20-40 segments, within kWSeg)."""
    for seed in range(4):
        x = summands(120000, 11 + seed, kind)
        got, seq_tiles = parallel_fold(x)
        assert got.hex() == seq_fold(x).hex()
        assert seq_tiles == 0, (kind, seed)


def slots_like_the_kernel(kinds, keys, lanes=256, per=16, wave=64):
    """wk_classify's distributed slot assignment (dq_weighted.hip): per lane
    its first / last member key and inner starts, the nearest earlier lane
    with members inside the wave, wave aggregates, then each item's slot.
    kinds[i]: 0 zero, 1 run member (key[i]), 2 special.  Returns {i: slot}."""
    L = [list(range(l * per, (l + 1) * per)) for l in range(lanes)]
    nsl = [sum(kinds[i] == 2 for i in L[l]) for l in range(lanes)]
    spb = [sum(nsl[:l]) for l in range(lanes)]
    nsp = sum(nsl)
    kf, kl, inner = [-1] * lanes, [-1] * lanes, [0] * lanes
    for l in range(lanes):
        sp = spb[l]
        for i in L[l]:
            if kinds[i] == 2:
                sp += 1
            elif kinds[i] == 1:
                k = (sp << 12) | keys[i]
                if kf[l] < 0:
                    kf[l] = k
                elif k != kl[l]:
                    inner[l] += 1
                kl[l] = k
    nw = lanes // wave
    starts, known, kprev_w = [0] * lanes, [False] * lanes, [-1] * lanes
    for l in range(lanes):
        w0 = (l // wave) * wave
        prev = [j for j in range(w0, l) if kf[j] >= 0]
        known[l] = bool(prev)
        kprev_w[l] = kl[prev[-1]] if prev else -1
        starts[l] = inner[l] + (1 if kf[l] >= 0 and known[l] and kf[l] != kprev_w[l] else 0)
    agg = []
    for w in range(nw):
        ls = [l for l in range(w * wave, (w + 1) * wave) if kf[l] >= 0]
        agg.append((kf[ls[0]] if ls else -1, kl[ls[-1]] if ls else -1,
                    sum(starts[w * wave:(w + 1) * wave])))
    slot = {}
    kp, sb, kprev = -1, [0] * nw, [-1] * nw
    acc = 0
    for w in range(nw):
        f, lk, ws = agg[w]
        add = ws + (1 if f >= 0 and f != kp else 0)
        sb[w], kprev[w] = acc, kp
        acc += add
        if lk >= 0:
            kp = lk
    ntot = acc
    for l in range(lanes):
        w = l // wave
        if kf[l] >= 0 and not known[l] and kf[l] != kprev[w]:
            starts[l] += 1
    for l in range(lanes):
        w = l // wave
        r = sb[w] + sum(starts[w * wave:l])
        sp = spb[l]
        key = kprev_w[l] if known[l] else kprev[w]
        for i in L[l]:
            if kinds[i] == 2:
                slot[i] = r + sp
                sp += 1
            elif kinds[i] == 1:
                k = (sp << 12) | keys[i]
                if k != key:
                    r += 1
                    key = k
                slot[i] = r - 1 + sp
    return slot, ntot + nsp


def test_kernel_slot_assignment_is_sequence_order():
    """The kernel's scan-based slots equal the sequential segmentation's,
    for class patterns with empty lanes, empty waves, keys that repeat
    across specials, and keys that go down."""
    rng = np.random.default_rng(5)
    for trial in range(60):
        n = 4096
        kinds = rng.choice([0, 1, 2], n, p=[0.5, 0.49, 0.01]).tolist()
        if trial % 3 == 0:   # an empty wave and empty lanes
            for i in range(1024, 2048):
                kinds[i] = 0
        keys = np.cumsum(rng.random(n) < 0.002).tolist() if trial % 2 else rng.integers(0, 3, n).tolist()
        keys = [int(k) + 26 for k in keys]
        slot, nseg = slots_like_the_kernel(kinds, keys)
        # sequential reference
        exp, cur, s, sp = {}, None, -1, 0
        for i in range(n):
            if kinds[i] == 2:
                s += 1
                exp[i] = s
                sp += 1
                cur = None
            elif kinds[i] == 1:
                k = (sp, keys[i])
                if k != cur:
                    s += 1
                    cur = k
                exp[i] = s
        assert slot == exp, trial
        assert nseg == s + 1
