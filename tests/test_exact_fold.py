"""CPU: the weighted path's exact parallel fold, as a model.

The GPU path reproduces the reference's sequential FP64 folds s += x_i
(DivQuantCluster.cpp:73-85, :496-517, :719-770) by classifying every summand
from a prefix estimate: a summand whose running sum provably stays in one
binade [2^e, 2^(e+1)) adds u * RNE(x / u), u = 2^(e-52), exactly; the rest
("specials": the first summand, binade crossings, ties) are added in order.
This file restates that algorithm in numpy with the GPU's tile size, margin,
segment limits and chain rules, and checks it bit for bit against the
sequential fold on summand sequences shaped like the reference's (weights
count / N times channel values and their squares, zeros for points not
taken), including sequences built to land on binade boundaries and ties.
"""
import math

import numpy as np
import pytest

TILE = 4096
MARGIN = 2.0 ** -20
SP_MAX, DE_MAX, SEG_MAX = 16, 16, 32


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
    runs = [e for k, e in zip(kinds, es) if k == "run"]
    e0 = min(runs) if runs else 0
    nsp = kinds.count("sp")
    if nsp > SP_MAX:
        return None
    bins = {}
    sps = []
    spb = 0
    for k, e, m, xi in zip(kinds, es, ms, x.tolist()):
        if k == "sp":
            sps.append(xi)
            spb += 1
        elif k == "run":
            if spb > SP_MAX or e - e0 >= DE_MAX:
                return None
            bins[(spb, e - e0)] = bins.get((spb, e - e0), 0) + m
    segs = []
    for sp in range(nsp + 1):
        for de in range(DE_MAX):
            m = bins.get((sp, de), 0)
            if m:
                segs.append(("run", e0 + de, m))
        if sp < nsp:
            segs.append(("sp", sps[sp]))
    if len(segs) > SEG_MAX:
        return None
    return segs


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


def test_describable_tiles_are_the_rule():
    """Only a node's first tile (many binade crossings from s = 0) may need
    the summand-by-summand fold on the reference-like sequences."""
    x = summands(400000, 11, "sum")
    got, seq_tiles = parallel_fold(x)
    assert got.hex() == seq_fold(x).hex()
    assert seq_tiles <= 1
