"""Jitter classes of the film splat (device_math.h jit_class, kernels.hip k_splat CODED).

ImageBlock::put (block.cpp:93-122) derives a sample's window weights from
P = fl(x + jit) - 0.5 - (offset - border): the box [ceil(P - r), floor(P + r)]
and, per tile cell c, the table index (int)(|c - P| * lookup).  The GPU stores
8 bits per axis in the sample record -- (floor(P) - (x - offset) - border + 1,
[f * lookup is an integer], q = floor(f * lookup)) of f = P - floor(P) -- and k_splat
rebuilds every cell's index from a representative offset of that class.
This test checks, in float32 (numpy rounds each operation as the device
does), that the class reproduces the direct formula's weight -- its table
index, or 0 outside the box -- for every window cell, for every pixel column 0..2047 of its
block, at the reference's power-of-two filters (box 0.5, tent 1, gaussian /
Mitchell 2), on random pcg32 jitters and on the edge values (0, 1/2, the
class boundaries q / lookup and their float neighbours, 1 - 2^-23).
"""
import numpy as np
import pytest

R = 32  # NORI_FILTER_RESOLUTION
BLOCK = 32
f32 = np.float32


def direct_indices(x, jit, radius, B):
    """Cell indices (or -1 outside the box) by the splat's direct formula."""
    lk = f32(R / radius)
    rad = f32(radius)
    K, TS = 2 * B + 1, BLOCK + 2 * B
    ox = (x // BLOCK) * BLOCK
    lx = x - ox
    px = ((x.astype(f32) + jit) - f32(0.5)) - (ox - B).astype(f32)
    x0 = np.maximum(np.ceil(px - rad).astype(np.int64), 0)
    x1 = np.minimum(np.floor(px + rad).astype(np.int64), TS - 1)
    out = []
    for d in range(K):
        cx = lx + d
        k = np.minimum(np.floor(np.abs(cx.astype(f32) - px) * lk).astype(np.int64), R)
        out.append(np.where((cx >= x0) & (cx <= x1), k, -1))
    return np.stack(out, -1)


def classes(x, jit, radius, B):
    """device_math.h jit_class."""
    lk = f32(R / radius)
    ox = (x // BLOCK) * BLOCK
    P = ((x.astype(f32) + jit) - f32(0.5)) - (ox - B).astype(f32)
    n = np.floor(P)
    f = P - n
    qf = f * lk
    q = np.floor(qf)
    return (n.astype(np.int64) - (x - ox) - B + 1) | np.where(q == qf, 2, 0) | (q.astype(np.int64) << 2)


def class_indices(c, radius, B):
    """k_splat's class table (CODED): the formula on a representative offset."""
    lk = f32(R / radius)
    rad = f32(radius)
    m = B + (c & 1) - 1
    q = (c >> 2).astype(f32)
    f = np.where((c & 2) != 0, q / lk, (q + f32(0.5)) / lk).astype(f32)
    lo = m + np.ceil(f - rad).astype(np.int64)
    hi = m + np.floor(f + rad).astype(np.int64)
    out = []
    for d in range(2 * B + 1):
        k = np.minimum(np.floor(np.abs((d - m).astype(f32) - f) * lk).astype(np.int64), R)
        out.append(np.where((d >= lo) & (d <= hi), k, -1))
    return np.stack(out, -1)


def jitters(radius, rng):
    lk = int(R / radius)
    step = 1 << 23
    m = [0, 1, 2, step - 1, step - 2]
    for k in range(lk + 1):  # class boundaries k / lookup and their neighbours
        b = k * step // lk
        m += [b + e for e in range(-40, 41)]
    m += [(step >> 1) + e for e in range(-3000, 3001)]  # jit near 1/2 (P near an integer)
    m += list(rng.integers(0, step, 20000))
    m = np.unique(np.clip(np.array(m, dtype=np.int64), 0, step - 1))
    return (m.astype(np.float64) * 2.0 ** -23).astype(f32)  # pcg32 nextFloat: (r >> 9) * 2^-23


@pytest.mark.parametrize("radius,B", [(0.5, 0), (1.0, 1), (2.0, 2)])
def test_class_reproduces_the_direct_weights(radius, B):
    rng = np.random.default_rng(7)
    jit = jitters(radius, rng)
    lk = int(R / radius)
    for x0 in range(0, 2048, 256):
        x = np.arange(x0, x0 + 256, dtype=np.int64)[:, None]
        X, J = np.broadcast_arrays(x, jit[None, :])
        want = direct_indices(X, J, radius, B)
        c = classes(X, J, radius, B)
        assert c.min() >= 0 and c.max() < 4 * lk  # 8 bits, k_splat's table size
        got = class_indices(c, radius, B)
        # the weight of index R is the table's 0 (runtime.hip filter_table), as
        # outside the box: fl(P + r) and fl(P - r) can round across an integer
        # only at a cell |c - P| >= r, i.e. index R (so the comparison is of weights)
        want, got = np.where(want == R, -1, want), np.where(got == R, -1, got)
        bad = np.argwhere(np.any(want != got, -1))
        assert bad.size == 0, (radius, X[tuple(bad[0])], J[tuple(bad[0])], want[tuple(bad[0])], got[tuple(bad[0])])


def test_window_has_the_full_support():
    """A sample at an integer P touches all K cells (both ends at |c - P| = r), else K - 1."""
    x = np.array([[40]])
    for jit, cells in [(f32(0.5), 5), (f32(0.25), 4), (f32(0.75), 4)]:
        idx = direct_indices(x, np.array([[jit]]), 2.0, 2)
        assert (idx >= 0).sum() == cells
