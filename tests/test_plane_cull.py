"""The scan's axis-plane cull (kernels.hip plane_may_hit) is exact: whenever
it says a ray cannot hit a triangle lying in an axis plane, the reference's
Moller-Trumbore test (mesh.cpp:83-120) rejects that ray.  Checked here in
float32 arithmetic with the device's evaluation order (device_math.h cross /
dot, no contraction; numpy float32 ops round like the GPU's), on the Cornell
box's axis-plane triangles, over random, grazing, on-plane and
boundary-of-[mint, maxt] rays."""
import numpy as np

import nori_amd
from conftest import scene_path

f32 = np.float32
LO, HI = f32(1.0 - 2.0 ** -16), f32(1.0 + 2.0 ** -16)


def cross(a, b):
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


def dot(a, b):
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


def moller_trumbore(p0, e1, e2, o, d, mint, maxt):
    """mesh.cpp:83-120 in float32, vectorised over rays (o, d: 3 arrays)."""
    with np.errstate(all="ignore"):
        pvec = cross(d, e2)
        det = dot(e1, pvec)
        inv = f32(1) / det
        tvec = (o[0] - p0[0], o[1] - p0[1], o[2] - p0[2])
        u = dot(tvec, pvec) * inv
        qvec = cross(tvec, e1)
        v = dot(d, qvec) * inv
        t = dot(e2, qvec) * inv
        return (~((det > f32(-1e-8)) & (det < f32(1e-8))) & ~((u < 0) | (u > 1)) & ~((v < 0) | (u + v > 1)) &
                (t >= mint) & (t <= maxt)), t


def may_hit(o, d, c, mint, maxt):
    """kernels.hip plane_may_hit (no bound on a side where mint <= 0 / maxt <= 0)."""
    with np.errstate(all="ignore"):
        T = o - c
        ad = np.abs(d)
        s = np.where(d > 0, -T, T)
        lo = np.where(mint > 0, mint * LO * ad, f32(-np.inf)).astype(f32)
        hi = np.where(maxt > 0, maxt * HI * ad, f32(np.inf)).astype(f32)
        return (s > lo) & (s < hi)


def plane_triangles():
    s = nori_amd.load_scene(scene_path("pa4", "cbox", "cbox_path_mis.xml"), 32, 32, 1)
    P = np.asarray(s.positions(), np.float32).reshape(-1, 3)
    out = []
    for f in np.asarray(s.indices()).reshape(-1, 3):
        p0 = P[f[0]]
        e1, e2 = P[f[1]] - p0, P[f[2]] - p0
        for a in range(3):
            if e1[a] == 0 and e2[a] == 0:
                out.append((p0, e1, e2, a))
    return out


def rays(rng, n):
    o = rng.uniform([-1.1, -0.1, -1.1], [1.1, 1.7, 1.1], size=(n, 3)).astype(f32)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d = d.astype(f32)
    m = rng.random(n) < 0.5  # grazing: one component tiny
    ax = rng.integers(0, 3, n)
    d[m, ax[m]] = (rng.choice([-1, 1], m.sum()) * 10.0 ** rng.uniform(-9, -2, m.sum())).astype(f32)
    return o, d


def test_cull_implies_reject(built):
    tris = plane_triangles()
    assert len(tris) >= 8  # cbox: floor, ceiling, back and right wall, light
    rng = np.random.default_rng(7)
    culled = checked = 0
    for p0, e1, e2, a in tris:
        c = p0[a]
        o, d = rays(rng, 200000)
        o[:50000, a] = c  # origins on the plane
        o[50000:80000, a] = c + f32(1e-7) * rng.choice([-1, 1], 30000).astype(f32)  # just off it
        mint = np.maximum(f32(1e-4), f32(1e-4) * np.abs(o).max(axis=1)).astype(f32)
        maxt = np.full(len(o), np.inf, f32)
        # maxt near the plane distance: the t-bound side of the cull
        with np.errstate(all="ignore"):
            tp = ((c - o[:, a]) / d[:, a]).astype(f32)
        k = slice(100000, 160000)
        maxt[k] = np.where(np.isfinite(tp[k]) & (tp[k] > 0), tp[k] * f32(1 + 3e-6) * rng.choice(
            [f32(1), f32(1 - 1e-5)], 60000), f32(1)).astype(f32)
        mint[160000:] = np.where(np.isfinite(tp[160000:]) & (tp[160000:] > 0), tp[160000:] * f32(1 - 3e-6),
                                 mint[160000:]).astype(f32)
        hit, _ = moller_trumbore(p0, e1, e2, (o[:, 0], o[:, 1], o[:, 2]), (d[:, 0], d[:, 1], d[:, 2]), mint, maxt)
        may = may_hit(o[:, a], d[:, a], c, mint, maxt)
        assert not (hit & ~may).any(), np.nonzero(hit & ~may)[0][:5]
        culled += int((~may).sum())
        checked += len(o)
    assert culled > checked // 4  # the cull is not vacuous


def test_cull_with_zero_mint_keeps_plane_hits(built):
    """mint = 0 (the trace API passes the caller's mint): origins on the plane
    are hit at t = +-0, which the cull must not skip."""
    rng = np.random.default_rng(9)
    kept = 0
    for p0, e1, e2, a in plane_triangles():
        c = p0[a]
        o, d = rays(rng, 50000)
        o[:, a] = c
        mint = np.zeros(len(o), f32)
        maxt = np.full(len(o), np.inf, f32)
        hit, t = moller_trumbore(p0, e1, e2, (o[:, 0], o[:, 1], o[:, 2]), (d[:, 0], d[:, 1], d[:, 2]), mint, maxt)
        may = may_hit(o[:, a], d[:, a], c, mint, maxt)
        assert not (hit & ~may).any()
        kept += int((hit & (t == 0)).sum())
    assert kept > 1000  # t = 0 hits exist and are kept


def moller_trumbore_plane(p0, e1, e2, o, d, mint, maxt, A):
    """kernels.hip tri_hit_plane<A>: the products with the zero components left out."""
    with np.errstate(all="ignore"):
        tv = (o[0] - p0[0], o[1] - p0[1], o[2] - p0[2])
        if A == 0:
            pv = (d[1] * e2[2] - d[2] * e2[1], -(d[0] * e2[2]), d[0] * e2[1])
            det = e1[1] * pv[1] + e1[2] * pv[2]
            qv = (tv[1] * e1[2] - tv[2] * e1[1], -(tv[0] * e1[2]), tv[0] * e1[1])
            tn = e2[1] * qv[1] + e2[2] * qv[2]
        elif A == 1:
            pv = (d[1] * e2[2], d[2] * e2[0] - d[0] * e2[2], -(d[1] * e2[0]))
            det = e1[0] * pv[0] + e1[2] * pv[2]
            qv = (tv[1] * e1[2], tv[2] * e1[0] - tv[0] * e1[2], -(tv[1] * e1[0]))
            tn = e2[0] * qv[0] + e2[2] * qv[2]
        else:
            pv = (-(d[2] * e2[1]), d[2] * e2[0], d[0] * e2[1] - d[1] * e2[0])
            det = e1[0] * pv[0] + e1[1] * pv[1]
            qv = (-(tv[2] * e1[1]), tv[2] * e1[0], tv[0] * e1[1] - tv[1] * e1[0])
            tn = e2[0] * qv[0] + e2[1] * qv[1]
        inv = f32(1) / det
        u = dot(tv, pv) * inv
        v = dot(d, qv) * inv
        t = tn * inv
        ok = (~((det > f32(-1e-8)) & (det < f32(1e-8))) & ~((u < 0) | (u > 1)) & ~((v < 0) | (u + v > 1)) &
              (t >= mint) & (t <= maxt))
        return ok, t, u, v


def test_plane_test_is_the_generic_test(built):
    """tri_hit_plane<A> accepts exactly the rays tri_hit_nb accepts, with the
    same t bits and the same u, v values (up to the sign of a zero)."""
    rng = np.random.default_rng(11)
    for p0, e1, e2, a in plane_triangles():
        o, d = rays(rng, 200000)
        o[:40000, a] = p0[a]
        mint = np.maximum(f32(1e-4), f32(1e-4) * np.abs(o).max(axis=1)).astype(f32)
        maxt = np.full(len(o), np.inf, f32)
        O, D = (o[:, 0], o[:, 1], o[:, 2]), (d[:, 0], d[:, 1], d[:, 2])
        h1, t1 = moller_trumbore(p0, e1, e2, O, D, mint, maxt)
        h2, t2, u2, v2 = moller_trumbore_plane(p0, e1, e2, O, D, mint, maxt, a)
        assert np.array_equal(h1, h2)
        assert np.array_equal(t1[h1].view(np.uint32), t2[h2].view(np.uint32))
        assert h1.sum() > 100
