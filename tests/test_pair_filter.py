"""The binned extension kernel's in-plane filter (kernels.hip pair_candidate,
constants from runtime.hip plane_filters) is exact: whenever it says a ray
cannot hit an axis-plane pair, the reference's Moller-Trumbore test
(mesh.cpp:83-120) rejects that ray for both triangles of the pair.  Checked in
float32 with the device's operation order (numpy float32 rounds like the GPU;
the kernel's fused multiply-adds are evaluated in float64 and rounded once to
float32 -- the product of two floats is exact in float64, so only a sum that
ties at float32 precision could round differently, far inside the margins),
on the Cornell box's pairs (the library's own scan list and constants,
nori_scene_scan_list), over random, grazing and on-plane rays and rays aimed
within a few ulps of the triangles' edges and corners."""
import numpy as np

import nori_amd
from conftest import scene_path
from test_plane_cull import LO, HI, moller_trumbore

f32 = np.float32


def fma(a, b, c):
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(f32)


def pair_candidate(A, f, o, d, mint, maxt):
    """kernels.hip pair_candidate<A> with f = the pair's 8 filter floats."""
    B, C = (A + 1) % 3, (A + 2) % 3
    with np.errstate(all="ignore"):
        rcp = (f32(1) / d[:, A]).astype(f32)
        tf = ((f32(f[5]) - o[:, A]) * rcp).astype(f32)
        dB = fma(tf, d[:, B], (o[:, B] - f32(f[0])).astype(f32))
        dC = fma(tf, d[:, C], (o[:, C] - f32(f[2])).astype(f32))
        so = (np.abs(o[:, B]) + np.abs(o[:, C])).astype(f32)
        sd = (np.abs(d[:, B]) + np.abs(d[:, C])).astype(f32)
        S = fma(np.abs(tf), sd, so)
        thB = fma(np.full_like(S, f[4]), S, np.full_like(S, f[1]))
        thC = fma(np.full_like(S, f[4]), S, np.full_like(S, f[3]))
        mlo = np.where(mint > 0, mint * LO, f32(-np.inf)).astype(f32)
        mhi = np.where(maxt > 0, maxt * HI, f32(np.inf)).astype(f32)
        return (tf > mlo) & (tf <= mhi) & ~(np.abs(dB) > thB) & ~(np.abs(dC) > thC)


def pairs():
    s = nori_amd.load_scene(scene_path("pa4", "cbox", "cbox_path_mis.xml"), 32, 32, 1)
    L = nori_amd.scan_list(s)
    out = []
    for g in range(len(L["plane_c"])):
        A = int(np.searchsorted(L["plane_end"], g, side="right"))
        recs = [L["records"][2 * g + k] for k in range(2)]
        out.append((A, L["plane_f"][g], recs))
    return out


def targeted_rays(rng, recs, A, n):
    """Rays through points within a few ulps of the triangles' edges and corners."""
    pts = []
    for r in recs:
        v0, e1, e2 = r[0:3].astype(np.float64), r[4:7].astype(np.float64), r[8:11].astype(np.float64)
        if not e1.any():
            continue
        V = [v0, v0 + e1, v0 + e2]
        for i in range(3):
            a, b = V[i], V[(i + 1) % 3]
            s = rng.random(n // 6)[:, None]
            p = a + s * (b - a)
            p[: n // 24] = a  # corners
            pts.append(p)
    p = np.concatenate(pts)
    jit = rng.normal(size=p.shape) * 10.0 ** rng.uniform(-8, -5, (len(p), 1))
    jit[:, A] = 0
    p = p + jit
    o = rng.uniform([-1.1, -0.1, -1.1], [1.1, 1.7, 1.1], size=p.shape)
    near = rng.random(len(p)) < 0.3  # grazing: origin close to the plane
    o[near, A] = p[near, A] + rng.choice([-1, 1], near.sum()) * 10.0 ** rng.uniform(-6, -1, near.sum())
    d = p - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return o.astype(f32), d.astype(f32)


def random_rays(rng, n):
    o = rng.uniform([-1.1, -0.1, -1.1], [1.1, 1.7, 1.1], size=(n, 3)).astype(f32)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d = d.astype(f32)
    m = rng.random(n) < 0.4
    ax = rng.integers(0, 3, n)
    d[m, ax[m]] = (rng.choice([-1, 1], m.sum()) * 10.0 ** rng.uniform(-9, -2, m.sum())).astype(f32)
    return o, d


def test_filter_implies_reject(built):
    ps = pairs()
    assert len(ps) == 5  # right wall, floor, ceiling, light, back wall
    rng = np.random.default_rng(5)
    rejected = checked = hits = 0
    for A, f, recs in ps:
        for o, d in (random_rays(rng, 300000), targeted_rays(rng, recs, A, 240000)):
            o[:20000, A] = f32(f[5])  # origins on the plane
            mint = np.maximum(f32(1e-4), f32(1e-4) * np.abs(o).max(axis=1)).astype(f32)
            maxt = np.full(len(o), np.inf, f32)
            cam = rng.random(len(o)) < 0.2  # camera-like rays: finite [mint, maxt]
            maxt[cam] = rng.uniform(0.5, 20, cam.sum()).astype(f32)
            mint[cam] = rng.uniform(1e-4, 1e-2, cam.sum()).astype(f32)
            mint[:5000] = 0.0  # trace-API rays with mint = 0, origins on the plane: t = +-0 hits
            O, D = (o[:, 0], o[:, 1], o[:, 2]), (d[:, 0], d[:, 1], d[:, 2])
            hit = np.zeros(len(o), bool)
            for r in recs:
                h, _ = moller_trumbore(r[0:3], r[4:7], r[8:11], O, D, mint, maxt)
                hit |= h
            cand = pair_candidate(A, f, o, d, mint, maxt)
            bad = hit & ~cand
            assert not bad.any(), (A, f[5], np.nonzero(bad)[0][:5])
            rejected += int((~cand).sum())
            hits += int(hit.sum())
            checked += len(o)
    assert hits > 50000  # the rays do hit the pairs, near their edges too
    assert rejected > checked // 2  # and the filter is not vacuous
