"""GPU: the scan's in-plane wall-pair filter (kernels.hip pair_candidate,
the CULL = 2 skip that k_extend_scan applies to waves of camera rays) drops no
hit.  The trace API runs the scan with the filter (NORI_TRACE_CULL=2, read at
context creation) and without any skip (NORI_TRACE_CULL=0) on the adversarial
rays of tests/test_pair_filter.py -- random, grazing (direction components of
1e-9 .. 1e-2 towards a wall), origins on the wall planes, mint = 0 rays
starting on a plane (a t = +-0 hit), and rays aimed within 1e-8 .. 1e-5 of
the pairs' edges and corners -- through the Cornell box, the odyssey scene (18
pairs in other planes) and the Veach MIS scene: t, primitive and u must be
equal bit for bit, and any-hit occlusion equal.  Renders with the filter switched off at run time
(NORI_CAMERA_CULL=0) must give the same image up to the film sums' order."""
import os

import numpy as np
import pytest

import nori_amd
from conftest import scene_path

pytestmark = pytest.mark.gpu
f32 = np.float32

TRACE_SCENES = [("pa4", "cbox", "cbox_path_mis.xml"), ("pa3", "odyssey", "odyssey_mis.xml"),
                ("pa3", "veach_mi", "veach_ems.xml")]
RENDER_SCENES = [("pa4", "cbox", "cbox_path_mis.xml"), ("project", "adv_cam", "cbox_adv_cam.xml"),
                 ("pa3", "odyssey", "odyssey_mis.xml"), ("project", "volumetric", "volumetric.xml")]


def _renderer(s, **env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return nori_amd.GpuRenderer(s, 0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _box(L):
    """The scan records' bounding box, widened by 10 %."""
    r = L["records"]
    tri = r[:, 7] == 0  # (e1.w == 0: triangles; spheres carry their radius there)
    v0, e1, e2 = r[tri, 0:3], r[tri, 4:7], r[tri, 8:11]
    pts = np.concatenate([v0, v0 + e1, v0 + e2])
    lo, hi = pts.min(axis=0), pts.max(axis=0)
    pad = 0.1 * (hi - lo)
    return lo - pad, hi + pad


def _random_rays(rng, n, lo, hi):
    """Random origins in the box, random directions, 40 % grazing (one component 1e-9 .. 1e-2)."""
    o = rng.uniform(lo, hi, size=(n, 3)).astype(f32)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d = d.astype(f32)
    m = rng.random(n) < 0.4
    ax = rng.integers(0, 3, n)
    d[m, ax[m]] = (rng.choice([-1, 1], m.sum()) * 10.0 ** rng.uniform(-9, -2, m.sum())).astype(f32)
    return o, d


def _targeted_rays(rng, recs, A, n, lo, hi):
    """Rays through points within 1e-8 .. 1e-5 of the pair's edges and corners (in-plane jitter)."""
    pts = []
    for r in recs:
        v0, e1, e2 = r[0:3].astype(np.float64), r[4:7].astype(np.float64), r[8:11].astype(np.float64)
        if not e1.any():
            continue
        V = [v0, v0 + e1, v0 + e2]
        for i in range(3):
            a, b = V[i], V[(i + 1) % 3]
            p = a + rng.random(n // 6)[:, None] * (b - a)
            p[: n // 24] = a  # corners
            pts.append(p)
    p = np.concatenate(pts)
    jit = rng.normal(size=p.shape) * 10.0 ** rng.uniform(-8, -5, (len(p), 1))
    jit[:, A] = 0
    p = p + jit
    o = rng.uniform(lo, hi, size=p.shape)
    near = rng.random(len(p)) < 0.3  # grazing: origin close to the plane
    o[near, A] = p[near, A] + rng.choice([-1, 1], near.sum()) * 10.0 ** rng.uniform(-6, -1, near.sum())
    d = p - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return o.astype(f32), d.astype(f32)


def _ray_set(s, seed):
    L = nori_amd.scan_list(s)
    assert len(L["plane_c"]) > 0, "scene without axis-plane pairs"
    lo, hi = _box(L)
    rng = np.random.default_rng(seed)
    os_, ds, mins, maxs = [], [], [], []
    for g in range(len(L["plane_c"])):
        A = int(np.searchsorted(L["plane_end"], g, side="right"))
        recs = [L["records"][2 * g + k] for k in range(2)]
        for o, d in (_random_rays(rng, 4000, lo, hi), _targeted_rays(rng, recs, A, 8000, lo, hi)):
            o[:1000, A] = f32(L["plane_c"][g])  # origins on the plane
            mint = np.maximum(f32(1e-4), f32(1e-4) * np.abs(o).max(axis=1)).astype(f32)
            maxt = np.full(len(o), np.inf, f32)
            cam = rng.random(len(o)) < 0.3  # camera-like rays: finite [mint, maxt]
            maxt[cam] = (rng.uniform(0.05, 2.0, cam.sum()) * np.linalg.norm(hi - lo)).astype(f32)
            mint[cam] = rng.uniform(1e-4, 1e-2, cam.sum()).astype(f32)
            mint[:400] = 0.0  # mint = 0 with the origin on the plane
            os_.append(o), ds.append(d), mins.append(mint), maxs.append(maxt)
    o, d = np.concatenate(os_), np.concatenate(ds)
    rays = np.zeros((len(o), 8), f32)
    rays[:, :3], rays[:, 3], rays[:, 4:7], rays[:, 7] = o, np.concatenate(mins), d, np.concatenate(maxs)
    return rays


@pytest.mark.parametrize("parts", TRACE_SCENES, ids=["/".join(p[1:]) for p in TRACE_SCENES])
def test_pair_filter_same_hits(built, parts):
    s = nori_amd.load_scene(scene_path(*parts), 64, 48, 4)
    rays = _ray_set(s, 31)
    filt, full = _renderer(s, NORI_TRACE_CULL="2"), _renderer(s, NORI_TRACE_CULL="0")
    try:
        a, b = filt.trace(rays), full.trace(rays)
        assert np.array_equal(a["t"].view(np.uint32), b["t"].view(np.uint32))
        assert np.array_equal(a["prim"], b["prim"])
        assert np.array_equal(a["u"].view(np.uint32), b["u"].view(np.uint32))
        hit = np.isfinite(b["t"])
        assert hit.sum() > len(rays) // 5, hit.sum()  # the rays do hit, at the edges too
        sh = rays.copy()
        sh[:, 7] = np.where(np.isfinite(b["t"]), b["t"] * f32(1.0001), f32(5.0))  # occlusion at the hit itself
        assert np.array_equal(filt.trace(sh, any_hit=True)["prim"] >= 0, full.trace(sh, any_hit=True)["prim"] >= 0)
    finally:
        filt.close()
        full.close()


@pytest.mark.parametrize("parts", RENDER_SCENES, ids=["/".join(p[1:]) for p in RENDER_SCENES])
def test_camera_cull_render_equal(built, parts):
    s = nori_amd.load_scene(scene_path(*parts), 96, 72, 8)
    on, off = _renderer(s), _renderer(s, NORI_CAMERA_CULL="0")
    try:
        fa, fb = on.render(), off.render()
        assert np.allclose(fa, fb, rtol=1e-5, atol=1e-6), np.abs(fa - fb).max()
    finally:
        on.close()
        off.close()


@pytest.mark.parametrize("parts", [("pa4", "cbox", "cbox_path_mis.xml"), ("project", "volumetric", "volumetric.xml")],
                         ids=["cbox", "volumetric"])
@pytest.mark.parametrize("traversal", ["scan", "bvh"])
def test_fused_trace_launch_same_image(built, parts, traversal):
    """One launch for an iteration's extension and shadow rays (nori_rtc_trace_both /
    k_trace_both; NORI_TRACE_FUSE=1) against the two separate launches (=0): the same
    image up to the film sums' order, in both traversal modes."""
    s = nori_amd.load_scene(scene_path(*parts), 96, 72, 8)
    fused, split = (_renderer(s, NORI_TRAVERSAL=traversal, NORI_TRACE_FUSE="1"),
                    _renderer(s, NORI_TRAVERSAL=traversal, NORI_TRACE_FUSE="0"))
    try:
        fa, fb = fused.render(), split.render()
        assert np.allclose(fa, fb, rtol=1e-5, atol=1e-6), np.abs(fa - fb).max()
    finally:
        fused.close()
        split.close()


@pytest.mark.parametrize("parts", TRACE_SCENES, ids=["/".join(p[1:]) for p in TRACE_SCENES])
def test_specialised_scan_same_hits(built, parts):
    """The scan compiled for the scene through hipRTC (csrc/rtc.hip: the scan list as
    literal operands) against the library's generic scan (NORI_RTC=0), on the same
    adversarial rays, with each pair-skip mode: t, primitive and u bit for bit,
    occlusion equal -- and the context reports which one it runs."""
    s = nori_amd.load_scene(scene_path(*parts), 64, 48, 4)
    rays = _ray_set(s, 37)
    sh = rays.copy()
    sh[:, 7] = np.random.default_rng(38).uniform(0.01, 2.0, size=sh.shape[0]).astype(f32)
    for cull in ("0", "1", "2"):
        spec, gen = _renderer(s, NORI_TRACE_CULL=cull), _renderer(s, NORI_TRACE_CULL=cull, NORI_RTC="0")
        try:
            a, b = spec.trace(rays), gen.trace(rays)
            assert np.array_equal(a["t"].view(np.uint32), b["t"].view(np.uint32)), cull
            assert np.array_equal(a["prim"], b["prim"]), cull
            assert np.array_equal(a["u"].view(np.uint32), b["u"].view(np.uint32)), cull
            assert np.array_equal(spec.trace(sh, any_hit=True)["prim"] >= 0, gen.trace(sh, any_hit=True)["prim"] >= 0)
            if cull == "1":
                spec.render()
                gen.render()
                assert spec.last_stats["scan_rtc"] == 1 and gen.last_stats["scan_rtc"] == 0
        finally:
            spec.close()
            gen.close()
