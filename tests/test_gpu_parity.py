"""GPU path (libnori_gpu.so via the C ABI) against the CPU oracle.

Tolerances:
* traversal: hit distance t bit-exact (both sides use the reference's
  Moeller-Trumbore / sphere / slab arithmetic with no FMA); primitive id
  equal except where two primitives return the identical t (shared edges),
  where the reference's DFS order picks the last one visited.
* images: same WAVE random streams on both sides; transcendentals differ by a
  few ulp (ROCm device library vs glibc), which can flip a rare branch, and the
  film sums arrive in another order.  BASELINE.json's bar is per-pixel L2 <
  1e-3 on linear RGB; the tests assert what the code achieves (measured 1e-15
  to 3e-12 at these sizes, nori_test_util.image_parity): L2 <= 1e-7 -- one
  flipped sample in an 80x60 frame stays under it, a BSDF lobe biased by 1 % on
  cbox (mean ~0.13) does not -- L2 <= 1e-9 without the worst 0.01 % of the
  pixels, and >= 99 % of the pixels equal to 1e-3 relative.
"""
import os

import numpy as np
import pytest

import synth

import nori_amd
import pyoracle
from conftest import scene_path
from nori_test_util import L2_TOL, assert_parity, image_parity, load_test_scenes, parse_test_xml, students_t_test

pytestmark = pytest.mark.gpu

def _rays(n, seed, lo, hi, mint=1e-4, axis_aligned=0.1):
    rng = np.random.default_rng(seed)
    org = rng.uniform(lo, hi, size=(n, 3))
    d = rng.normal(size=(n, 3))
    k = int(n * axis_aligned)  # exercise the d_i == 0 slab branch (bbox.h:344-346)
    d[:k] = 0.0
    d[np.arange(k), rng.integers(0, 3, size=k)] = rng.choice([-1.0, 1.0], size=k)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.zeros((n, 8), np.float32)
    rays[:, :3], rays[:, 3], rays[:, 4:7], rays[:, 7] = org, mint, d, np.inf
    return rays


def _compare_hits(g, c):
    assert (np.isfinite(g["t"]) == np.isfinite(c["t"])).all()
    fin = np.isfinite(c["t"])
    assert (g["t"][fin] == c["t"][fin]).all(), np.abs(g["t"][fin] - c["t"][fin]).max()
    same = g["prim"] == c["prim"]
    assert same.mean() > 0.999, same.mean()


def _renderer(scene, mode=None):
    """GpuRenderer with a forced traversal mode ('scan' or 'bvh'; None = automatic)."""
    old = os.environ.get("NORI_TRAVERSAL")
    if mode:
        os.environ["NORI_TRAVERSAL"] = mode
    try:
        return nori_amd.GpuRenderer(scene, 0)
    finally:
        if old is None:
            os.environ.pop("NORI_TRAVERSAL", None)
        else:
            os.environ["NORI_TRAVERSAL"] = old


@pytest.fixture(scope="module", params=["scan", "bvh"])
def cbox(built, request):
    s = nori_amd.load_scene(scene_path("pa4", "cbox", "cbox_path_mis.xml"), 64, 64, 16)
    r = _renderer(s, request.param)
    yield s, r, pyoracle.OracleScene(s)
    r.close()


@pytest.fixture(scope="module")
def hfield(built, tmp_path_factory):
    xml = synth.heightfield_scene(str(tmp_path_factory.mktemp("hf")), n=48, width=96, height=72, spp=8)
    s = nori_amd.load_scene(xml)
    r = _renderer(s)
    yield s, r, pyoracle.OracleScene(s)
    r.close()


def test_trace_closest_matches_oracle(cbox):
    s, r, o = cbox
    rays = np.concatenate([_rays(20000, 1, [-0.9, 0.05, -0.9], [0.9, 1.5, 0.9]),
                           _rays(5000, 2, [-3, -1, -3], [3, 3, 6], mint=0.01)])
    _compare_hits(r.trace(rays), o.trace(rays))


def test_trace_shadow_matches_oracle(cbox):
    s, r, o = cbox
    rays = _rays(20000, 3, [-0.9, 0.05, -0.9], [0.9, 1.5, 0.9])
    rays[:, 7] = np.random.default_rng(4).uniform(0.01, 2.0, size=rays.shape[0])
    g, c = r.trace(rays, any_hit=True), o.trace(rays, any_hit=True)
    assert ((g["prim"] >= 0) == (c["prim"] >= 0)).all()


@pytest.mark.parametrize("parts", [("project", "volumetric", "volumetric.xml"),
                                   ("project", "disney", "cbox_path_mis.xml"),
                                   ("pa4", "cbox_denoiser", "cbox_path_mis.xml")])
def test_render_scene_matches_oracle(built, parts):
    """Volumetric integrator + medium (a21), Disney BSDF (a17), the sphere-less
    diffuse cbox: GPU image vs the oracle on identical WAVE streams."""
    s = nori_amd.load_scene(scene_path(*parts), 80, 60, 8)
    with nori_amd.GpuRenderer(s, 0) as r:
        raw = r.render()
        st = r.last_stats
    gpu = nori_amd.develop(s, raw)
    cpu_raw = pyoracle.OracleScene(s).render(rng="wave")
    cpu = nori_amd.develop(s, cpu_raw)
    assert st["samples"] == 80 * 60 * 8
    assert np.isfinite(gpu).all()
    l2 = float(np.mean((gpu - cpu) ** 2))
    exact = float(np.mean(np.all(raw == cpu_raw, axis=-1)))
    p = image_parity(gpu, cpu)
    print(f"{'/'.join(parts)}: {p}, bit-identical film cells {exact:.3f}")
    assert_parity(p)
    assert float(np.mean(gpu)) > 0.0


@pytest.mark.parametrize("integrator", ["path_mis", "path_mats"])
def test_render_envmap_matches_oracle(built, tmp_path, integrator):
    """Config C4: Disney sphere + env-mapped sky sphere (a18)."""
    xml = synth.envmap_scene(str(tmp_path), 80, 60, 8, integrator=integrator)
    s = nori_amd.load_scene(xml)
    with nori_amd.GpuRenderer(s, 0) as r:
        raw = r.render()
    gpu = nori_amd.develop(s, raw)
    cpu_raw = pyoracle.OracleScene(s).render(rng="wave")
    cpu = nori_amd.develop(s, cpu_raw)
    assert np.isfinite(gpu).all()
    p = image_parity(gpu, cpu)
    print(f"envmap {integrator}: {p}, mean {gpu.mean():.4f}")
    assert_parity(p)
    assert float(gpu.mean()) > 0.05  # the sky lights the box through its open side


@pytest.mark.parametrize("xml", ["cbox_path_mis.xml", "cbox_path_mats.xml"])
def test_render_matches_oracle(built, xml):
    s = nori_amd.load_scene(scene_path("pa4", "cbox", xml), 96, 72, 16)
    with nori_amd.GpuRenderer(s, 0) as r:
        raw = r.render()
        gpu = nori_amd.develop(s, raw)
        st = r.last_stats
    cpu_raw = pyoracle.OracleScene(s).render(rng="wave")
    cpu = nori_amd.develop(s, cpu_raw)
    assert st["samples"] == 96 * 72 * 16
    assert np.isfinite(gpu).all()
    rel = float(np.mean((gpu - cpu) ** 2 / (cpu ** 2 + 1e-2)))
    p = image_parity(gpu, cpu)
    print(f"{xml}: {p}, relMSE {rel:.3e}")
    assert_parity(p)


def test_render_pass_split_and_pool_invariance(cbox):
    s, r, o = cbox
    whole = r.render(passes=8)
    part = r.render(passes=5, pass_begin=0, path_pool=4096)
    part = r.render(passes=3, pass_begin=5, out=part, path_pool=65536)
    # same samples, different accumulation order only
    assert np.allclose(whole, part, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("filt", ["gaussian", "mitchell", "tent", "box"])  # radii 2, 2, 1, 1/2
def test_splat_jitter_classes_match_the_pcg_jitter(built, tmp_path, filt):
    """k_splat reading the filter weights from the records' jitter classes
    (device_math.h jit_class) against re-deriving the jitter from pcg32
    (NORI_JIT_CODE=0): the same weights, so the same film up to the order of
    the tile atomics."""
    path = scene_path("pa4", "cbox", "cbox_path_mis.xml")
    src = open(path).read().replace('name="filename" value="', f'name="filename" value="{os.path.dirname(path)}/')
    rf = f'<rfilter type="{filt}"/>'
    xml = tmp_path / "cbox_filter.xml"
    xml.write_text(src.replace("<camera type=\"perspective\">", "<camera type=\"perspective\">" + rf, 1))
    s = nori_amd.load_scene(str(xml), 72, 56, 8)
    films = []
    for code in ("1", "0"):
        old = os.environ.get("NORI_JIT_CODE")
        os.environ["NORI_JIT_CODE"] = code
        try:
            with nori_amd.GpuRenderer(s, 0) as r:
                films.append(r.render())
        finally:
            if old is None:
                os.environ.pop("NORI_JIT_CODE")
            else:
                os.environ["NORI_JIT_CODE"] = old
    a, b = films
    assert a.shape == b.shape and np.isfinite(a).all()
    assert np.abs(a - b).max() <= 1e-6 * np.abs(b).max(), np.abs(a - b).max()


def test_render_block_subsets_tile_the_frame(cbox):
    s, r, o = cbox
    whole = r.render(passes=4)
    n = s.num_blocks()
    part = r.render(passes=4, blocks=list(range(0, n, 2)))
    part = r.render(passes=4, blocks=list(range(1, n, 2)), out=part)
    assert np.allclose(whole, part, rtol=1e-4, atol=1e-4)


def test_furnace_gpu(built, tmp_path):
    path = scene_path("pa4", "tests", "test-furnace.xml")
    meta = parse_test_xml(path)
    for (scene, integ), ref in zip(load_test_scenes(path, tmp_path, spp=40000), meta["references"]):
        with nori_amd.GpuRenderer(scene, 0) as r:
            img = nori_amd.develop(scene, r.render())
        mean_o, var_o = pyoracle.OracleScene(scene).ttest(100000)
        val = float((img[0, 0] * [0.212671, 0.715160, 0.072169]).sum())
        ok, p = students_t_test(val, var_o, ref, 40000, 0.01, len(meta["references"]))
        assert ok, (integ, ref, val, p)


def test_trace_large_mesh_bvh(hfield):
    s, r, o = hfield
    rays = np.concatenate([_rays(30000, 5, [-0.9, 0.05, -0.9], [0.9, 1.5, 0.9]),
                           _rays(5000, 6, [-3, -1, -3], [3, 3, 6], mint=0.01)])
    _compare_hits(r.trace(rays), o.trace(rays))
    sh = rays.copy()
    sh[:, 7] = np.random.default_rng(7).uniform(0.01, 2.0, size=sh.shape[0])
    assert ((r.trace(sh, any_hit=True)["prim"] >= 0) == (o.trace(sh, any_hit=True)["prim"] >= 0)).all()


def test_render_large_mesh_matches_oracle(hfield):
    s, r, o = hfield
    gpu = nori_amd.develop(s, r.render())
    cpu = nori_amd.develop(s, o.render(rng="wave"))
    p = image_parity(gpu, cpu)
    print(f"heightfield microfacet path_mis: {p}")
    assert np.isfinite(gpu).all()
    assert_parity(p)


@pytest.mark.parametrize("mode", ["scan", "bvh"])
def test_render_modes_agree(built, mode):
    s = nori_amd.load_scene(scene_path("pa4", "cbox", "cbox_path_mis.xml"), 64, 48, 8)
    r = _renderer(s, mode)
    gpu = nori_amd.develop(s, r.render())
    r.close()
    cpu = nori_amd.develop(s, pyoracle.OracleScene(s).render(rng="wave"))
    assert_parity(image_parity(gpu, cpu))


def test_plane_cull_same_hits(built):
    """The scan's exact axis-plane culls (kernels.hip plane_may_hit: a wave
    skips a wall pair that no ray of it can hit) against the scan without
    them (NORI_PLANE_CULL=0, read at context creation): the same hit on every
    ray -- t bit for bit -- and the same image up to the film sums' order.
    Rays include grazing ones (direction components of 1e-7 .. 1e-3 towards
    the walls), origins on the wall planes, and origins on the planes with
    mint = 0 (a t = 0 hit the culls must keep)."""
    s = nori_amd.load_scene(scene_path("pa4", "cbox", "cbox_path_mis.xml"), 64, 48, 8)
    rays = np.concatenate([_rays(30000, 21, [-0.9, 0.05, -0.9], [0.9, 1.5, 0.9]),
                           _rays(5000, 22, [-3, -1, -3], [3, 3, 6], mint=0.01)])
    rng = np.random.default_rng(24)
    graze = _rays(20000, 25, [-0.9, 0.05, -0.9], [0.9, 1.5, 0.9])
    ax = rng.integers(0, 3, graze.shape[0])
    graze[np.arange(graze.shape[0]), 4 + ax] = (rng.choice([-1, 1], graze.shape[0]) *
                                                10.0 ** rng.uniform(-7, -3, graze.shape[0]))
    on = graze[:10000].copy()  # origins on the wall planes y = 0, y = 1.59, x = 1, z = -1.04
    which = rng.integers(0, 4, on.shape[0])
    on[which == 0, 1] = 0.0
    on[which == 1, 1] = 1.59
    on[which == 2, 0] = 1.0
    on[which == 3, 2] = -1.04
    zero = on.copy()  # mint = 0 (trace API): Moller-Trumbore accepts t = +-0 on the plane itself
    zero[:, 3] = 0.0
    rays = np.concatenate([rays, graze, on, zero]).astype(np.float32)
    sh = rays.copy()
    sh[:, 7] = np.random.default_rng(23).uniform(0.01, 2.0, size=sh.shape[0])
    os.environ["NORI_PLANE_CULL"] = "0"
    try:
        full = nori_amd.GpuRenderer(s, 0)
    finally:
        os.environ.pop("NORI_PLANE_CULL", None)
    filt = nori_amd.GpuRenderer(s, 0)
    try:
        a, b = filt.trace(rays), full.trace(rays)
        assert np.array_equal(a["t"].view(np.uint32), b["t"].view(np.uint32))
        assert np.array_equal(a["prim"], b["prim"])
        assert np.array_equal(a["u"].view(np.uint32), b["u"].view(np.uint32))
        assert np.array_equal(filt.trace(sh, any_hit=True)["prim"] >= 0, full.trace(sh, any_hit=True)["prim"] >= 0)
        fa, fb = filt.render(), full.render()
        assert np.allclose(fa, fb, rtol=1e-5, atol=1e-6), np.abs(fa - fb).max()
    finally:
        filt.close()
        full.close()
