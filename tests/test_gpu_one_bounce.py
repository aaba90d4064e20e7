"""GPU path (libnori_gpu.so, k_direct + k_splat and the path kernels' camera /
texture / light code) against the CPU oracle for the widened plugins: the
one-bounce integrators, point and spot lights, the checkerboard texture and
the thinlens / advancedCamera ray generators.

Tolerance: identical WAVE random streams on both sides; per-pixel L2 <= 1e-7 on
linear RGB (BASELINE.json's bar is 1e-3), as in test_gpu_parity.py.  The full-size
renders are additionally compared with the reference's golden EXRs in
expectation (channel means, 16x16-block relMSE).
"""
import numpy as np
import pytest

import nori_amd
import pyoracle
import synth
from conftest import scene_path
from nori_test_util import load_test_scenes, parse_test_xml, students_t_test

pytestmark = pytest.mark.gpu

L2_TOL = 1e-7


def _gpu_vs_oracle(s):
    with nori_amd.GpuRenderer(s, 0) as r:
        raw = r.render()
        st = r.last_stats
    gpu = nori_amd.develop(s, raw)
    cpu_raw = pyoracle.OracleScene(s).render(rng="wave")
    cpu = nori_amd.develop(s, cpu_raw)
    assert st["samples"] == s.width * s.height * s.spp
    assert np.isfinite(gpu).all()
    l2 = float(np.mean((gpu - cpu) ** 2))
    exact = float(np.mean(np.all(raw == cpu_raw, axis=-1)))
    return gpu, cpu, l2, exact, st


SCENES = ["pa1/sphere-analytic.xml", "pa1/sphere-mesh.xml", "pa1/sphere-texture.xml", "pa1/mesh-texture.xml",
          "pa3/sphere/point_ems.xml", "pa3/sphere/sphere_ems.xml", "pa3/sphere/sphere_mats.xml", "pa3/sphere/sphere_mesh_ems.xml",
          "pa3/odyssey/odyssey_ems.xml", "pa3/odyssey/odyssey_mats.xml", "pa3/odyssey/odyssey_mis.xml",
          "pa3/veach_mi/veach_mis.xml", "project/spotlight/sphere-texture.xml"]


@pytest.mark.parametrize("xml", SCENES)
def test_one_bounce_matches_oracle(built, xml):
    s = nori_amd.load_scene(scene_path(xml), 96, 80, 8)
    gpu, cpu, l2, exact, st = _gpu_vs_oracle(s)
    print(f"{xml} [{s.integrator}]: L2 {l2:.3e}, bit-identical film cells {exact:.3f}, "
          f"rays {st['rays_closest']}+{st['rays_shadow']}")
    assert l2 < L2_TOL
    assert st["rays_closest"] >= s.width * s.height * s.spp


@pytest.mark.parametrize("xml,golden", [("pa3/sphere/sphere_ems.xml", "pa3/sphere/ref/sphere_ems.exr"),
                                        ("pa3/odyssey/odyssey_mis.xml", "pa3/odyssey/ref/odyssey_mis_32spp.exr"),
                                        ("pa3/veach_mi/veach_mis.xml", "pa3/veach_mi/ref/veach_mis_128spp.exr"),
                                        ("pa1/sphere-texture.xml", "pa1/ref/sphere-texture.exr"),
                                        ("pa1/mesh-texture.xml", "pa1/ref/mesh-texture.exr")])
def test_one_bounce_full_size_matches_golden(built, xml, golden):
    s = nori_amd.load_scene(scene_path(xml))
    with nori_amd.GpuRenderer(s, 0) as r:
        img = nori_amd.develop(s, r.render())
    ref = nori_amd.read_exr(scene_path(golden))
    m, mr = img.mean(axis=(0, 1)), ref.mean(axis=(0, 1))
    h, w = img.shape[0] // 16 * 16, img.shape[1] // 16 * 16
    bi = img[:h, :w].reshape(h // 16, 16, w // 16, 16, 3).mean(axis=(1, 3))
    br = ref[:h, :w].reshape(h // 16, 16, w // 16, 16, 3).mean(axis=(1, 3))
    rb = float(np.mean((bi - br) ** 2 / (br ** 2 + 1e-2)))
    print(f"{xml} full size: means {m} golden {mr}, 16x16-block relMSE {rb:.2e}")
    assert np.all(np.abs(m - mr) / np.maximum(mr, 1e-3) < 5e-3)
    assert rb < 1e-3


@pytest.mark.parametrize("xml", ["test-av.xml", "test-direct.xml"])
def test_pa1_ttests_gpu(built, tmp_path, xml):
    """Student-t tests of the reference (1x1-pixel scenes): the GPU's pixel
    value at 40k spp against the reference values."""
    path = scene_path("pa1", xml)
    meta = parse_test_xml(path)
    fails = []
    for (scene, integ), ref in zip(load_test_scenes(path, tmp_path, spp=40000), meta["references"]):
        with nori_amd.GpuRenderer(scene, 0) as r:
            img = nori_amd.develop(scene, r.render())
        _, var_o = pyoracle.OracleScene(scene).ttest(20000)
        val = float((img[0, 0] * [0.212671, 0.715160, 0.072169]).sum())
        ok, p = students_t_test(val, var_o, ref, 40000, 0.01, len(meta["references"]))
        if not ok:
            fails.append((integ, ref, val, p))
    assert not fails, fails


CAMERAS = {
    "thinlens": ("thinlens", '<float name="lensRadius" value="0.08"/><float name="focalDist" value="4.8"/>'),
    "adv_lens": ("advancedCamera", '<float name="lensRadius" value="0.08"/><float name="focalDist" value="4.8"/>'),
    "adv_distortion": ("advancedCamera", '<vector name="distortion" value="0.4, 0.2"/>'),
    "adv_all": ("advancedCamera", '<float name="lensRadius" value="0.05"/><float name="focalDist" value="5"/>'
                                  '<vector name="distortion" value="3, 3"/>'),
}


@pytest.mark.parametrize("cam", sorted(CAMERAS))
@pytest.mark.parametrize("integrator", ["path_mis", "direct_mis"])
def test_cameras_match_oracle(built, tmp_path, cam, integrator):
    ctype, props = CAMERAS[cam]
    xml = synth.cbox_variant(str(tmp_path), cam, integrator=integrator, camera_type=ctype, camera_props=props,
                             width=80, height=64)
    s = nori_amd.load_scene(xml, 0, 0, 8)
    gpu, cpu, l2, exact, st = _gpu_vs_oracle(s)
    print(f"{cam} {integrator}: L2 {l2:.3e}, bit-identical film cells {exact:.3f}")
    assert l2 < L2_TOL
    assert gpu.mean() > 0.0


def test_chromatic_aberration_one_bounce(built, tmp_path):
    """advancedCamera chromatic aberration: three rays per sample, each
    weighted by its channel (render.cpp:106-121)."""
    xml = synth.cbox_variant(str(tmp_path), "chroma", integrator="direct_mis", camera_type="advancedCamera",
                             camera_props='<float name="lensRadius" value="0.05"/><float name="focalDist" value="5"/>'
                                          '<vector name="chromaticAberation" value="4, 2, 3.3"/>',
                             width=80, height=64)
    s = nori_amd.load_scene(xml, 0, 0, 8)
    gpu, cpu, l2, exact, st = _gpu_vs_oracle(s)
    print(f"chromatic direct_mis: L2 {l2:.3e}, bit-identical {exact:.3f}")
    assert l2 < L2_TOL
    assert st["rays_closest"] >= 3 * s.width * s.height * s.spp


# the chromatic aberration of the reference's project scene (scenes/project/final.xml:15)
FINAL_CHROMA = '<vector name="chromaticAberation" value="3.5, 2, 2.5"/>'


@pytest.mark.parametrize("integrator", ["path_mis", "path_mats", "volumetric"])
def test_chromatic_aberration_path_integrators(built, tmp_path, integrator):
    """advancedCamera chromatic aberration under the path integrators
    (render.cpp:106-121, as scenes/project/final.xml uses it with path_mis):
    a sample's three channel paths run one after another in one path slot on
    one pcg32 stream, each contributing only its own channel."""
    props = '<float name="lensRadius" value="0.05"/><float name="focalDist" value="5"/>' + FINAL_CHROMA
    if integrator == "volumetric":
        src = open(scene_path("project", "volumetric", "volumetric.xml")).read()
        src = src.replace('value="meshes/', f'value="{scene_path("project", "volumetric", "meshes")}/')
        src = src.replace('<camera type="perspective">', '<camera type="advancedCamera">' + props)
        xml = str(tmp_path / "chroma_vol.xml")
        open(xml, "w").write(src)
        s = nori_amd.load_scene(xml, 80, 60, 4)
    else:
        xml = synth.cbox_variant(str(tmp_path), f"chroma_{integrator}", integrator=integrator,
                                 camera_type="advancedCamera", camera_props=props, width=80, height=64)
        s = nori_amd.load_scene(xml, 0, 0, 8)
    assert list(s.desc.camera.chromatic) == [3.5, 2.0, 2.5]
    gpu, cpu, l2, exact, st = _gpu_vs_oracle(s)
    print(f"chromatic {integrator}: L2 {l2:.3e}, bit-identical {exact:.3f}, rays {st['rays_closest']}")
    assert l2 < L2_TOL
    # every sample traces at least its three camera rays
    assert st["rays_closest"] + st["rays_finish"] >= 3 * s.width * s.height * s.spp
    assert gpu.mean() > 0.0


@pytest.mark.parametrize("integrator", ["path_mis", "path_mats"])
def test_point_spot_lights_in_path_integrators(built, tmp_path, integrator):
    """Free-standing point and spot emitters next to the area light, in the
    path integrators' next-event estimation (path_mats never samples them)."""
    extra = ('<emitter type="point"><point name="position" value="0.3,1.2,0.2"/>'
             '<color name="power" value="2,1.5,1"/></emitter>'
             '<emitter type="spotlight"><point name="position" value="-0.4,1.5,0.5"/>'
             '<color name="color" value="4,4,6"/><vector name="direction" value="0.2,-1,-0.1"/>'
             '<float name="falloffStart" value="10"/><float name="totalWidth" value="30"/></emitter>')
    xml = synth.cbox_variant(str(tmp_path), f"lights_{integrator}", integrator=integrator, extra=extra,
                             width=80, height=64)
    s = nori_amd.load_scene(xml, 0, 0, 8)
    assert [e.type for e in s.emitters()][-2:] == [nori_amd._abi.EMITTER_POINT, nori_amd._abi.EMITTER_SPOT]
    gpu, cpu, l2, exact, st = _gpu_vs_oracle(s)
    print(f"point+spot {integrator}: L2 {l2:.3e}")
    assert l2 < L2_TOL


@pytest.mark.parametrize("integrator", ["av", "normals"])
def test_av_normals_on_cbox(built, tmp_path, integrator):
    props = '<float name="length" value="0.6"/>' if integrator == "av" else ""
    xml = synth.cbox_variant(str(tmp_path), integrator, integrator=integrator, integrator_props=props,
                             width=96, height=80)
    s = nori_amd.load_scene(xml, 0, 0, 8)
    gpu, cpu, l2, exact, st = _gpu_vs_oracle(s)
    print(f"{integrator} cbox: L2 {l2:.3e}, bit-identical {exact:.3f}")
    assert l2 < L2_TOL
