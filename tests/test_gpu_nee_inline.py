"""GPU: next-event shadow rays traced inside the shade kernel (S.nee_inline,
kernels.hip k_shade: the work-group's shadow rays compacted into LDS slots,
any hit through the wave-uniform scan, then one read-modify-write of each
sample record -- emission first, then the unoccluded NEE term, the order of
the separate k_shadow_scan launch) against the shadow queue
(NORI_NEE_INLINE=0): the same image up to the film sums' order, the same ray
counts, for each integrator that traces shadow rays (path_mis, volumetric)
and for path_mats (emission only).  Only the basic-plugin shade kernels
carry the inline path (kernels.h kNeeFull): on scenes with the full plugin
set (point lights, Disney, chromatic aberration) NORI_NEE_INLINE=1 keeps
the queue.  The defaults are checked too: on for the basic-plugin Cornell
box, off for the full-plugin volumetric scene and for BVH scenes."""
import os
import re

import numpy as np
import pytest

import nori_amd
from conftest import scene_path
import synth

pytestmark = pytest.mark.gpu

CHROMA = ('<float name="lensRadius" value="0.05"/><float name="focalDist" value="5"/>'
          '<vector name="chromaticAberation" value="3.5, 2, 2.5"/>')


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


def _scene(kind, tmp_path):
    if kind == "cbox_path_mis":
        return nori_amd.load_scene(scene_path("pa4", "cbox", "cbox_path_mis.xml"), 96, 72, 8)
    if kind in ("volumetric", "volumetric_basic"):
        src = open(scene_path("project", "volumetric", "volumetric.xml")).read()
        src = src.replace('value="meshes/', f'value="{scene_path("project", "volumetric", "meshes")}/')
        if kind == "volumetric_basic":  # the Disney sphere made diffuse: the basic plugin set
            src = re.sub(r'<bsdf type="disney">.*?</bsdf>',
                         '<bsdf type="diffuse"><color name="albedo" value="0.5 0.5 0.5"/></bsdf>', src, flags=re.S)
        xml = str(tmp_path / f"{kind}.xml")
        open(xml, "w").write(src)
        return nori_amd.load_scene(xml, 80, 60, 8)
    if kind in ("path_mats", "lights_path_mis"):
        extra = ""
        if kind == "lights_path_mis":
            extra = ('<emitter type="point"><point name="position" value="0.3,1.2,0.2"/>'
                     '<color name="power" value="2,1.5,1"/></emitter>')
        xml = synth.cbox_variant(str(tmp_path), kind, integrator="path_mats" if kind == "path_mats" else "path_mis",
                                 extra=extra, width=80, height=64)
        return nori_amd.load_scene(xml, 0, 0, 8)
    assert kind == "chroma_path_mis"
    xml = synth.cbox_variant(str(tmp_path), kind, integrator="path_mis", camera_type="advancedCamera",
                             camera_props=CHROMA, width=80, height=64)
    return nori_amd.load_scene(xml, 0, 0, 8)


BASIC = ["cbox_path_mis", "path_mats", "volumetric_basic"]


@pytest.mark.parametrize("kind", BASIC + ["lights_path_mis", "volumetric", "chroma_path_mis"])
def test_inline_nee_same_image(built, tmp_path, kind):
    s = _scene(kind, tmp_path)
    inl, que = _renderer(s, NORI_NEE_INLINE="1"), _renderer(s, NORI_NEE_INLINE="0")
    try:
        a, b = inl.render(), que.render()
        sa, sb = inl.last_stats, que.last_stats
        assert sa["nee_inline"] == (1 if kind in BASIC else 0) and sb["nee_inline"] == 0
        assert np.allclose(a, b, rtol=1e-5, atol=1e-6), np.abs(a - b).max()
        for k in ("samples", "invalid_samples", "rays_closest", "rays_shadow", "rays_finish"):
            assert sa[k] == sb[k], (k, sa[k], sb[k])
        if kind != "path_mats":
            assert sa["rays_shadow"] > 0
        assert a.mean() > 0.0
    finally:
        inl.close()
        que.close()


def test_inline_nee_defaults(built):
    cbox = nori_amd.load_scene(scene_path("pa4", "cbox", "cbox_path_mis.xml"), 64, 48, 2)
    vol = nori_amd.load_scene(scene_path("project", "volumetric", "volumetric.xml"), 64, 48, 2)
    for s, on in ((cbox, 1), (vol, 0)):
        r = _renderer(s)
        try:
            r.render()
            assert r.last_stats["nee_inline"] == on
        finally:
            r.close()
    r = _renderer(cbox, NORI_TRAVERSAL="bvh", NORI_NEE_INLINE="1")  # BVH walks: always the queue
    try:
        r.render()
        assert r.last_stats["nee_inline"] == 0 and r.last_stats["rays_shadow"] > 0
    finally:
        r.close()
