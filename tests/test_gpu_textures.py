"""ImageTexture albedo and NormalMap on the GPU against the CPU oracle
(identical WAVE streams; bar: per-pixel L2 <= 1e-7 as in test_gpu_parity.py).

Scenes: the reference's scenes/project/cbox_path_mis.xml (ImageTexture albedo
on the right wall and a sphere, textures/texture.jpg) and the same file with
its commented-out NormalMap elements enabled (textures/textureNormals.jpg),
with the path_mis and the normals integrators.  The reference holds no render
of these scenes: the texture path is pinned GPU <-> oracle only (parity
unpinned against the reference); the oracle restates imagetexture.cpp /
normalmap.cpp literally (its bilinear form included)."""
import os

import numpy as np
import pytest

import nori_amd
import pyoracle
from conftest import ROOT

pytestmark = pytest.mark.gpu
SCENES = os.path.join(ROOT, "scenes", "project", "textured")


@pytest.mark.parametrize("xml,spp", [("cbox_path_mis.xml", 8), ("cbox_normalmap.xml", 8),
                                     ("cbox_normalmap_normals.xml", 2), ("cbox_normals.xml", 2)])
def test_textured_scene_matches_oracle(built, xml, spp):
    s = nori_amd.load_scene(os.path.join(SCENES, xml), 96, 72, spp)
    with nori_amd.GpuRenderer(s, 0) as r:
        raw = r.render()
        st = r.last_stats
    cpu_raw = pyoracle.OracleScene(s).render(rng="wave")
    gpu, cpu = nori_amd.develop(s, raw), nori_amd.develop(s, cpu_raw)
    assert st["samples"] == 96 * 72 * spp
    assert np.isfinite(gpu).all() and float(gpu.mean()) > 0
    l2 = float(np.mean((gpu - cpu) ** 2))
    exact = float(np.mean(np.all(raw == cpu_raw, axis=-1)))
    print(f"{xml}: L2 {l2:.3e}, bit-identical film cells {exact:.3f}")
    assert l2 < 1e-7
    if "normals" in xml:  # one bounce, no transcendental-dependent branching
        assert l2 < 1e-10
