"""ImageTexture albedo and NormalMap on the GPU against the CPU oracle
(identical WAVE streams; bar: per-pixel L2 <= 1e-7 as in test_gpu_parity.py).

Scenes: the reference's scenes/project/cbox_path_mis.xml (ImageTexture albedo
on the right wall and a sphere, textures/texture.jpg) and the same file with
its commented-out NormalMap elements enabled (textures/textureNormals.jpg),
with the path_mis and the normals integrators; the texture path is pinned
GPU <-> oracle (the oracle restates imagetexture.cpp / normalmap.cpp
literally, its bilinear form included).

Reference-side evidence: report-project/images/texture.png (and
texture_normal*.png, texture_clamp.png) are screenshots of this textured
Cornell box.  They cannot be reproduced from the checkout's files: the
reference later overwrote scenes/project/meshes/{left,right}wall.obj with the
walls of its final "tree" scene (those are what the scene file loads today),
and the cbox walls of scenes/pa4 carry a single texture coordinate, while
the screenshot's right wall shows the brick texture.  So
test_texture_report_screenshot renders the scene file with the pa4 cbox walls
and compares region means of the aligned 8-bit image with the screenshot:
a qualitative pin of the textured sphere and the rest of the box (green and
blue means within 6 %; red within 12 %, since the screenshot's brick wall
adds red light the constant wall does not; measured on the textured sphere:
red -6.6 %, green +1.5 %, blue +4.7 %).
"""
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


def test_texture_report_screenshot(built, tmp_path):
    from nori_test_util import read_png

    shot = "/report-project/images/texture.png"
    golden = os.path.join(ROOT, "tests", "golden", "project", "report_texture.png")
    src = open(os.path.join(SCENES, "cbox_path_mis.xml")).read()
    cbox = os.path.join(ROOT, "scenes", "pa4", "cbox", "meshes")
    src = src.replace('value="meshes/leftwall.obj"', f'value="{cbox}/leftwall.obj"')
    src = src.replace('value="meshes/rightwall.obj"', f'value="{cbox}/rightwall.obj"')
    src = src.replace('value="meshes/', f'value="{SCENES}/meshes/').replace('value="textures/', f'value="{SCENES}/textures/')
    xml = str(tmp_path / "texture_cbox.xml")
    open(xml, "w").write(src)
    s = nori_amd.load_scene(xml, 800, 600, 64)
    with nori_amd.GpuRenderer(s, 0) as r:
        ours = nori_amd.ldr_bytes(nori_amd.develop(s, r.render())).astype(np.float64)
    ref = read_png(golden)[..., :3].astype(np.float64)
    lum = ref.sum(-1)  # the screenshot's black margins
    rows = np.where((lum > 30).mean(1) > 0.5)[0]
    cols = np.where((lum > 30).mean(0) > 0.5)[0]
    c = ref[rows.min():rows.max() + 1, cols.min():cols.max() + 1]
    h, w = c.shape[:2]
    g, gc = ours.mean(-1), c.mean(-1)
    best = min((np.mean((g[dy:dy + h:4, dx:dx + w:4] - gc[::4, ::4]) ** 2), dy, dx)
               for dy in range(0, 600 - h + 1) for dx in range(0, 800 - w + 1))
    err, dy, dx = best
    o = ours[dy:dy + h, dx:dx + w]
    print(f"{shot}: aligned at ({dy}, {dx}), RMS {np.sqrt(err):.1f} LDR levels")
    assert err < 400, best
    for name, (y0, y1, x0, x1) in {"textured sphere": (360, 520, 440, 610), "back wall": (100, 300, 200, 600),
                                   "left wall": (50, 500, 20, 120), "mirror sphere": (350, 500, 180, 340)}.items():
        m, mr = o[y0:y1, x0:x1].reshape(-1, 3).mean(0), c[y0:y1, x0:x1].reshape(-1, 3).mean(0)
        rel = np.abs(m - mr) / mr
        print(f"  {name}: ours {m.round(1)} screenshot {mr.round(1)}")
        assert rel[0] < 0.12 and rel[1] < 0.06 and rel[2] < 0.06, (name, m, mr)
