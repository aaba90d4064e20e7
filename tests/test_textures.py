"""ImageTexture / NormalMap (src/imagetexture.cpp, src/normalmap.cpp) on the
host side: the image decoder, the loader's image table and the oracle.

The reference decodes textures with stbi_load(.., STBI_rgb) of the stb_image
v1.39 its GUI dependency vendors; image_decode.cpp restates that version's
arithmetic (file:line in its header).  stb_image itself cannot be built here
(building the reference's vendored sources was refused), so the
decoder is checked against an independent decoder, Pillow:
* PNG is lossless: bit-exact on every colour type stb v1.39 reads (8-bit
  gray, gray+alpha, RGB, RGBA, palette) and on an Adam7-interlaced file;
* baseline JPEG: the IDCT (12-bit vs libjpeg-turbo's 13-bit constants) and
  the chroma upsampling round differently, so the bar is |d| <= 3 per byte
  and a mean |d| < 0.1 -- exact stb agreement is "parity unpinned";
* progressive JPEG and PNGs of other bit depths fail as in stb v1.39.
"""
import os
import struct
import zlib

import numpy as np
import pytest

import nori_amd
import pyoracle
from nori_amd import _abi
from conftest import ROOT

PIL = pytest.importorskip("PIL.Image")
TEX = os.path.join(ROOT, "scenes", "project", "textured", "textures")
SCENES = os.path.join(ROOT, "scenes", "project", "textured")


@pytest.mark.parametrize("name", ["texture.jpg", "textureNormals.jpg", "fun.jpeg", "default1.jpg",
                                  "floor_albedo.jpg", "floor_normal.jpg"])
def test_jpeg_matches_independent_decoder(built, name):
    p = os.path.join(TEX, name)
    mine = nori_amd.read_image(p).astype(int)
    ref = np.asarray(PIL.open(p).convert("RGB")).astype(int)
    assert mine.shape == ref.shape
    d = np.abs(mine - ref)
    print(f"{name}: {mine.shape}, max |d| {d.max()}, mean |d| {d.mean():.4f}")
    assert d.max() <= 3 and d.mean() < 0.1


def test_progressive_jpeg_and_low_depth_png_are_rejected(built):
    with pytest.raises(nori_amd.NoriError) as e:
        nori_amd.read_image(os.path.join(TEX, "earth.jpg"))  # SOF2
    assert e.value.code == _abi.NORI_ERR_UNSUPPORTED and "progressive" in str(e.value)
    with pytest.raises(nori_amd.NoriError) as e:
        nori_amd.read_image(os.path.join(TEX, "default.png"))  # 4-bit palette
    assert e.value.code == _abi.NORI_ERR_UNSUPPORTED


@pytest.mark.parametrize("mode", ["L", "LA", "RGB", "RGBA", "P"])
def test_png_bit_exact(built, tmp_path, mode):
    rng = np.random.default_rng(len(mode))
    w, h = 37, 23
    if mode == "P":
        im = PIL.fromarray(rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)).quantize(200)
    else:
        ch = {"L": 1, "LA": 2, "RGB": 3, "RGBA": 4}[mode]
        arr = rng.integers(0, 256, size=(h, w, ch), dtype=np.uint8)
        # smooth ramps too, so every row filter gets used by the encoder
        arr[: h // 2] = (np.arange(w)[None, :, None] * 7 + np.arange(h // 2)[:, None, None] * 3) % 256
        im = PIL.fromarray(arr[..., 0] if ch == 1 else arr, mode)
    p = str(tmp_path / f"t_{mode}.png")
    im.save(p, optimize=True)
    mine = nori_amd.read_image(p)
    ref = np.asarray(PIL.open(p).convert("RGB"))
    assert np.array_equal(mine, ref)


def _png_chunk(t, data):
    return struct.pack(">I", len(data)) + t + data + struct.pack(">I", zlib.crc32(t + data) & 0xFFFFFFFF)


def test_png_adam7_interlaced(built, tmp_path):
    """Hand-built Adam7 file (Pillow does not write interlaced PNGs): passes of
    filter-0 rows, pixel (x, y) = (x, y, x ^ y)."""
    w, h = 13, 11
    img = np.zeros((h, w, 3), np.uint8)
    yy, xx = np.mgrid[0:h, 0:w]
    img[..., 0], img[..., 1], img[..., 2] = xx * 9, yy * 11, (xx ^ yy) * 5
    raw = b""
    for x0, y0, dx, dy in [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2),
                           (0, 1, 1, 2)]:
        sub = img[y0::dy, x0::dx]
        if sub.size == 0:
            continue
        for row in sub:
            raw += b"\x00" + row.tobytes()
    ihdr = struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 1)
    data = b"\x89PNG\r\n\x1a\n" + _png_chunk(b"IHDR", ihdr) + _png_chunk(b"IDAT", zlib.compress(raw)) + \
        _png_chunk(b"IEND", b"")
    p = tmp_path / "adam7.png"
    p.write_bytes(data)
    assert np.array_equal(nori_amd.read_image(str(p)), img)


def test_loader_builds_image_table(built):
    s = nori_amd.load_scene(os.path.join(SCENES, "cbox_normalmap.xml"), 40, 30, 1)
    d = s.desc
    assert d.num_images == 4
    tex = nori_amd.read_image(os.path.join(TEX, "texture.jpg"))
    nrm = nori_amd.read_image(os.path.join(TEX, "textureNormals.jpg"))
    albedo = [d.bsdfs[i].albedo_image for i in range(d.num_bsdfs)]
    nmaps = [d.shapes[i].normal_map for i in range(d.num_shapes)]
    assert [a >= 0 for a in albedo] == [False, True, False, False, True, False]
    assert [m >= 0 for m in nmaps] == [False, True, False, False, True, False]
    for i in albedo + nmaps:
        if i < 0:
            continue
        im = d.images[i]
        assert (im.width, im.height, im.wrap) == (1600, 1546, _abi.WRAP_REPEAT)
        got = np.ctypeslib.as_array(im.rgb, shape=(im.height, im.width, 3))
        assert np.array_equal(got, tex if i in albedo else nrm)
    for i in range(d.num_bsdfs):
        assert (d.bsdfs[i].albedo_texture == _abi.TEXTURE_IMAGE) == (albedo[i] >= 0)


def test_bad_wrap_name_is_a_parse_error(built, tmp_path):
    xml = open(os.path.join(SCENES, "cbox_path_mis.xml")).read().replace('value="repeat"', 'value="mirror"')
    p = tmp_path / "bad.xml"
    p.write_text(xml.replace('meshes/', os.path.join(SCENES, "meshes") + '/').replace(
        'textures/', os.path.join(TEX) + '/'))
    with pytest.raises(nori_amd.NoriError) as e:
        nori_amd.load_scene(str(p), 8, 8, 1)
    assert e.value.code == _abi.NORI_ERR_PARSE and "wrap" in str(e.value)


def test_oracle_normal_map_bends_shading_normals(built, tmp_path):
    """normals integrator (normals.cpp) on the reference's Cornell box with its
    commented-out normal maps enabled: the right wall (a mesh with vertex
    normals) changes; a normal map on the sphere alone changes nothing -- the
    mesh code is its only consumer (mesh.cpp:147-155)."""
    a = nori_amd.load_scene(os.path.join(SCENES, "cbox_normals.xml"), 64, 48, 1)
    b = nori_amd.load_scene(os.path.join(SCENES, "cbox_normalmap_normals.xml"), 64, 48, 1)
    xml = open(os.path.join(SCENES, "cbox_normalmap_normals.xml")).read()
    first = xml.find('<texture type="NormalMap"')
    end = xml.find("</texture>", first) + len("</texture>")
    xml = (xml[:first] + xml[end:]).replace('"meshes/', '"' + os.path.join(SCENES, "meshes") + "/").replace(
        '"textures/', '"' + TEX + "/")
    (tmp_path / "sphere_only.xml").write_text(xml)
    c = nori_amd.load_scene(str(tmp_path / "sphere_only.xml"), 64, 48, 1)
    assert [c.desc.shapes[i].normal_map >= 0 for i in range(c.desc.num_shapes)].count(True) == 1
    ia, ib, ic = (nori_amd.develop(x, pyoracle.OracleScene(x).render(rng="wave")) for x in (a, b, c))
    assert np.isfinite(ib).all()
    frac = float((np.abs(ia - ib).max(axis=-1) > 1e-4).mean())
    print(f"pixels changed by the wall's normal map: {frac:.3f}")
    assert 0.05 < frac < 0.6
    assert np.abs(ia - ic).max() < 1e-6  # (film summation order only)
