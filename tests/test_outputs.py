"""Output formats, no GPU needed:
* nori_write_png <- Bitmap::saveToLDR (bitmap.cpp:109-139): the bytes are the
  reference's TO_BYTE(v) = (uint8_t) Clamp(255 * GammaCorrect(v) + 0.5, 0, 255)
  restated in numpy (float32; pow may differ by an ulp from glibc's powf, which
  moves a byte by one only at exact .5 boundaries), the PNG structure and CRCs
  are checked with zlib.
* nori_film_variance: the variance of each pixel's mean from (sum L, sum L^2, n),
  against a float64 numpy restatement.
"""
import struct
import zlib

import numpy as np

import nori_amd
from conftest import scene_path


def _read_png(path):
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, chunks = 8, []
    while pos < len(data):
        (n,) = struct.unpack(">I", data[pos:pos + 4])
        kind, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        (crc,) = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert crc == zlib.crc32(kind + body) & 0xFFFFFFFF, kind
        chunks.append((kind, body))
        pos += 12 + n
    assert [k for k, _ in chunks] == [b"IHDR", b"IDAT", b"IEND"]
    w, h, depth, ctype, comp, filt, inter = struct.unpack(">IIBBBBB", chunks[0][1])
    assert (depth, ctype, comp, filt, inter) == (8, 2, 0, 0, 0)
    raw = np.frombuffer(zlib.decompress(chunks[1][1]), np.uint8).reshape(h, 1 + 3 * w)
    assert (raw[:, 0] == 0).all()  # filter type 0 on every scanline
    return raw[:, 1:].reshape(h, w, 3)


def _to_byte(v):  # bitmap.cpp:109-139 in float32
    v = v.astype(np.float32)
    g = np.where(v <= np.float32(0.0031308), np.float32(12.92) * v,
                 np.float32(1.055) * np.power(np.maximum(v, 0), np.float32(1 / 2.4), dtype=np.float32) - np.float32(0.055))
    return np.clip(np.float32(255) * g.astype(np.float32) + np.float32(0.5), 0, 255).astype(np.uint8)


def test_png_matches_save_to_ldr(built, tmp_path):
    rng = np.random.default_rng(1)
    img = (rng.random((37, 53, 3)) * 1.4 - 0.1).astype(np.float32)
    img[0, 0] = [np.inf, -np.inf, 0.0031308]
    img[np.isinf(img)] = 0.5  # the reference clamps NaN/Inf undefined; keep the test finite
    p = str(tmp_path / "x.png")
    nori_amd.write_png(p, img)
    got = _read_png(p).astype(int)
    want = _to_byte(img).astype(int)
    assert got.shape == want.shape
    assert np.abs(got - want).max() <= 1
    assert (got == want).mean() > 0.999


def test_film_variance(built):
    s = nori_amd.load_scene(scene_path("pa4", "cbox", "cbox_path_mis.xml"), 6, 4, 1)
    rng = np.random.default_rng(2)
    L = rng.gamma(2.0, 0.3, size=(16, 4, 6, 3))
    st = np.zeros((4, 6, 8), np.float32)
    st[..., 0:3] = L.sum(0)
    st[..., 3:6] = (L ** 2).sum(0)
    st[..., 6] = 16
    st[0, 0, 6] = 1  # n < 2: no estimate
    v = nori_amd.film_variance(s, st)
    s1, s2 = st[..., 0:3].astype(np.float64), st[..., 3:6].astype(np.float64)
    n = st[..., 6:7].astype(np.float64)
    want = (s2 - s1 * s1 / n) / (n * (n - 1.0))
    want[0, 0] = 0.0
    assert np.allclose(v, want, rtol=1e-5, atol=1e-9)
    assert np.allclose(v[1:, 1:], L.var(0, ddof=1)[1:, 1:] / 16, rtol=1e-3)
