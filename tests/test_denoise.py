"""NL-means denoiser (denoiser/denoiser.py) host side: the float64 checker
(oracle/nlmeans_check.py) against a direct per-pixel evaluation, the
variance image the script reads (hdrToLdr PNG bytes, OpenCV grey), and the
ABI arguments.  GPU parity: test_gpu_denoise.py.

Parity status: pinned by the reference's own denoiser output
(tests/golden/denoiser/final*.png: the checker reproduces final_denoised.png
to the byte on all but a handful of pixels, each within 1 LSB), and to the
direct definition below."""
import struct
import zlib

import numpy as np
import pytest

import nori_amd
import nlmeans_check  # oracle/ (on sys.path via conftest)


def _direct(img, var, r, f, k, mode):
    """Sums written out pixel by pixel (slow; tiny images only)."""
    H, W = var.shape
    h = f - 1
    n2 = (2 * h + 1) ** 2

    def dist(i, j, a, b):
        if not (0 <= i < H and 0 <= j < W):
            return 0.0
        qi, qj = (i - a) % H, (j - b) % W
        vq, vp = var[qi, qj], var[i, j]
        v1, v2 = (2 * vq, 2 * vq) if mode == 0 else (vp + min(vp, vq), vp + vq)
        return (float(np.sum((img[qi, qj] - img[i, j]) ** 2)) - v1) / (1e-3 + k * k * v2)

    out = np.zeros_like(img)
    for i in range(H):
        for j in range(W):
            num, den = np.zeros(3), 0.0
            for a in range(-r, r + 1):
                for b in range(-r, r + 1):
                    w = 0.0
                    for u in range(i - h, i + h + 1):
                        for v in range(j - h, j + h + 1):
                            if 0 <= u < H and 0 <= v < W:
                                patch = sum(dist(x, y, a, b) for x in range(u - h, u + h + 1)
                                            for y in range(v - h, v + h + 1)) / n2
                                w += np.exp(-max(0.0, patch))
                    w /= n2
                    num += w * img[(i - a) % H, (j - b) % W]
                    den += w
            out[i, j] = num / den
    return out


def test_window_mean_zero_padded():
    rng = np.random.default_rng(1)
    a = rng.random((7, 9))
    m = nlmeans_check.window_mean(a, 2)
    ref = np.zeros_like(a)
    for i in range(7):
        for j in range(9):
            ref[i, j] = a[max(0, i - 2):i + 3, max(0, j - 2):j + 3].sum() / 25
    assert np.allclose(m, ref, rtol=0, atol=1e-13)


@pytest.mark.parametrize("mode", [0, 1])
def test_checker_matches_direct_definition(mode):
    rng = np.random.default_rng(2 + mode)
    img = rng.random((5, 6, 3)) * 0.05
    var = rng.random((5, 6)) * 0.01
    a = nlmeans_check.nlmeans(img, var, r=1, f=2, k=0.02, mode=mode)
    b = _direct(img, var, 1, 2, 0.02, mode)
    assert np.allclose(a, b, rtol=1e-12, atol=0)


def test_checker_keeps_constant_images():
    img = np.full((12, 10, 3), 0.3)
    var = np.full((12, 10), 0.02)
    assert np.allclose(nlmeans_check.nlmeans(img, var), img, rtol=1e-12)


def _png_bytes(path):
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w, h = 8, b"", 0, 0
    while pos < len(data):
        n, kind = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        if kind == b"IHDR":
            w, h = struct.unpack(">II", body[:8])
        elif kind == b"IDAT":
            idat += body
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + 3 * w)
    assert (raw[:, 0] == 0).all()  # filter type None on every row
    return raw[:, 1:].reshape(h, w, 3)


def test_variance_gray_is_the_png_the_script_reads(built, tmp_path):
    rng = np.random.default_rng(4)
    var = (rng.random((9, 11, 3)) ** 3).astype(np.float32) * 1.2
    var[0, 0] = (1, 0, 0)
    path = tmp_path / "v.png"
    nori_amd.write_png(str(path), var)
    assert np.array_equal(_png_bytes(path), nori_amd.ldr_bytes(var))
    g = nori_amd.variance_gray(var)
    assert g.shape == (9, 11) and g.dtype == np.float32
    # OpenCV reads B, G, R and RGB2GRAY weighs channel 0 (blue) as red
    assert g[0, 0] == pytest.approx(((1868 * 255 + 8192) >> 14) / 255.0)


def test_denoise_rejects_bad_arguments(built):
    img = np.zeros((8, 8, 3), np.float32)
    with pytest.raises(ValueError):
        nori_amd.denoise(img, np.zeros((8, 7), np.float32))
    with pytest.raises(nori_amd.NoriError):
        nori_amd.denoise(img, np.zeros((8, 8), np.float32), radius=9)


def test_cli_png_reader_and_grey(built, tmp_path):
    """The CLI's PNG path gives the same grey image as variance_gray()."""
    from nori_amd.denoiser import png_gray, read_png_rgb8

    rng = np.random.default_rng(5)
    var = rng.random((6, 7, 3)).astype(np.float32)
    nori_amd.write_png(str(tmp_path / "v.png"), var)
    assert np.array_equal(png_gray(read_png_rgb8(str(tmp_path / "v.png"))), nori_amd.variance_gray(var))


GOLD = __import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "denoiser")


def reference_triple(stem, var_stem, out_stem):
    """The script's inputs from the reference's PNGs (denoiser.py:16-21: / 255,
    grey variance through OpenCV's BGR read + COLOR_RGB2GRAY) and its output
    bytes."""
    import os
    rd = lambda n: nori_amd.read_image(os.path.join(GOLD, n + ".png"))
    img = rd(stem).astype(np.float64) / 255.0
    var = nori_amd.variance_gray_bytes(rd(var_stem)).astype(np.float64)
    return img, var, rd(out_stem).astype(np.int64)


def compare_bytes(out01, ref_bytes):
    got = np.round(np.clip(np.asarray(out01, np.float64) * 255.0, 0, 255)).astype(np.int64)
    d = np.abs(got - ref_bytes)
    return float((d == 0).mean()), int(d.max()), float((d <= 2).mean())


def test_checker_reproduces_reference_final_denoised(built):
    """denoiser.py at its own parameters (r = 3, f = 3, k = 0.02) on the
    reference's final.png + final_variance.png: the checker's output, taken to
    bytes, is the reference's final_denoised.png (measured: 99.9996 % of the
    values equal, the rest 1 LSB -- the script's float64 order of sums)."""
    img, var, ref = reference_triple("final", "final_variance", "final_denoised")
    exact, dmax, _ = compare_bytes(nlmeans_check.nlmeans(img, var, r=3, f=3, k=0.02, mode=0), ref)
    assert exact >= 0.9999 and dmax <= 1, (exact, dmax)


def test_checker_near_reference_denoised(built):
    """The 800x600 triple (image.png + variance.png -> denoised.png) is not the
    script at its committed parameters: at k = 0.02 83 % of the bytes are
    equal and 96 % within 2 LSB, with up to 54 LSB on a few thousand pixels
    (the best k, about 0.5, gives 91.5 % equal) -- the output of an earlier
    parameterisation or variance image.  A qualitative pin: >= 95 % within
    2 LSB."""
    img, var, ref = reference_triple("image", "variance", "denoised")
    exact, dmax, near = compare_bytes(nlmeans_check.nlmeans(img, var, r=3, f=3, k=0.02, mode=0), ref)
    assert near >= 0.95 and exact >= 0.8, (exact, dmax, near)
