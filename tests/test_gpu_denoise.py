"""nori_denoise (k_nlmeans) against the float64 checker
(oracle/nlmeans_check.py).  Tolerance: the kernel computes in fp32 with
fp32 exp; |gpu - checker| <= 2e-4 * max(|checker|, 1e-2) per value, i.e.
fp32 rounding through 49 offsets x two 25-tap box means."""
import os
import subprocess
import sys
import time

import numpy as np
import pytest

import nori_amd
import nlmeans_check  # oracle/ (test infrastructure)

pytestmark = pytest.mark.gpu


def _check(img, var, **kw):
    gpu = nori_amd.denoise(img, var, script_scale=False, **kw)
    mode = kw.get("mode", 0)
    ref = nlmeans_check.nlmeans(img, var, r=kw.get("radius", 3), f=kw.get("patch", 3), k=kw.get("k", 0.02), mode=mode)
    err = np.abs(gpu - ref) / np.maximum(np.abs(ref), 1e-2)
    return gpu, ref, float(err.max())


@pytest.mark.parametrize("shape", [(37, 45), (4, 5), (16, 32), (61, 70)])
@pytest.mark.parametrize("mode", [0, 1])
def test_denoise_matches_checker(built, shape, mode):
    rng = np.random.default_rng(shape[0] * 131 + shape[1] + mode)
    img = (rng.random(shape + (3,)) * 0.004).astype(np.float32)   # the script's /255 scale
    var = (rng.random(shape) * 0.05).astype(np.float32)
    gpu, ref, err = _check(img, var, mode=mode)
    print(f"{shape} mode {mode}: max rel err {err:.2e}")
    assert np.isfinite(gpu).all() and err < 2e-4


@pytest.mark.parametrize("radius,patch", [(0, 1), (1, 2), (5, 4), (8, 5)])
def test_denoise_parameters(built, radius, patch):
    rng = np.random.default_rng(radius * 10 + patch)
    img = (rng.random((40, 50, 3)) * 0.004).astype(np.float32)
    var = (rng.random((40, 50)) * 0.05).astype(np.float32)
    gpu, ref, err = _check(img, var, radius=radius, patch=patch, k=0.05)
    assert err < 2e-4


def test_denoise_rendered_cbox(built, tmp_path):
    """A 16-spp path_mis render with its variance image.  (1) Denoised as the
    script would (EXR / 255, grey 8-bit variance): parity with the checker.
    With the script's distance and scales every weight saturates at 1, so
    its output is a plain box blur -- the MSE against a 512-spp render is
    printed, not asserted.  (2) The textbook distance on linear values with
    the summed per-channel variance of each pixel mean lowers the MSE."""
    from conftest import scene_path

    s = nori_amd.load_scene(scene_path("pa4/cbox/cbox_path_mis.xml"), 160, 120, 16)
    stats = np.zeros((s.height, s.width, 8), np.float32)
    with nori_amd.GpuRenderer(s, 0) as r:
        noisy = nori_amd.develop(s, r.render(variance=stats))
    fvar = nori_amd.film_variance(s, stats)
    var = nori_amd.variance_gray(fvar)
    ref_s = nori_amd.load_scene(scene_path("pa4/cbox/cbox_path_mis.xml"), 160, 120, 512)
    with nori_amd.GpuRenderer(ref_s, 0) as r:
        clean = nori_amd.develop(ref_s, r.render())
    t0 = time.perf_counter()
    den = nori_amd.denoise(noisy, var)
    t1 = time.perf_counter()
    chk = nlmeans_check.nlmeans(noisy / 255.0, var) * 255.0
    err = float((np.abs(den - chk) / np.maximum(np.abs(chk), 1e-2)).max())

    def mse(a):
        return float(np.mean((np.clip(a, 0, 1) - np.clip(clean, 0, 1)) ** 2))

    tb = nori_amd.denoise(noisy, fvar.sum(axis=2), mode=1, script_scale=False)
    print(f"cbox 160x120: denoise {1e3 * (t1 - t0):.2f} ms (host buffers), max rel err {err:.2e}, "
          f"MSE vs 512 spp: noisy {mse(noisy):.3e}, script {mse(den):.3e}, textbook linear {mse(tb):.3e}")
    assert err < 2e-4
    assert mse(tb) < mse(noisy)


def test_denoise_cli(built, tmp_path):
    s = nori_amd.load_scene(__import__("conftest").scene_path("pa4/cbox/cbox_path_mis.xml"), 64, 48, 8)
    stats = np.zeros((s.height, s.width, 8), np.float32)
    with nori_amd.GpuRenderer(s, 0) as r:
        img = nori_amd.develop(s, r.render(variance=stats))
    nori_amd.write_exr(str(tmp_path / "c.exr"), img)
    nori_amd.write_png(str(tmp_path / "c_variance.png"), nori_amd.film_variance(s, stats))
    r = subprocess.run([sys.executable, "-m", "nori_amd.denoiser", "--img_path", str(tmp_path / "c.exr"),
                        "--var_path", str(tmp_path / "c_variance.png")], capture_output=True, text=True,
                       timeout=120, env=dict(os.environ, PYTHONPATH=os.path.dirname(os.path.dirname(nori_amd.__file__))))
    assert r.returncode == 0, r.stderr
    out = nori_amd.read_exr(str(tmp_path / "c_denoised.exr"))
    var = nori_amd.variance_gray(nori_amd.film_variance(s, stats))
    assert np.allclose(out, nori_amd.denoise(img, var), rtol=1e-6, atol=1e-7)


def test_denoise_reproduces_reference_final_denoised(built):
    """nori_denoise (mode 0, the script's parameters) on the reference's
    final.png + final_variance.png against the reference's final_denoised.png:
    >= 99.99 % of the bytes equal and none off by more than 1 LSB (fp32 in the
    kernel against the script's float64)."""
    from test_denoise import compare_bytes, reference_triple

    img, var, ref = reference_triple("final", "final_variance", "final_denoised")
    out = nori_amd.denoise(img.astype(np.float32), var.astype(np.float32), radius=3, patch=3, k=0.02, mode=0,
                           script_scale=False)
    exact, dmax, _ = compare_bytes(out, ref)
    print(f"final_denoised: {exact * 100:.4f} % equal bytes, max {dmax} LSB")
    assert exact >= 0.9999 and dmax <= 1, (exact, dmax)
