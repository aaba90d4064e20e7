"""GPU output paths: the per-pixel sample statistics behind <stem>_variance.exr
(nori_gpu_render_desc.variance_out) against the oracle's per-sample radiance on
identical WAVE streams, and the `python -m nori_amd` command line (nori_euler)."""
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

import nori_amd
import pyoracle
from conftest import ROOT, scene_path

pytestmark = pytest.mark.gpu


def _oracle_stats(s):
    """(H, W, 8) sums of L, L^2 and the valid count from the oracle's per-sample radiance."""
    W, H, spp = s.width, s.height, s.spp
    ids = np.arange(spp * W * H, dtype=np.uint64)
    smp = pyoracle.OracleScene(s).wave_samples(ids)
    L = smp[:, 2:5].astype(np.float64).reshape(spp, H, W, 3)
    ok = np.all(np.isfinite(L) & (L >= 0), axis=-1, keepdims=True)
    L = np.where(ok, L, 0.0)
    st = np.zeros((H, W, 8))
    st[..., 0:3] = L.sum(0)
    st[..., 3:6] = (L * L).sum(0)
    st[..., 6] = ok[..., 0].sum(0)
    return st


@pytest.mark.parametrize("xml,size", [(("pa4", "cbox", "cbox_path_mis.xml"), (40, 36, 16)),
                                      (("pa3", "odyssey", "odyssey_mis.xml"), (48, 27, 8))])
def test_variance_statistics_match_oracle(built, xml, size):
    s = nori_amd.load_scene(scene_path(*xml), *size)
    st = np.zeros((s.height, s.width, 8), np.float32)
    with nori_amd.GpuRenderer(s, 0) as r:
        r.render(variance=st)
    want = _oracle_stats(s)
    assert np.array_equal(st[..., 6], want[..., 6])  # same valid samples per pixel
    assert np.allclose(st[..., 0:6], want[..., 0:6], rtol=2e-3, atol=2e-3)
    var = nori_amd.film_variance(s, st)
    assert np.isfinite(var).all() and (var >= 0).all() and var.max() > 0


# device-memory statistics (torch tensors): tests/test_gpu_torch.py::test_variance_statistics_device_buffers


def test_cli_writes_exr_variance_png(built, tmp_path):
    src = os.path.dirname(scene_path("pa4", "cbox", "cbox_path_mis.xml"))
    dst = tmp_path / "cbox"
    shutil.copytree(src, dst)
    xml = str(dst / "cbox_path_mis.xml")
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "nori-ray-tracer_amd"))
    p = subprocess.run([sys.executable, "-m", "nori_amd", xml, "--width", "64", "--height", "48", "--spp", "16",
                        "--png"], capture_output=True, text=True, env=env, timeout=120)
    assert p.returncode == 0, p.stderr
    assert "Rendering .. done." in p.stdout
    img = nori_amd.read_exr(str(dst / "cbox_path_mis.exr"))
    var = nori_amd.read_exr(str(dst / "cbox_path_mis_variance.exr"))
    assert img.shape == (48, 64, 3) and var.shape == (48, 64, 3)
    assert img.mean() > 0.05 and (var >= 0).all()
    assert open(dst / "cbox_path_mis.png", "rb").read(4) == b"\x89PNG"
