"""The C++ adapter of INTEGRATION.md (integration/nori_gpu_euler.cpp: the
reference's RenderThread + nori_euler written against include/nori_gpu.h
only), built by the package Makefile.

CPU: it links against libnori_gpu and, with no device, stops with the HIP
error (exit 4) after loading the scene.  GPU: it renders the Cornell box to an
EXR equal to the Python binding's render of the same passes and seed (same C
ABI, same streams; only the film's float summation order may differ)."""
import os
import subprocess

import numpy as np
import pytest

import nori_amd
from conftest import ROOT, scene_path

EXE = os.path.join(ROOT, "integration", "nori_gpu_euler")


def _run(*args, timeout=120):
    return subprocess.run([EXE, *args], capture_output=True, text=True, timeout=timeout)


def test_adapter_is_built_and_links(built):
    assert os.access(EXE, os.X_OK), "integration/nori_gpu_euler not built (make -C nori-ray-tracer_amd)"
    r = _run()
    assert r.returncode == 2 and "usage" in r.stderr


def test_adapter_reports_load_errors(built, tmp_path):
    r = _run(str(tmp_path / "missing.xml"))
    assert r.returncode == 1 and "loading the scene" in r.stderr


def test_adapter_without_device_fails_loudly(built, tmp_path):
    if nori_amd.device_count() > 0:
        pytest.skip("a device is present")
    r = _run(scene_path("pa4", "cbox", "cbox_path_mis.xml"), "--spp", "2", "--size", "32", "32",
             "--out", str(tmp_path / "x"))
    assert r.returncode == 4 and "no HIP device" in r.stderr


@pytest.mark.gpu
def test_adapter_renders_like_the_python_binding(built, tmp_path):
    xml = scene_path("pa4", "cbox", "cbox_path_mis.xml")
    r = _run(xml, "--spp", "8", "--size", "96", "72", "--png", "--out", str(tmp_path / "cbox"))
    assert r.returncode == 0, r.stderr
    assert "Rendering done: 55296 samples" in r.stdout
    img = nori_amd.read_exr(str(tmp_path / "cbox.exr"))
    assert os.path.getsize(tmp_path / "cbox.png") > 0
    s = nori_amd.load_scene(xml, 96, 72, 8)
    with nori_amd.GpuRenderer(s, 0) as g:
        ref = nori_amd.develop(s, g.render())
    assert img.shape == ref.shape
    assert np.abs(img - ref).max() < 1e-5, np.abs(img - ref).max()
