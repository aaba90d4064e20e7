"""The C-ABI boundary: libnori_gpu.so loads, exports every entry point that
include/nori_gpu.h declares, and the ctypes mirror matches the C layout."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import nori_amd
from nori_amd import _abi
from conftest import ROOT, scene_path

HEADER = os.path.join(ROOT, "include", "nori_gpu.h")


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(nori_[a-z_0-9]+)\s*\(", text, re.M)))


def test_library_exports_every_declared_symbol(built):
    names = declared_functions()
    assert len(names) >= 15
    lib = C.CDLL(_abi.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(_abi.SIGNATURES), set(names) ^ set(_abi.SIGNATURES)


def test_struct_layout_matches_c(built, tmp_path):
    structs = {"nori_shape_desc": _abi.ShapeDesc, "nori_bsdf_desc": _abi.BsdfDesc,
               "nori_emitter_desc": _abi.EmitterDesc, "nori_camera_desc": _abi.CameraDesc,
               "nori_medium_desc": _abi.MediumDesc, "nori_scene_desc": _abi.SceneDesc,
               "nori_gpu_render_desc": _abi.RenderDesc, "nori_gpu_stats": _abi.Stats,
               "nori_gpu_hit": _abi.Hit, "nori_image_desc": _abi.ImageDesc}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'printf("{cname}.{fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", str(src), "-o", str(exe)], check=True)
    out = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                         check=True).stdout.split("\n") if l)
    for cname, py in structs.items():
        assert int(out[cname]) == C.sizeof(py), cname
        for fname, _ in py._fields_:
            assert int(out[f"{cname}.{fname}"]) == getattr(py, fname).offset, (cname, fname)


def test_no_device_fails_loudly_or_renders(built):
    s = nori_amd.load_scene(scene_path("pa4", "cbox", "cbox_path_mis.xml"), 32, 32, 1)
    if nori_amd.device_count() == 0:
        with pytest.raises(nori_amd.NoriError) as e:
            nori_amd.GpuRenderer(s, 0)
        assert e.value.code == _abi.NORI_ERR_HIP


def test_write_exr_roundtrip_header(built, tmp_path):
    img = np.random.default_rng(0).random((5, 7, 3)).astype(np.float32)
    p = str(tmp_path / "x.exr")
    nori_amd.write_exr(p, img)
    data = open(p, "rb").read()
    assert data[:4] == b"\x76\x2f\x31\x01"
    # last scanline: y, size, then B, G, R planes of width floats
    w = 7
    line = np.frombuffer(data[-(8 + 12 * w):], dtype=np.float32, offset=8).reshape(3, w)
    assert np.array_equal(line[2], img[-1, :, 0]) and np.array_equal(line[0], img[-1, :, 2])
