"""Interpreter exit with live Scene objects (and a module-level one) prints
nothing: Scene.__del__ and GpuRenderer.close must not touch module globals
that Python may already have torn down (nori_amd/__init__.py)."""
import os
import subprocess
import sys

from conftest import ROOT, scene_path

SCRIPT = r"""
import sys
import nori_amd
keep = nori_amd.load_scene(sys.argv[1], 16, 16, 1)
scenes = [nori_amd.load_scene(sys.argv[1], 16, 16, 1) for _ in range(3)]
nori_amd.load_scene(sys.argv[1], 16, 16, 1)   # freed at once


class Holder:  # a reference cycle: collected only by the final collection, after the modules are cleared
    pass


h = Holder()
h.me, h.scene = h, nori_amd.load_scene(sys.argv[1], 16, 16, 1)
nori_amd.__dict__["_cycle"] = h   # also reachable from the package itself
del h
print("ok")
if len(sys.argv) > 2:  # an uncaught exception: its traceback keeps a frame with a Scene until the very end
    def fail():
        scene = nori_amd.load_scene(sys.argv[1], 16, 16, 1)
        raise RuntimeError("boom")
    fail()
"""


def test_exit_with_live_scenes_is_clean(built):
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "nori-ray-tracer_amd"))
    r = subprocess.run([sys.executable, "-c", SCRIPT, scene_path("pa4", "cbox", "cbox_path_mis.xml")], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr
    assert r.stderr.strip() == "", r.stderr


def test_exit_after_uncaught_exception_is_clean(built):
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "nori-ray-tracer_amd"))
    r = subprocess.run([sys.executable, "-c", SCRIPT, scene_path("pa4", "cbox", "cbox_path_mis.xml"), "raise"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 1 and "RuntimeError: boom" in r.stderr, r.stderr
    assert "Exception ignored" not in r.stderr and "AttributeError" not in r.stderr, r.stderr


def test_del_does_not_need_module_globals(built, monkeypatch):
    """What interpreter teardown does (module globals set to None, as seen on a
    GPU box with torch loaded): Scene.__del__ / GpuRenderer.close still work."""
    import nori_amd

    s = nori_amd.load_scene(scene_path("pa4", "cbox", "cbox_path_mis.xml"), 16, 16, 1)
    monkeypatch.setattr(nori_amd, "_abi", None)
    monkeypatch.setattr(nori_amd, "lib", None)
    s.__del__()
    assert s._h is None
