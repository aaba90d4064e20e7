"""The scene-specialised scan kernels (csrc/rtc.hip): the library's embedded
scan sources compile through hipRTC for gfx950 with a scene's scan list as
literals (no device needed), for the headline Cornell box and for a scene
with 18 wall pairs; a BVH scene has nothing to specialise.  Parity of the
specialised kernels with the oracle is the GPU suite's (they are the default
for scan-mode scenes; NORI_RTC=0 restores the generic ones)."""
import pytest

import nori_amd
from conftest import scene_path


@pytest.mark.parametrize("parts", [("pa4", "cbox", "cbox_path_mis.xml"), ("pa3", "odyssey", "odyssey_mis.xml")],
                         ids=["cbox", "odyssey"])
def test_scan_rtc_compiles(built, parts, tmp_path, monkeypatch):
    monkeypatch.setenv("NORI_RTC_CACHE", str(tmp_path))  # a cold cache: really compile
    s = nori_amd.load_scene(scene_path(*parts), 32, 32, 1)
    try:
        n, ms = nori_amd.scan_rtc(s, "gfx950")
    except nori_amd.NoriError as e:
        if "libhiprtc not found" in str(e):
            pytest.skip("hipRTC is not installed")
        raise
    assert n > 10000 and ms > 0.0
    assert len(list(tmp_path.glob("scan_*.co"))) == 1
    n2, ms2 = nori_amd.scan_rtc(s, "gfx950")  # the process cache
    assert n2 == n and ms2 < ms


def test_scan_rtc_bvh_scene(built):
    s = nori_amd.load_scene(scene_path("pa1", "sphere-mesh.xml"), 32, 32, 1)
    assert len(nori_amd.scan_list(s)["records"]) == 0  # a BVH scene
    assert nori_amd.scan_rtc(s, "gfx950") == (0, 0.0)
