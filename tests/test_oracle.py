"""CPU oracle pinned against the reference's own fixtures (no GPU needed).

* pcg32 known-answer vector: ext/pcg32/pcg32-demo.out (tests/golden/pcg32_demo.json)
* Student-t scene tests: scenes/pa4/tests/test-furnace.xml, test-direct.xml
  (ttest.cpp:147-194, 100k paths, alpha = 0.01 Sidak-corrected)
* Student-t BSDF test: scenes/pa3/tests/ttest-microfacet.xml (ttest.cpp:107-145)
"""
import json
import os

import numpy as np
import pytest

import nori_amd
import pyoracle
from conftest import ROOT, scene_path
from nori_test_util import load_test_scenes, parse_test_xml, students_t_test

GOLDEN = os.path.join(ROOT, "tests", "golden")


def test_pcg32_known_answer(built):
    kat = json.load(open(os.path.join(GOLDEN, "pcg32_demo.json")))
    rng = pyoracle.Pcg32(*kat["seed"])
    number, suit = "A23456789TJQK", "hcds"
    for rnd in kat["rounds"]:
        assert [rng.next_uint() for _ in range(6)] == rnd["u32"]
        assert "".join("H" if rng.next_uint(2) else "T" for _ in range(65)) == rnd["coins"]
        assert [rng.next_uint(6) + 1 for _ in range(33)] == rnd["rolls"]
        cards = rng.shuffle(range(52))
        assert [number[c // 4] + suit[c % 4] for c in cards] == rnd["cards"]


def test_pcg32_float_is_mantissa_trick(built):
    # pcg32.h:101-110: float = bits((u >> 9) | 0x3f800000) - 1
    a, b = pyoracle.Pcg32(7, 11), pyoracle.Pcg32(7, 11)
    for _ in range(100):
        u = a.next_uint()
        f = np.frombuffer(np.uint32((u >> 9) | 0x3F800000).tobytes(), np.float32)[0] - np.float32(1)
        assert b.next_float() == f


@pytest.mark.parametrize("xml", ["test-furnace.xml", "test-direct.xml"])
def test_scene_ttests(built, tmp_path, xml):
    path = scene_path("pa4", "tests", xml)
    meta = parse_test_xml(path)
    scenes = load_test_scenes(path, tmp_path)
    refs = meta["references"]
    assert len(refs) == len(scenes)
    failures = []
    for (scene, integ), ref in zip(scenes, refs):
        o = pyoracle.OracleScene(scene)
        mean, var = o.ttest(meta["sampleCount"])
        ok, p = students_t_test(mean, var, ref, meta["sampleCount"], meta["significanceLevel"], len(refs))
        if not ok:
            failures.append((integ, ref, mean, p))
    assert not failures, failures


def test_microfacet_bsdf_ttest(built):
    path = scene_path("pa3", "tests", "ttest-microfacet.xml")
    meta = parse_test_xml(path)
    b = nori_amd._abi.BsdfDesc()
    p = meta["bsdf_props"]
    b.type = nori_amd._abi.BSDF_MICROFACET
    b.alpha = p["alpha"]
    b.int_ior = p["intIOR"]
    b.ext_ior = p["extIOR"]
    b.kd[:] = p["kd"]
    fails = []
    for ang, ref in zip(meta["angles"], meta["references"]):
        mean, var = pyoracle.bsdf_ttest(b, ang, meta["sampleCount"])
        ok, pv = students_t_test(mean, var, ref, meta["sampleCount"], meta["significanceLevel"], len(meta["references"]))
        if not ok:
            fails.append((ang, ref, mean, pv))
    assert not fails, fails


def test_wave_and_block_streams_agree_statistically(built):
    # Both RNG layouts estimate the same image; compare block means.
    s = nori_amd.load_scene(scene_path("pa4", "cbox", "cbox_path_mis.xml"), 64, 64, 16)
    o = pyoracle.OracleScene(s)
    a = nori_amd.develop(s, o.render(rng="wave"))
    b = nori_amd.develop(s, o.render(rng="block"))
    assert np.isfinite(a).all() and np.isfinite(b).all()
    ma, mb = a.mean(axis=(0, 1)), b.mean(axis=(0, 1))
    assert np.allclose(ma, mb, rtol=0.05), (ma, mb)


def test_pass_split_is_additive(built):
    s = nori_amd.load_scene(scene_path("pa4", "cbox", "cbox_path_mats.xml"), 48, 40, 4)
    o = pyoracle.OracleScene(s)
    whole = o.render(passes=4, rng="wave")
    part = o.render(passes=2, pass_begin=0, rng="wave")
    part = o.render(passes=2, pass_begin=2, rng="wave", out=part)
    assert np.allclose(whole, part, rtol=1e-5, atol=1e-5)


def test_block_subsets_tile_the_frame(built):
    s = nori_amd.load_scene(scene_path("pa4", "cbox", "cbox_path_mis.xml"), 70, 40, 2)
    o = pyoracle.OracleScene(s)
    whole = o.render(rng="wave")
    n = s.num_blocks()
    part = o.render(rng="wave", blocks=list(range(0, n, 2)))
    part = o.render(rng="wave", blocks=list(range(1, n, 2)), out=part)
    assert np.allclose(whole, part, rtol=1e-5, atol=1e-5)


def test_trace_closest_vs_bruteforce(built):
    # BVH traversal must return the closest of all primitive hits.
    s = nori_amd.load_scene(scene_path("pa4", "cbox", "cbox_path_mis.xml"), 32, 32, 1)
    o = pyoracle.OracleScene(s)
    rng = np.random.default_rng(3)
    n = 4000
    org = rng.uniform([-0.9, 0.05, -0.9], [0.9, 1.5, 0.9], size=(n, 3))
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.zeros((n, 8), np.float32)
    rays[:, :3], rays[:, 3], rays[:, 4:7], rays[:, 7] = org, 1e-4, d, np.inf
    hits = o.trace(rays)
    assert (hits["prim"] >= 0).mean() > 0.8  # the box is open towards the camera
    occl = o.trace(rays, any_hit=True)
    assert ((hits["prim"] >= 0) == (occl["prim"] >= 0)).all()
    # a shorter maxt than the hit distance must miss
    short = rays.copy()
    short[:, 7] = np.where(np.isfinite(hits["t"]), hits["t"] * 0.999, np.inf)
    h2 = o.trace(short)
    ok = np.isfinite(hits["t"]) & (hits["t"] > 2e-3)
    assert (h2["prim"][ok] == -1).mean() > 0.999
