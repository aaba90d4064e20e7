"""Test helpers: the reference's statistical harness restated in Python.

students_t_test  <- hypothesis::students_t_test (ext/hypothesis/hypothesis.h:314-345)
parse_test_xml   <- StudentsTTest property parsing (src/ttest.cpp:60-80)
load_test_scenes <- <test type="ttest"> children: each <scene> is written to its
                    own XML next to the original so relative OBJ paths resolve.
"""
import os
import xml.etree.ElementTree as ET

import numpy as np
from scipy import stats

import nori_amd


def students_t_test(mean, variance, reference, n, alpha, num_tests):
    t = abs(mean - reference) * np.sqrt(n / max(variance, 1e-5))
    p = 2 * (1 - stats.t.cdf(t, n - 1))
    sidak = 1.0 - (1.0 - alpha) ** (1.0 / num_tests)
    ok = not (p < sidak or not np.isfinite(p))
    return ok, p


def _floats(s):
    return [float(x) for x in s.replace(",", " ").split()]


def parse_test_xml(path):
    root = ET.parse(path).getroot()
    out = {"sampleCount": 100000, "significanceLevel": 0.01, "angles": [], "references": []}
    for ch in root:
        name = ch.get("name")
        if ch.tag == "string" and name in ("references", "angles"):
            out[name] = _floats(ch.get("value"))
        elif ch.tag == "integer" and name == "sampleCount":
            out["sampleCount"] = int(ch.get("value"))
        elif ch.tag == "float" and name == "significanceLevel":
            out["significanceLevel"] = float(ch.get("value"))
        elif ch.tag == "bsdf":
            props = {}
            for p in ch:
                v = p.get("value")
                props[p.get("name")] = _floats(v) if p.tag == "color" else float(v)
            out["bsdf_props"] = props
            out["bsdf_type"] = ch.get("type")
    return out


def load_test_scenes(path, tmpdir, width=0, height=0, spp=0):
    """Return [(Scene, integrator name)] for every <scene> child of a test XML."""
    root = ET.parse(path).getroot()
    base = os.path.dirname(os.path.abspath(path))
    res = []
    for i, sc in enumerate([c for c in root if c.tag == "scene"]):
        # rewrite relative filenames to absolute so the temp XML can live anywhere
        for s in sc.iter("string"):
            if s.get("name") == "filename" and not os.path.isabs(s.get("value")):
                s.set("value", os.path.join(base, s.get("value")))
        p = os.path.join(str(tmpdir), f"scene_{i}.xml")
        ET.ElementTree(sc).write(p)
        scene = nori_amd.load_scene(p, width, height, spp)
        res.append((scene, scene.integrator))
    return res
