"""BVH build: the library's host build (nori_scene_bvh_info,
the same code nori_gpu_create runs; subtrees of >= 16k primitives on their own
threads) against the oracle's serial restatement of BVH::build -- identical
reference-layout node count, BVH::statistics SAH cost and leaf order."""
import pytest

import nori_amd
import pyoracle
import synth
from conftest import scene_path


def _compare(s):
    g = nori_amd.bvh_info(s)
    n, sah, h = pyoracle.OracleScene(s).bvh_stats()
    assert g["ref_nodes"] == n
    assert g["sah_cost"] == sah
    assert g["order_hash"] == h
    return g


@pytest.mark.parametrize("parts", [("pa4", "cbox", "cbox_path_mis.xml"), ("pa4", "table", "table_path_mis.xml"),
                                   ("project", "volumetric", "volumetric.xml")])
def test_bvh_matches_oracle(built, parts):
    g = _compare(nori_amd.load_scene(scene_path(*parts), 32, 32, 1))
    assert g["device_nodes"] >= 1 and g["depth"] <= 64


def test_parallel_build_deterministic(built, tmp_path):
    """131k triangles: the top of the tree is built on several threads."""
    s = nori_amd.load_scene(synth.heightfield_scene(str(tmp_path), n=256, width=32, height=32, spp=1))
    a = nori_amd.bvh_info(s)
    b = nori_amd.bvh_info(s)
    assert a == b
    assert a["num_prims"] == 2 * 256 * 256 + 12 + 0  # height field + cbox walls and light
    _compare(s)
