"""The trace launches' queue indexing (csrc/seg_index.h: seg_grid,
seg_group, seg_first, seg_entry -- the functions k_extend, k_shadow,
k_extend_scan and k_shadow_scan index the segmented queues with), compiled
for the host with g++: every index any thread of a launch loads is inside the
queue and inside its segment's count, and the live rays cover every queued
entry exactly once -- over empty, partial, full and trailing segments and
segment counts G that are not multiples of kTraceGroup (round 5's
illegal-access fault came from an index past G * kSeg of an empty group)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_seg_index_in_bounds(tmp_path):
    exe = tmp_path / "seg_index_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-I", os.path.join(ROOT, "nori-ray-tracer_amd", "csrc"),
                    os.path.join(ROOT, "tests", "seg_index_check.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-3000:]
    assert "0 failures" in r.stdout, r.stdout
