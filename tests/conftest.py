import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "nori-ray-tracer_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

SCENES = os.path.join(ROOT, "scenes")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libnori_gpu.so on cuda:0)")


@pytest.fixture(scope="session")
def built():
    """Build the product library and the oracle once per session."""
    import subprocess

    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "nori-ray-tracer_amd")], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    return True


def scene_path(*parts):
    return os.path.join(SCENES, *parts)
