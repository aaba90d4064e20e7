"""GPU interop used by bench.py --gpus N: the film (and the per-pixel sample
statistics) live in torch tensors on the device (device_ptr), and the
cross-rank sum goes through RCCL.  Each check runs in a fresh process with
torch initialised first (tests/torch_worker.py explains why)."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("check", ["device_film", "device_variance", "rccl_reduce"])
def test_torch_interop(built, check):
    pytest.importorskip("torch")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "torch_worker.py"), check],
                       capture_output=True, text=True, timeout=150)
    assert p.returncode == 0 and p.stdout.strip().endswith("ok"), p.stdout[-2000:] + p.stderr[-4000:]
