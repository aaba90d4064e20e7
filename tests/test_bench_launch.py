"""bench.py's multi-GPU launch plan (CPU only): `bench.py --gpus N` without a
launcher starts torch.distributed.run with N processes itself, a rank of such
a job runs in place, and inconsistent requests are refused before any GPU
call."""
import importlib.util
import os
import sys

import pytest

from conftest import ROOT


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_single_gpu_runs_in_place():
    b = _bench()
    assert b.launch_plan(1, {}, 1, []) is None
    assert b.launch_plan(1, {}, 8, ["--steps", "3"]) is None


def test_n_gpus_without_launcher_spawns_torchrun():
    b = _bench()
    argv = ["--gpus", "4", "--steps", "7"]
    plan = b.launch_plan(4, {}, 8, argv, port=29555)
    assert plan[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in plan and "--nnodes=1" in plan
    assert "--master-addr=127.0.0.1" in plan and "--master-port=29555" in plan
    i = plan.index(os.path.join(ROOT, "bench.py"))
    assert plan[i + 1:] == argv  # the ranks see the same arguments (and WORLD_SIZE=4)


def test_rank_of_a_launched_job_runs_in_place():
    b = _bench()
    env = {"WORLD_SIZE": "8", "LOCAL_WORLD_SIZE": "8", "RANK": "3", "LOCAL_RANK": "3"}
    assert b.launch_plan(8, env, 8, []) is None


@pytest.mark.parametrize("gpus,env,devices", [
    (2, {"WORLD_SIZE": "4"}, 8),   # --gpus disagrees with the launcher
    (4, {"WORLD_SIZE": "4", "LOCAL_WORLD_SIZE": "4"}, 2),  # more local ranks than GPUs
    (8, {}, 1),                     # more GPUs than the node has
    (0, {}, 8),
])
def test_inconsistent_requests_are_refused(gpus, env, devices):
    b = _bench()
    with pytest.raises(SystemExit):
        b.launch_plan(gpus, env, devices, [])
