"""Multi-process sharding on CPU (gloo, world size 2): the same logic bench.py
runs over RCCL, with the oracle as the per-rank renderer."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, scene_path

SCENE = scene_path("pa4", "cbox", "cbox_path_mis.xml")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mode, out_path):
    import sys

    for p in (os.path.join(ROOT, "nori-ray-tracer_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import nori_amd
    import pyoracle
    from nori_amd import distributed as nd

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    scene = nori_amd.load_scene(SCENE, 64, 48, 2)
    o = pyoracle.OracleScene(scene)
    if mode == "passes":
        pb, pc = nd.pass_range(rank, 2)
        film = o.render(passes=pc, pass_begin=pb, rng="wave", threads=2)
    else:
        film = o.render(passes=4, rng="wave", blocks=nd.block_subset(rank, world, scene.num_blocks()), threads=2)
    t = torch.from_numpy(film)
    nd.reduce_film(t, dist)
    if rank == 0:
        np.save(out_path, t.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["passes", "blocks"])
def test_two_rank_sharding_matches_single_process(built, tmp_path, mode):
    import nori_amd
    import pyoracle

    out = str(tmp_path / "film.npy")
    mp.start_processes(_worker, args=(2, _free_port(), mode, out), nprocs=2, join=True, start_method="spawn")
    got = np.load(out)
    scene = nori_amd.load_scene(SCENE, 64, 48, 2)
    ref = pyoracle.OracleScene(scene).render(passes=4, rng="wave")
    assert np.allclose(got, ref, rtol=1e-5, atol=1e-5)
