"""GPU interop used by bench.py --gpus N: the film lives in a torch tensor on
the device (device_ptr), and the cross-rank sum goes through RCCL."""
import os
import socket

import numpy as np
import pytest

import nori_amd
from conftest import scene_path

pytestmark = pytest.mark.gpu


def test_device_pointer_film_matches_host(built):
    torch = pytest.importorskip("torch")
    s = nori_amd.load_scene(scene_path("pa4", "cbox", "cbox_path_mis.xml"), 64, 48, 4)
    with nori_amd.GpuRenderer(s, 0) as r:
        host = r.render()
        film = torch.zeros(s.film_shape(), dtype=torch.float32, device="cuda:0")
        torch.cuda.synchronize()
        r.render(device_ptr=film.data_ptr())
        torch.cuda.synchronize()
    assert np.allclose(film.cpu().numpy(), host, rtol=1e-4, atol=1e-4)


def test_rccl_single_rank_film_reduce(built):
    torch = pytest.importorskip("torch")
    import torch.distributed as dist
    from nori_amd import distributed as nd

    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        s = nori_amd.load_scene(scene_path("pa4", "cbox", "cbox_path_mats.xml"), 32, 32, 2)
        film = torch.zeros(s.film_shape(), dtype=torch.float32, device="cuda:0")
        with nori_amd.GpuRenderer(s, 0) as r:
            pb, pc = nd.pass_range(0, 2)
            r.render(passes=pc, pass_begin=pb, device_ptr=film.data_ptr())
        before = film.clone()
        nd.reduce_film(film, dist)
        torch.cuda.synchronize()
        assert torch.equal(before, film)
        assert float(film[..., 3].sum()) > 0
    finally:
        dist.destroy_process_group()
