"""Torch-interop checks run in a fresh process (tests/test_gpu_torch.py).

torch initialises its HIP context first, then libnori_gpu -- the order of
bench.py's multi-GPU path.  (In a process where a libnori_gpu context was
created and destroyed before torch's first CUDA call, torch's lazy init
reports "No HIP GPUs are available" on this image, so these checks do not
share the pytest process with the other GPU tests.)

usage: python tests/torch_worker.py <check>   (exit status 0 = pass)
"""
import os
import socket
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(ROOT, "nori-ray-tracer_amd")]
torch.zeros(1, device="cuda:0")  # torch's context first
import nori_amd  # noqa: E402


def scene(name, w, h, spp):
    return nori_amd.load_scene(os.path.join(ROOT, "scenes", "pa4", "cbox", name), w, h, spp)


def device_film():
    s = scene("cbox_path_mis.xml", 64, 48, 4)
    with nori_amd.GpuRenderer(s, 0) as r:
        host = r.render()
        film = torch.zeros(s.film_shape(), dtype=torch.float32, device="cuda:0")
        torch.cuda.synchronize()
        r.render(device_ptr=film.data_ptr())
        torch.cuda.synchronize()
    assert np.allclose(film.cpu().numpy(), host, rtol=1e-4, atol=1e-4)


def device_variance():
    s = scene("cbox_path_mats.xml", 32, 32, 8)
    with nori_amd.GpuRenderer(s, 0) as r:
        host = np.zeros((s.height, s.width, 8), np.float32)
        r.render(variance=host)
        film = torch.zeros(s.film_shape(), dtype=torch.float32, device="cuda:0")
        st = torch.zeros((s.height, s.width, 8), dtype=torch.float32, device="cuda:0")
        torch.cuda.synchronize()
        r.render(device_ptr=film.data_ptr(), variance=st.data_ptr())
        torch.cuda.synchronize()
    assert np.allclose(st.cpu().numpy(), host, rtol=1e-4, atol=1e-4)
    assert (host[..., 6] == 8).all()


def rccl_reduce():
    import torch.distributed as dist
    from nori_amd import distributed as nd

    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        s = scene("cbox_path_mats.xml", 32, 32, 2)
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


if __name__ == "__main__":
    {"device_film": device_film, "device_variance": device_variance, "rccl_reduce": rccl_reduce}[sys.argv[1]]()
    print("ok")
