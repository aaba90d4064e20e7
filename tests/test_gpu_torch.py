"""GPU interop used by bench.py: the film and the per-pixel sample statistics
in torch-allocated device memory (device_ptr), and the library's own RCCL
film sum (nori_gpu_render_sharded) on a one-rank communicator.

These run in the pytest process after the other GPU tests' libnori_gpu
contexts: nori_amd maps PyTorch's HIP runtime before libnori_gpu
(nori_amd._abi._one_hip_runtime), so torch and the library share ONE
runtime.  (Round 1 had to run them in fresh processes: two runtimes were
mapped and torch's reported "No HIP GPUs are available".)"""
import os

import numpy as np
import pytest

import nori_amd
from conftest import scene_path
from nori_amd import distributed as nd

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _scene(name, w, h, spp):
    return nori_amd.load_scene(scene_path("pa4", "cbox", name), w, h, spp)


def test_one_hip_runtime_in_process(built):
    nori_amd.lib()
    torch.zeros(1, device="cuda:0")
    maps = {l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l}
    assert len(maps) == 1, maps
    rccl = nori_amd.lib().nori_gpu_comm_library()
    assert rccl is not None and os.path.dirname(rccl.decode()) == os.path.dirname(maps.pop()), rccl


def test_device_film(built):
    s = _scene("cbox_path_mis.xml", 64, 48, 4)
    with nori_amd.GpuRenderer(s, 0) as r:
        host = r.render()
        film = torch.zeros(s.film_shape(), dtype=torch.float32, device="cuda:0")
        torch.cuda.synchronize()
        r.render(device_ptr=film.data_ptr())
        torch.cuda.synchronize()
    assert np.allclose(film.cpu().numpy(), host, rtol=1e-4, atol=1e-4)


def test_variance_statistics_device_buffers(built):
    s = _scene("cbox_path_mats.xml", 32, 32, 8)
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


@pytest.mark.parametrize("mode", ["passes", "blocks"])
def test_render_sharded_one_rank(built, mode):
    """nori_gpu_render_sharded on a one-rank RCCL communicator: zeroes the
    film, renders the (whole) share and sums it in place = the plain render."""
    s = _scene("cbox_path_mis.xml", 80, 48, 6)
    comm = nd.FilmComm(nd.comm_id(), 1, 0, 0)
    with nori_amd.GpuRenderer(s, 0) as r:
        host = r.render()
        film = torch.full(s.film_shape(), 7.0, dtype=torch.float32, device="cuda:0")  # must be zeroed by the call
        torch.cuda.synchronize()
        r.render_sharded(comm, film.data_ptr(), mode=mode, root=0)
        torch.cuda.synchronize()
        assert r.last_stats["samples"] == 80 * 48 * 6
        r.render_sharded(comm, film.data_ptr(), mode=mode, root=-1)  # all-reduce form
        torch.cuda.synchronize()
    comm.close()
    assert np.allclose(film.cpu().numpy(), host, rtol=1e-4, atol=1e-4)


def test_render_sharded_rejects_variance(built):
    """Per-pixel statistics are not summed across ranks: a sharded render
    with variance_out set fails with NORI_ERR_INVALID before touching it."""
    s = _scene("cbox_path_mis.xml", 32, 32, 2)
    comm = nd.FilmComm(nd.comm_id(), 1, 0, 0)
    with nori_amd.GpuRenderer(s, 0) as r:
        film = torch.zeros(s.film_shape(), dtype=torch.float32, device="cuda:0")
        host_stats = np.zeros((s.height, s.width, 8), np.float32)
        with pytest.raises(nori_amd.NoriError) as e:
            r.render_sharded(comm, film.data_ptr(), variance=host_stats.ctypes.data)
        assert e.value.code == nori_amd._abi.NORI_ERR_INVALID
        r.render_sharded(comm, film.data_ptr())  # the communicator still works
        torch.cuda.synchronize()
    comm.close()


def test_render_sharded_cancel_returns_and_comm_survives(built):
    """nori_gpu_cancel during a sharded render: the rank still joins the status
    exchange (no hang), returns NORI_ERR_CANCELLED, and the communicator stays
    usable for the next frame."""
    import threading
    import time

    s = _scene("cbox_path_mis.xml", 2048, 2048, 512)
    comm = nd.FilmComm(nd.comm_id(), 1, 0, 0)
    with nori_amd.GpuRenderer(s, 0) as r:
        film = torch.zeros(s.film_shape(), dtype=torch.float32, device="cuda:0")
        torch.cuda.synchronize()
        err = []

        def run():
            try:
                r.render_sharded(comm, film.data_ptr())
            except nori_amd.NoriError as e:
                err.append(e)

        th = threading.Thread(target=run)
        t0 = time.time()
        th.start()
        # cancel once the render is under way (its progress moved), not after
        # a fixed sleep: a fast device could otherwise finish first
        while th.is_alive() and not 0.0 < r.progress() < 1.0 and time.time() - t0 < 30:
            time.sleep(0.002)
        cancelled_early = th.is_alive()
        r.cancel()
        th.join(timeout=60)
        assert not th.is_alive()
        if cancelled_early and r.progress() < 1.0:
            assert err and err[0].code == nori_amd._abi.NORI_ERR_CANCELLED, err
        else:  # the frame was done before the cancel landed: a normal finish
            assert not err or err[0].code == nori_amd._abi.NORI_ERR_CANCELLED, err
        assert time.time() - t0 < 30
        r.render_sharded(comm, film.data_ptr(), passes=2)
        torch.cuda.synchronize()
        assert r.last_stats["samples"] == 2048 * 2048 * 2
    comm.close()
