"""Diagnostic: two ranks of nori_gpu_render_sharded on ONE GPU (RCCL with both
ranks on device 0).  Prints the outcome; exits 0 whether RCCL accepts it or not."""
import os
import socket
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nori-ray-tracer_amd"))
SCENE = os.path.join(ROOT, "scenes", "pa4", "cbox", "cbox_path_mis.xml")
W, H, SPP = 80, 48, 6


def worker(rank, world, port, out_dir):
    sys.path.insert(0, os.path.join(ROOT, "nori-ray-tracer_amd"))
    import torch
    import torch.distributed as dist

    import nori_amd
    from nori_amd import distributed as nd

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    comm = nd.film_comm(dist, 0)  # both ranks on device 0
    scene = nori_amd.load_scene(SCENE, W, H, SPP)
    with nori_amd.GpuRenderer(scene, 0) as r:
        for mode in ("passes", "blocks"):
            film = torch.full(scene.film_shape(), 3.0, dtype=torch.float32, device="cuda:0")
            torch.cuda.synchronize()
            r.render_sharded(comm, film.data_ptr(), mode=mode, root=-1)
            torch.cuda.synchronize()
            np.save(os.path.join(out_dir, f"{mode}_{rank}.npy"), film.cpu().numpy())
    dist.barrier()
    comm.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    import torch.multiprocessing as mp

    import nori_amd

    scene = nori_amd.load_scene(SCENE, W, H, SPP)
    with nori_amd.GpuRenderer(scene, 0) as r:
        ref = r.render()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    d = tempfile.mkdtemp()
    try:
        mp.start_processes(worker, args=(2, port, d), nprocs=2, join=True, start_method="spawn")
    except Exception as e:  # RCCL may refuse two ranks on one device
        print("probe: two ranks on one GPU not possible:", str(e)[-400:])
        sys.exit(0)
    for mode in ("passes", "blocks"):
        for rank in (0, 1):
            got = np.load(os.path.join(d, f"{mode}_{rank}.npy"))
            print("probe:", mode, rank, "max |diff|", float(np.abs(got - ref).max()), "allclose", np.allclose(got, ref, rtol=1e-5, atol=1e-5))
