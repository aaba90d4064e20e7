"""Multi-process sharding on CPU (gloo): the split bench.py --gpus N and
nori_gpu_render_sharded use (nori_gpu_shard_desc, the library's C code),
with the oracle as each rank's renderer and a gloo all_reduce in place of the
RCCL film sum.  The summed film must equal the single-process render of the
whole frame (same WAVE streams; only the float summation order differs)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, scene_path

SCENE = scene_path("pa4", "cbox", "cbox_path_mis.xml")
W, H, SPP = 80, 48, 5  # 3x2 blocks (ragged last column), 5 passes: uneven splits


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
    scene = nori_amd.load_scene(SCENE, W, H, SPP)
    pb, pc, blocks = nd.shard(scene, rank, world, mode)
    film = np.zeros(scene.film_shape(), np.float32)
    if pc:
        pyoracle.OracleScene(scene).render(passes=pc, pass_begin=pb, rng="wave", blocks=blocks, threads=2, out=film)
    t = torch.from_numpy(film)
    dist.all_reduce(t)  # the film sum nori_gpu_render_sharded does over RCCL
    if rank == 0:
        np.save(out_path, t.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("mode", ["passes", "blocks"])
def test_sharded_frame_matches_single_process(built, tmp_path, mode, world):
    import nori_amd
    import pyoracle

    out = str(tmp_path / "film.npy")
    mp.start_processes(_worker, args=(world, _free_port(), mode, out), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(out)
    scene = nori_amd.load_scene(SCENE, W, H, SPP)
    ref = pyoracle.OracleScene(scene).render(rng="wave")
    assert np.allclose(got, ref, rtol=1e-5, atol=1e-5)


def test_shard_partitions_the_frame(built):
    """Every (pass, block) of the frame is in exactly one rank's share, for
    more ranks than passes or blocks too (empty shares)."""
    import nori_amd
    from nori_amd import distributed as nd

    scene = nori_amd.load_scene(SCENE, W, H, SPP)
    nb = scene.num_blocks()
    for mode in ("passes", "blocks"):
        for world in (1, 2, 3, 4, 7, 9):
            seen = np.zeros((SPP, nb), np.int32)
            for r in range(world):
                pb, pc, blocks = nd.shard(scene, r, world, mode)
                for b in (range(nb) if blocks is None else blocks):
                    seen[pb:pb + pc, b] += 1
            assert (seen == 1).all(), (mode, world)
    # restricted frame: a block subset split again over the ranks
    sub = [0, 2, 5]
    got = sorted(b for r in range(2) for b in nd.shard(scene, r, 2, "blocks", blocks=sub)[2])
    assert got == sub
    assert nd.shard(scene, 1, 2, "passes", passes=4, pass_begin=10)[:2] == (12, 2)


def test_shard_block_lists_are_checked_and_deduplicated(built):
    """Both modes check a restricting block list against the frame and drop
    repeated ids, so a share never overflows the caller's block buffer (one
    entry per frame block); the pass count defaults to the scene's spp."""
    import nori_amd
    from nori_amd import distributed as nd

    scene = nori_amd.load_scene(SCENE, W, H, SPP)
    nb = scene.num_blocks()
    dup = [1, 4, 1, 4, 4, 0] * 3
    pb, pc, blocks = nd.shard(scene, 0, 2, "passes", blocks=dup)
    assert (pb, pc) == (0, SPP // 2) and blocks == [1, 4, 0]
    got = sorted(b for r in range(3) for b in nd.shard(scene, r, 3, "blocks", blocks=dup)[2])
    assert got == [0, 1, 4]
    for mode in ("passes", "blocks"):
        with pytest.raises(nori_amd.NoriError):
            nd.shard(scene, 0, 2, mode, blocks=[0, nb])
    assert nd.shard(scene, 1, 2, "passes", passes=0)[:2] == (SPP // 2, SPP - SPP // 2)


def test_status_word_encoding(built):
    """The status exchange's word (runtime.hip comm_status_word): severity << 16
    | rank, reduced by max -- the worst outcome wins and names its rank."""
    from nori_amd import _abi
    f = _abi.lib().nori_gpu_comm_status_word
    assert f(_abi.NORI_OK, 3) == 3
    assert f(_abi.NORI_ERR_CANCELLED, 5) == (1 << 16) | 5
    for rc in (_abi.NORI_ERR_INVALID, _abi.NORI_ERR_HIP, _abi.NORI_ERR_OOM, _abi.NORI_ERR_IO):
        assert f(rc, 7) == (2 << 16) | 7
    words = [f(_abi.NORI_OK, 0), f(_abi.NORI_ERR_CANCELLED, 1), f(_abi.NORI_OK, 2)]
    assert max(words) >> 16 == 1 and max(words) & 0xFFFF == 1
    words.append(f(_abi.NORI_ERR_OOM, 2))
    assert max(words) >> 16 == 2 and max(words) & 0xFFFF == 2
    assert f(_abi.NORI_OK, 65535) == 65535


def test_comm_timeout_scales_with_the_share(built, monkeypatch):
    """Watchdog bound of the sharded collectives after a rendered share:
    max(30 s, 20 x own render time x largest share / own share); 600 s
    without a share; the env wins."""
    from nori_amd import _abi
    monkeypatch.delenv("NORI_COMM_TIMEOUT_S", raising=False)
    f = _abi.lib().nori_gpu_comm_timeout
    ok = _abi.NORI_OK
    assert f(ok, 0.03, 1e6, 1e6) == 30.0           # a 30 ms frame: the 30 s floor
    assert f(ok, 10.0, 1e6, 1e6) == 200.0          # 20x a 10 s share
    assert f(ok, 10.0, 1e6, 2e6) == 400.0          # a peer holds twice the samples
    assert f(ok, 10.0, 2e6, 1e6) == 200.0          # never below the own share's bound
    assert f(ok, 0.0, 0.0, 1e6) == 600.0           # no share: no own time to scale
    monkeypatch.setenv("NORI_COMM_TIMEOUT_S", "5")
    assert f(ok, 10.0, 1e6, 1e6) == 5.0
    assert f(_abi.NORI_ERR_CANCELLED, 0.01, 1e6, 1e6) == 5.0


def test_comm_timeout_of_a_failed_or_cancelled_rank(built, monkeypatch):
    """A rank whose own render threw (own time never measured: 0) or was
    cancelled early (a truncated time) must not fall to the 30 s floor or to
    a bound scaled from that time: its peers may render for much longer, so it
    keeps the fixed 600 s bound."""
    from nori_amd import _abi
    monkeypatch.delenv("NORI_COMM_TIMEOUT_S", raising=False)
    f = _abi.lib().nori_gpu_comm_timeout
    for rc in (_abi.NORI_ERR_CANCELLED, _abi.NORI_ERR_OOM, _abi.NORI_ERR_INVALID, _abi.NORI_ERR_HIP):
        assert f(rc, 0.0, 1e6, 1e6) == 600.0       # threw before its time was taken
        assert f(rc, 0.5, 1e6, 1e6) == 600.0       # cancelled after 0.5 s
        assert f(rc, 100.0, 1e6, 1e6) == 600.0     # never a bound scaled from a failed share
