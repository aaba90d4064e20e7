"""Several GPUs of one node, one process per GPU (nori_gpu_comm_* in the C ABI).

Camera samples are independent, so a frame shards without a data-path
collective.  The only exchange is the final film sum -- the reference's
ImageBlock::put(block) merge (block.cpp:124-133), summed because the borders
of neighbouring 32x32 blocks overlap -- done by libnori_gpu itself with RCCL
over xGMI on the render stream (nori_gpu_render_sharded).

Shard modes (nori_gpu_shard_desc, the same C code on every rank):
* "passes" (default): rank r renders passes [P r/N, P (r+1)/N) of the whole
  frame.  Every (pass, pixel) sample owns its random stream, so the summed
  film equals the single-GPU film up to float summation order, and every rank
  gets the same work (no tile-cost imbalance).
* "blocks": rank r renders blocks r, r+N, ... of the BlockGenerator's spiral
  order (block.cpp:140-188), all passes.

Strong scaling: the frame (W x H x spp) is fixed and split over the ranks.

The communicator id is 128 opaque bytes made by rank 0; any byte channel
delivers it (here: torch.distributed's object broadcast, on gloo).
"""
import ctypes as C

import numpy as np

from . import _abi
from ._abi import check, lib


def comm_id():
    """A fresh communicator id (ncclGetUniqueId), rank 0 only."""
    buf = (C.c_ubyte * _abi.COMM_ID_BYTES)()
    check(lib().nori_gpu_comm_id(buf))
    return bytes(buf)


class FilmComm:
    """RCCL communicator of this process's GPU (nori_gpu_comm_create; collective)."""

    def __init__(self, id_bytes, nranks, rank, device):
        assert len(id_bytes) == _abi.COMM_ID_BYTES
        buf = (C.c_ubyte * _abi.COMM_ID_BYTES).from_buffer_copy(id_bytes)
        h = C.c_void_p()
        check(lib().nori_gpu_comm_create(buf, int(nranks), int(rank), int(device), C.byref(h)))
        self.handle, self.nranks, self.rank, self.device = h, nranks, rank, device

    def ranks(self):
        """(nranks, rank) as the library's communicator reports them (nori_gpu_comm_rank)."""
        n, r = C.c_int(), C.c_int()
        check(lib().nori_gpu_comm_rank(self.handle, C.byref(n), C.byref(r)))
        return n.value, r.value

    def close(self):
        if self.handle is not None and self.handle.value:
            lib().nori_gpu_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def film_comm(dist, device):
    """FilmComm over the ranks of an initialised torch.distributed group:
    rank 0's id reaches the others through broadcast_object_list."""
    obj = [comm_id() if dist.get_rank() == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return FilmComm(obj[0], dist.get_world_size(), dist.get_rank(), device)


def shard(scene, rank, world, mode="passes", passes=None, pass_begin=0, blocks=None):
    """This rank's (pass_begin, pass_count, block ids or None) -- nori_gpu_shard_desc."""
    rd = _abi.RenderDesc()
    rd.pass_begin = int(pass_begin)
    rd.pass_count = int(scene.spp if passes is None else passes)
    ids = None
    if blocks is not None:
        ids = np.ascontiguousarray(np.asarray(blocks, dtype=np.uint32))
        rd.num_blocks = ids.size
        rd.block_ids = ids.ctypes.data_as(C.POINTER(C.c_uint32))
    out = _abi.RenderDesc()
    buf = np.zeros(max(scene.num_blocks(), 1), np.uint32)
    check(lib().nori_gpu_shard_desc(scene.desc_ptr, C.byref(rd), _abi.SHARD_MODES[mode], int(world), int(rank),
                                    C.byref(out), buf.ctypes.data_as(C.POINTER(C.c_uint32))))
    sel = buf[:out.num_blocks].tolist() if out.num_blocks else None
    if mode == "blocks" and sel is None:
        sel = []
    return out.pass_begin, out.pass_count, sel
