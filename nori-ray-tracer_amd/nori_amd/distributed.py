"""Work sharding for several GPUs (one process per GPU).

Camera samples are independent, so a render shards without any data-path
collective; the only exchange is the final film sum -- the reference's
ImageBlock::put(block) merge (block.cpp:124-133).  Borders of neighbouring
32x32 blocks overlap, hence a sum (all_reduce), not a gather.

* pass sharding (weak scaling): rank r renders sample passes
  [r*spp, (r+1)*spp) of the same frame -- the per-GPU work is fixed.
* block sharding (strong scaling): rank r renders the blocks r, r+N, ... of
  the BlockGenerator's order for all passes.
"""


def pass_range(rank, spp):
    """(pass_begin, pass_count) of `rank` under pass sharding."""
    return rank * spp, spp


def block_subset(rank, world, num_blocks):
    """Block ids of `rank` under round-robin block sharding."""
    return list(range(rank, num_blocks, world))


def reduce_film(film, dist, group=None):
    """Sum the RGBW films of all ranks in place (RCCL on GPU tensors, gloo on CPU)."""
    dist.all_reduce(film, group=group)
    return film
