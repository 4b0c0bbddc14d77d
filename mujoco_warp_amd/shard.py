"""World sharding across GPUs (one process per GPU, no collective on the data path).

Worlds never interact, so a node-level run is a set of
independent shards: rank r owns global world ids [offset, offset + count).
The only cross-rank operations are the timing barrier and a max/sum of scalars
(bench.py).  `world_offset` feeds the Halton index of the benchmark control
noise so a sharded run reproduces the single-GPU sequence world for world.
"""


def weak_shard(nworld_per_rank: int, rank: int):
  """Weak scaling: every rank owns nworld_per_rank worlds."""
  return rank * nworld_per_rank, nworld_per_rank


def strong_shard(nworld_total: int, rank: int, nranks: int):
  """Strong scaling: split nworld_total as evenly as possible (first ranks take the remainder)."""
  base, rem = divmod(nworld_total, nranks)
  count = base + (1 if rank < rem else 0)
  offset = rank * base + min(rank, rem)
  return offset, count
