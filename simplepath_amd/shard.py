"""Tile sharding across ranks and the frame-end gather.

The reference renders one frame with N threads pulling tiles from one ColumnMajorTileScheduler
(main.cpp:109-130).  Here each GPU (one process per GPU, torch.distributed over RCCL) owns the
tiles `shard_tiles(rank, world)` -- the scheduler's order dealt round-robin, which spreads cheap
(sky) and expensive (geometry) tiles evenly -- renders them with no collective, and one
`gather` at frame end brings every rank's tile-packed radiance to rank 0, which scatters it into
scheduler order (the input of sp_tiles_to_image / Image)."""
from __future__ import annotations

import numpy as np


def shard_tiles(n_tiles: int, rank: int, world: int) -> np.ndarray:
    """Tile indices owned by `rank` of `world` (ColumnMajorTileScheduler order, interleaved)."""
    return np.arange(rank, n_tiles, world, dtype=np.int32)


def per_rank_capacity(n_tiles: int, world: int) -> int:
    """Tiles in the largest shard: every rank's gather buffer has this many 64x3 slots."""
    return (n_tiles + world - 1) // world


def gather_frame(local_tiles, n_tiles: int, rank: int, world: int, dist, gathered=None, frame=None,
                 collective: bool = False):
    """Collect the tile buffers of all ranks on rank 0.

    local_tiles: torch tensor [per_rank_capacity, 64, 3] holding this rank's shard in shard order
    (a CUDA tensor under the nccl = RCCL backend, a CPU tensor under gloo).
    Returns, on rank 0, `frame` [n_tiles, 64, 3] in scheduler order (allocated if not given);
    None elsewhere.  `gathered` may be a preallocated list of `world` tensors shaped like
    local_tiles (rank 0 only).  With world == 1 the copy is local unless `collective` is set
    (then the same dist.gather runs over the one-rank group: device tests of the RCCL path)."""
    import torch

    if world == 1 and not collective:
        if frame is None:
            return local_tiles[:n_tiles]
        frame.copy_(local_tiles[:n_tiles])
        return frame
    if rank == 0 and gathered is None:
        gathered = [torch.empty_like(local_tiles) for _ in range(world)]
    dist.gather(local_tiles, gathered if rank == 0 else None, dst=0)
    if rank != 0:
        return None
    if frame is None:
        frame = torch.empty((n_tiles, 64, 3), dtype=local_tiles.dtype, device=local_tiles.device)
    for r in range(world):
        k = len(range(r, n_tiles, world))
        frame[r::world] = gathered[r][:k]
    return frame
