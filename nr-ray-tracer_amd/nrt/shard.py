"""Row sharding of one frame over N ranks.

Rank r renders image rows y = r, r + N, r + 2N, ... (interleaving spreads the
Cornell box's light and ceiling rows over every GPU); each rank's rows are
compact in a (rows_max, W, 3) buffer, padded to rows_max = ceil(H / N) so that
all ranks contribute equal-sized buffers to one gather.  The RNG is keyed by
pixel index, so the assembled frame is bitwise identical for every N.
"""
from typing import List


def rows_max(height: int, world: int) -> int:
    return (height + world - 1) // world


def rows_of(height: int, rank: int, world: int) -> int:
    """Number of image rows rank renders (= nrt_rows_selected with offset rank, stride world)."""
    return 0 if rank >= height else (height - rank + world - 1) // world


def assemble(gathered: List["torch.Tensor"], height: int) -> "torch.Tensor":
    """gathered[r] = rank r's (rows_max, W, 3) buffer -> the (H, W, 3) frame: row y comes from
    rank y % N, compact row y // N.  Works on any device (one stack + view + copy)."""
    import torch

    world = len(gathered)
    rmax, width = gathered[0].shape[0], gathered[0].shape[1]
    return torch.stack(gathered, 0).transpose(0, 1).reshape(rmax * world, width, 3)[:height]


def gather_frame(buf: "torch.Tensor", height: int, dist, rank: int, world: int, out=None):
    """The single collective of a step: dist.gather of every rank's row buffer to rank 0,
    then the un-permute into `out` (rank 0).  Returns the frame on rank 0, None elsewhere."""
    import torch

    parts = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, gather_list=parts, dst=0)
    if rank != 0:
        return None
    frame = assemble(parts, height)
    if out is None:
        return frame.contiguous()
    out.copy_(frame)
    return out
