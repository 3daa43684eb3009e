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


_staging = {}


def gather_frame(buf: "torch.Tensor", height: int, dist, rank: int, world: int, out=None, host: bool = False):
    """The single collective of a step: dist.gather of every rank's row buffer to rank 0,
    straight into slices of one cached (N, rows_max, W, 3) staging tensor, then the
    un-permute into `out` (rank 0) as one strided copy.  Returns the frame on rank 0,
    None elsewhere.  host=True (gloo, whose collectives take host tensors): each rank's rows
    go through host memory and rank 0 copies the assembled frame back into `out`."""
    import torch

    if host and buf.is_cuda:
        frame = gather_frame(buf.cpu(), height, dist, rank, world)
        if rank != 0:
            return None
        if out is None:
            return frame.to(buf.device)
        out.copy_(frame)
        return out
    if rank != 0:
        dist.gather(buf, gather_list=None, dst=0)
        return None
    key = (buf.device, buf.dtype, world, tuple(buf.shape))
    stage = _staging.get(key)
    if stage is None:
        stage = _staging[key] = torch.empty((world,) + tuple(buf.shape), dtype=buf.dtype, device=buf.device)
    dist.gather(buf, gather_list=list(stage.unbind(0)), dst=0)
    rmax, width = buf.shape[0], buf.shape[1]
    if out is None:
        return assemble(list(stage.unbind(0)), height).contiguous()
    if rmax * world == height:  # row y = compact row y // N of rank y % N
        out.view(rmax, world, width, 3).copy_(stage.transpose(0, 1))
    else:
        out.copy_(stage.transpose(0, 1).reshape(rmax * world, width, 3)[:height])
    return out
