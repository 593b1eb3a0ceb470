"""Multi-GPU layout of the render path: one process per GPU.

Frames are independent units: frame f renders on rank f % world (C3, 1 frame per GPU)
with no data-path collective; the only exchange is one all-gather of the rendered
maps (depth, DINO, colour) so every rank (or rank 0) holds the full batch.  Within a
frame, contiguous row bands of the image can be rendered on different ranks (ray-tile
mode) -- each rank then owns a contiguous slice of the ray index r = (v H + y) W + x.

The reference has no multi-GPU inference path of its own (NeRFRenderer.bind_parallel
wraps torch DataParallel only when `gpus` is given, scenedino/renderer/nerf.py:641-658,
and no shipped caller passes it).  Works with any torch.distributed backend: "nccl"
(RCCL over xGMI) on the GPU box, "gloo" in the CPU tests.
"""
from __future__ import annotations

import torch


def frames_of_rank(n_frames: int, rank: int, world: int) -> list[int]:
    """Frames rendered by `rank` (round-robin: frame f -> rank f % world)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    return list(range(rank, n_frames, world))


def row_band(H: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous image rows [y0, y1) of `rank` in ray-tile mode (bands differ by <= 1 row)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    base, extra = divmod(H, world)
    y0 = rank * base + min(rank, extra)
    return y0, y0 + base + (1 if rank < extra else 0)


def pack_maps(coarse: dict) -> torch.Tensor:
    """Rendered maps of one frame -> one (R, 1 + D + 3 nv) float32 tensor
    [depth | dino_features | rgb] (one collective instead of three)."""
    depth = coarse["depth"].reshape(-1, 1)
    R = depth.shape[0]
    dino = coarse["dino_features"].reshape(R, -1)
    rgb = coarse["rgb"].reshape(R, -1)
    return torch.cat((depth.float(), dino.float(), rgb.float()), 1).contiguous()


def unpack_maps(maps: torch.Tensor, D: int) -> dict:
    return {"depth": maps[:, 0], "dino_features": maps[:, 1:1 + D], "rgb": maps[:, 1 + D:]}


def gather_maps(maps: torch.Tensor, group=None, out: list | None = None) -> list:
    """All-gather every rank's packed maps (same shape on all ranks): list[world]."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    bufs = out if out is not None else [torch.empty_like(maps) for _ in range(world)]
    dist.all_gather(bufs, maps, group=group)
    return bufs


def allreduce_grads(params, group=None) -> None:
    """Data-parallel training of the field head (frames sharded over ranks, the training
    path of scenedino_amd/autograd.py on each): average the parameter gradients with ONE
    all-reduce of a flat bucket (the ResnetFC's 46 k parameters are far below a ring's
    per-link latency floor, so one collective beats one per tensor).  Replaces what
    DistributedDataParallel does for the reference's trainer (base_trainer.py)."""
    import torch.distributed as dist
    ps = [p for p in params if p.grad is not None]
    if not ps:
        return
    world = dist.get_world_size(group)
    flat = torch.cat([p.grad.reshape(-1) for p in ps])
    dist.all_reduce(flat, group=group)
    flat /= world
    o = 0
    for p in ps:
        n = p.grad.numel()
        p.grad.copy_(flat[o:o + n].view_as(p.grad))
        o += n
