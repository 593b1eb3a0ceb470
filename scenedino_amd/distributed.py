"""Multi-GPU layout of the render path: one process per GPU.

Frames are independent units: frame f renders on rank f % world (C3, 1 frame per GPU)
with no data-path collective; the only exchange is one all-gather of the rendered
maps (depth, DINO, colour) so every rank (or rank 0) holds the full batch.  The render
kernel writes its maps straight into packed [dino | depth | rgb] rows (BTSNet.render_into,
sd_render_args output strides; dino first so its 16-B stores stay aligned), which are the
send buffer of ONE all_gather_into_tensor into a preallocated (world, R, D + 1 + 3 nv)
receive buffer; MapGather double-buffers both
so that frame i's gather (RCCL's own stream) overlaps frame i+1's render.  Within a
frame, contiguous row bands of the image can be rendered on different ranks (ray-tile
mode) -- each rank then owns a contiguous slice of the ray index r = (v H + y) W + x.
The SSCBench voxel query (C5) shards by x-slabs of the voxel grid (slab_range,
query_voxels_slab in scenedino_amd/sscbench.py) and all-gathers the slabs the same way.

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
    """Rendered maps of one frame -> one (R, D + 1 + 3 nv) float32 tensor
    [dino_features | depth | rgb] (one collective instead of three; the row layout
    BTSNet.render_into writes)."""
    depth = coarse["depth"].reshape(-1, 1)
    R = depth.shape[0]
    dino = coarse["dino_features"].reshape(R, -1)
    rgb = coarse["rgb"].reshape(R, -1)
    return torch.cat((dino.float(), depth.float(), rgb.float()), 1).contiguous()


def unpack_maps(maps: torch.Tensor, D: int) -> dict:
    return {"depth": maps[:, D], "dino_features": maps[:, :D], "rgb": maps[:, D + 1:]}


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
    DistributedDataParallel does for the reference's trainer (base_trainer.py).  Every
    parameter that requires a gradient has a slot in the bucket (zeros where this rank
    produced no gradient), so the layout is identical on every rank; the bucket ends with
    one has-gradient flag per parameter, and a parameter no rank produced a gradient for
    keeps ``grad = None`` as under DDP (Adam skips it: no momentum step, no weight decay
    on learn_empty's vector or the salience downsampler on steps that do not use them)."""
    import torch.distributed as dist
    ps = [p for p in params if p.requires_grad]
    if not ps:
        return
    world = dist.get_world_size(group)
    dev = ps[0].device
    has = torch.tensor([0.0 if p.grad is None else 1.0 for p in ps], device=dev)
    flat = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1).to(dev)
                      for p in ps] + [has])
    dist.all_reduce(flat, group=group)
    # the flags are read back (one device sync) only when this rank lacks some gradient
    any_grad = ((flat[-len(ps):] > 0).tolist() if any(p.grad is None for p in ps)
                else [True] * len(ps))
    flat /= world
    o = 0
    for p, used in zip(ps, any_grad):
        n = p.numel()
        g = flat[o:o + n].view_as(p)
        if not used:
            p.grad = None
        elif p.grad is None:
            p.grad = g.clone()
        else:
            p.grad.copy_(g)
        o += n


class MapGather:
    """Asynchronous all-gather of every rank's packed rendered maps, ``depth`` slots deep.

    ``send(i)`` returns the (R, width) float32 send buffer of frame i (after waiting for
    the gather that last used that slot), ``start(i)`` launches the gather of frame i
    (all_gather_into_tensor into ``recv[i % depth]``, (world, R, width)), ``wait_all()``
    completes every outstanding gather.  With ``host_stage`` (gloo on one shared GPU: the
    dry-run of a multi-rank launch) the maps go through host memory synchronously."""

    def __init__(self, R: int, width: int, device, group=None, depth: int = 2,
                 host_stage: bool = False):
        import torch.distributed as dist
        self.dist, self.group, self.depth, self.host = dist, group, depth, host_stage
        self.world = dist.get_world_size(group)
        self._send = [torch.empty(R, width, device=device) for _ in range(depth)]
        rdev = "cpu" if host_stage else device
        self.recv = [torch.empty(self.world, R, width, device=rdev) for _ in range(depth)]
        self._work = [None] * depth

    def send(self, i: int) -> torch.Tensor:
        k = i % self.depth
        if self._work[k] is not None:
            self._work[k].wait()
            self._work[k] = None
        return self._send[k]

    def start(self, i: int) -> None:
        k = i % self.depth
        if self.host:
            h = self._send[k].cpu()
            self.dist.all_gather(list(self.recv[k].unbind(0)), h, group=self.group)
            return
        self._work[k] = self.dist.all_gather_into_tensor(self.recv[k], self._send[k],
                                                         group=self.group, async_op=True)

    def wait_all(self) -> None:
        for k in range(self.depth):
            if self._work[k] is not None:
                self._work[k].wait()
                self._work[k] = None
