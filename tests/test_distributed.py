"""CPU (gloo, world size 2) tests of the multi-GPU layout in scenedino_amd/distributed.py:
frame / row-band sharding covers every unit exactly once and the all-gather of packed
rendered maps returns every rank's frame in rank order."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from scenedino_amd import distributed as sdd


def test_frames_and_row_bands_partition():
    for world in (1, 2, 3, 8):
        frames = sorted(f for r in range(world) for f in sdd.frames_of_rank(8, r, world))
        assert frames == list(range(8))
        rows = []
        for r in range(world):
            y0, y1 = sdd.row_band(192, r, world)
            rows += list(range(y0, y1))
        assert rows == list(range(192))
    with pytest.raises(ValueError):
        sdd.row_band(192, 2, 2)


def test_pack_unpack_roundtrip():
    R, D, nv = 50, 64, 1
    c = {"depth": torch.rand(1, R), "dino_features": torch.rand(1, R, D),
         "rgb": torch.rand(1, R, 3 * nv)}
    m = sdd.pack_maps(c)
    assert m.shape == (R, D + 1 + 3)
    u = sdd.unpack_maps(m, D)
    assert torch.equal(u["depth"], c["depth"].reshape(R))
    assert torch.equal(u["dino_features"], c["dino_features"].reshape(R, D))
    assert torch.equal(u["rgb"], c["rgb"].reshape(R, 3))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, R, D, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        frames = sdd.frames_of_rank(world, rank, world)
        assert frames == [rank]
        g = torch.Generator().manual_seed(100 + rank)
        c = {"depth": torch.rand(1, R, generator=g), "dino_features": torch.rand(1, R, D, generator=g),
             "rgb": torch.rand(1, R, 3, generator=g)}
        got = sdd.gather_maps(sdd.pack_maps(c))
        ok = True
        for r in range(world):
            g2 = torch.Generator().manual_seed(100 + r)
            ref = {"depth": torch.rand(1, R, generator=g2),
                   "dino_features": torch.rand(1, R, D, generator=g2),
                   "rgb": torch.rand(1, R, 3, generator=g2)}
            ok &= torch.equal(got[r], sdd.pack_maps(ref))
        dist.barrier()
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_gather_maps_gloo_world2():
    world, R, D = 2, 300, 64
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, R, D, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = dict(q.get(timeout=10) for _ in range(world))
    assert res == {0: True, 1: True}


def _grad_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lin = torch.nn.Linear(5, 3)
        g = torch.Generator().manual_seed(rank)
        lin.weight.grad = torch.randn(3, 5, generator=g)
        b = torch.randn(3, generator=g)
        lin.bias.grad = b if rank == 0 else None  # rank 1 produced no bias gradient
        unused = torch.nn.Parameter(torch.zeros(4))  # no gradient on any rank (DDP: stays None)
        sdd.allreduce_grads(list(lin.parameters()) + [unused])
        ws, bs = [], []
        for r in range(world):
            g2 = torch.Generator().manual_seed(r)
            ws.append(torch.randn(3, 5, generator=g2))
            b2 = torch.randn(3, generator=g2)
            bs.append(b2 if r == 0 else torch.zeros(3))
        ok = torch.allclose(lin.weight.grad, sum(ws) / world, atol=1e-6) and \
            torch.allclose(lin.bias.grad, sum(bs) / world, atol=1e-6) and unused.grad is None
        dist.barrier()
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_allreduce_grads_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grad_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = dict(q.get(timeout=10) for _ in range(world))
    assert res == {0: True, 1: True}


def _spawn(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    return dict(q.get(timeout=10) for _ in range(world))


def _mapgather_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        R, width = 40, 68
        mg = sdd.MapGather(R, width, "cpu", depth=2, host_stage=True)
        ok = True
        for i in range(5):  # frames i: rank r's maps = f(r, i)
            buf = mg.send(i)
            buf.copy_(torch.full((R, width), 100.0 * rank + i))
            mg.start(i)
            got = mg.recv[i % 2]
            for r in range(world):
                ok &= bool((got[r] == 100.0 * r + i).all())
        mg.wait_all()
        dist.barrier()
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_map_gather_host_stage_gloo_world2():
    assert _spawn(_mapgather_worker, 2) == {0: True, 1: True}


def _slab_predict(p):
    """A deterministic stand-in for the field + head (GPU-free): sigma and class of a
    voxel centre from its coordinates."""
    sig = torch.sin(3.1 * p[:, 0]) + torch.cos(1.7 * p[:, 1]) * p[:, 2]
    seg = ((p[:, 0] * 7 + p[:, 1] * 3).floor().remainder(19)).to(torch.uint8)
    return sig, seg


def _slab_worker(rank, world, port, q):
    import torch.distributed as dist
    from scenedino_amd import sscbench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dims = (16, 6, 5)
        g = torch.Generator().manual_seed(3)
        pts = torch.rand(dims[0] * dims[1] * dims[2], 3, generator=g) * 4 - 2
        # CPU stand-ins for the field query and the grow (sd_grow3's parity vs max_pool3d is
        # tests/test_seg.py::test_grow3_equals_max_pool3d): this test is the halo logic
        pool = lambda t: torch.nn.functional.max_pool3d(t.unsqueeze(0), 3, 1, 1).squeeze(0)
        sig, seg = sscbench.query_voxels_slab(_slab_predict, pts, dims, rank, world, grow_fn=pool)
        full_s, full_g = sscbench.gather_slabs(sig, seg, dims)
        # unsharded reference: the whole grid, grown by the 3x3x3 max-pool
        rs, rg = _slab_predict(pts)
        rs = torch.nn.functional.max_pool3d(rs.reshape(1, *dims), 3, 1, 1).reshape(dims)
        ok = torch.equal(full_s, rs) and torch.equal(full_g, rg.reshape(dims))
        dist.barrier()
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_voxel_slabs_gloo_world2_equal_unsharded():
    assert _spawn(_slab_worker, 2) == {0: True, 1: True}


def test_slab_range_partition():
    from scenedino_amd import sscbench
    for world in (1, 2, 3, 8):
        xs = []
        for r in range(world):
            a, b = sscbench.slab_range(256, r, world)
            xs += list(range(a, b))
        assert xs == list(range(256))
    assert sscbench.slab_range(256, 3, 8) == (96, 128)
