"""GPU: the C3 multi-rank path (frame f on rank f, rendered straight into the packed
[depth | dino | rgb] send buffer, all-gathered) reproduces single-process renders bit for
bit.  Two rank processes share cuda:0 (the box has one GPU) and gather through host
memory over gloo -- the same MapGather / BTSNet.render_into path bench.py runs over RCCL."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu

R = 192 * 640
WIDTH = 1 + 64 + 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _render(frame, into, band=None):
    sys.path.insert(0, ROOT)
    import bench
    net, _, wrapper, sampler, pose, Ks = bench.make_scene(frame, torch.device("cuda:0"), "bf16",
                                                          offset_pose=True)
    net.render_into = into
    torch.manual_seed(1234)  # the renderer's z-jitter seed
    with torch.no_grad():
        bench.render_step(net, wrapper, sampler, pose, Ks, band)
    torch.cuda.synchronize()


def _worker(rank, world, port, out_path, rows=False):
    import torch.distributed as dist
    from scenedino_amd import distributed as sdd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if rows:  # one frame's row bands (ray-tile sharding)
            y0, y1 = sdd.row_band(192, rank, world)
            band = (y0 * 640, y1 * 640)
            mg = sdd.MapGather(band[1] - band[0], WIDTH, torch.device("cuda:0"), depth=1, host_stage=True)
            _render(0, mg.send(0), band)
        else:
            mg = sdd.MapGather(R, WIDTH, torch.device("cuda:0"), depth=1, host_stage=True)
            _render(rank, mg.send(0))
        mg.start(0)
        mg.wait_all()
        if rank == 0:
            torch.save(mg.recv[0].clone(), out_path)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_two_ranks_gather_equals_single_process(tmp_path):
    out = str(tmp_path / "gathered.pt")
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    got = torch.load(out, weights_only=True)
    assert tuple(got.shape) == (2, R, WIDTH)
    for f in range(2):
        ref = torch.empty(R, WIDTH, device="cuda:0")
        _render(f, ref)
        assert torch.equal(got[f], ref.cpu()), f"frame {f} differs"
    assert not torch.equal(got[0], got[1])


def test_two_ranks_row_bands_equal_whole_frame(tmp_path):
    """Ray-tile sharding (north star; SURVEY §8(e) rows 24 g .. 24 g + 23 at 8 GPUs): two
    ranks render the two row bands of ONE frame (the in-kernel depth jitter keyed by the
    frame ray index), the gathered bands equal the single-process whole-frame render."""
    out = str(tmp_path / "bands.pt")
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, out, True)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    got = torch.load(out, weights_only=True)
    assert tuple(got.shape) == (2, R // 2, WIDTH)
    ref = torch.empty(R, WIDTH, device="cuda:0")
    _render(0, ref)
    assert torch.equal(got.reshape(R, WIDTH), ref.cpu())
