"""GPU: the multi-rank paths reproduce single-process results bit for bit.

* C3 (frame f on rank f, rendered straight into the packed [dino | depth | rgb] send buffer,
  all-gathered) and ray-tile bands of one frame: two rank processes share cuda:0 (the box
  has one GPU) and gather through host memory over gloo -- the same MapGather /
  BTSNet.render_into path bench.py runs over RCCL.
* C5 x-slabs (evaluate_model_sscbench.py:675-756): two ranks on cuda:0 each run
  query_voxels_slab through the real kernels (sd_field_query -> sd_seg_query -> sd_grow3),
  gather_slabs equals the single-process query_voxels, bf16 and fp8.
* The RCCL branch of MapGather (host_stage=False: all_gather_into_tensor(async_op=True) on
  the "nccl" backend, double-buffered waits): world 1 on the one GPU.
Rank processes are always reaped (terminate / kill after the join timeout)."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu

R = 192 * 640
WIDTH = 64 + 1 + 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_ranks(target, world, *args, timeout=300):
    """Start ``world`` spawn processes target(rank, world, port, *args), join them, and reap
    any still alive after ``timeout`` (so a hung rank never keeps the GPU for later
    tests).  Returns the exit codes."""
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + args) for r in range(world)]
    try:
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout)
    finally:
        for p in procs:
            if p.is_alive():
                p.terminate()
                p.join(10)
            if p.is_alive():
                p.kill()
                p.join(10)
    return [p.exitcode for p in procs]


def _init(rank, world, port, backend="gloo"):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    if backend == "nccl":
        dist.init_process_group(backend, rank=rank, world_size=world,
                                device_id=torch.device("cuda:0"))
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    return dist


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
    from scenedino_amd import distributed as sdd
    dist = _init(rank, world, port)
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
    assert _run_ranks(_worker, 2, out) == [0, 0]
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
    assert _run_ranks(_worker, 2, out, True) == [0, 0]
    got = torch.load(out, weights_only=True)
    assert tuple(got.shape) == (2, R // 2, WIDTH)
    ref = torch.empty(R, WIDTH, device="cuda:0")
    _render(0, ref)
    assert torch.equal(got.reshape(R, WIDTH), ref.cpu())


def _c5(precision):
    sys.path.insert(0, ROOT)
    import bench
    return bench.c5_scene(torch.device("cuda:0"), precision, 0)


def _slab_worker(rank, world, port, out_path, precision):
    from scenedino_amd import sscbench
    dist = _init(rank, world, port)
    try:
        net, pts, dims = _c5(precision)

        def predict(p):  # the per-slab call bench.py's C5 path makes (sd_field_query + sd_seg_query)
            sig, seg = net.predict_voxels(p.reshape(1, -1, 3), voxel_size=sscbench.VOXEL_SIZE)
            return sig.reshape(-1), seg.reshape(-1)

        with torch.no_grad():
            sig, seg = sscbench.query_voxels_slab(predict, pts, dims, rank, world)  # sd_grow3
            full_s, full_g = sscbench.gather_slabs(sig.cpu(), seg.cpu(), dims)  # gloo: host
        if rank == 0:
            torch.save({"sigma": full_s, "seg": full_g}, out_path)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("precision", ["bf16", "fp8"])
def test_c5_xslabs_real_kernels_equal_unsharded(tmp_path, precision):
    from scenedino_amd import sscbench
    out = str(tmp_path / f"slabs_{precision}.pt")
    assert _run_ranks(_slab_worker, 2, out, precision) == [0, 0]
    got = torch.load(out, weights_only=True)
    net, pts, dims = _c5(precision)
    with torch.no_grad():
        ref_s, ref_g = sscbench.query_voxels(net, pts, dims)
    assert tuple(got["sigma"].shape) == tuple(dims)
    assert torch.equal(got["sigma"], ref_s.cpu())
    assert torch.equal(got["seg"], ref_g.cpu())
    assert int(ref_g.cpu().unique().numel()) > 2  # a non-degenerate class map


def _rccl_worker(rank, world, port, out_path):
    from scenedino_amd import distributed as sdd
    dist = _init(rank, world, port, backend="nccl")
    try:
        assert dist.get_backend() == "nccl"
        mg = sdd.MapGather(R, WIDTH, torch.device("cuda:0"), depth=2, host_stage=False)
        for i in range(3):  # frame 2 reuses slot 0: send(2) waits for frame 0's gather
            _render(i, mg.send(i))
            mg.start(i)
            assert mg._work[i % 2] is not None  # the async RCCL work handle
        mg.wait_all()
        torch.save({"f1": mg.recv[1].cpu().clone(), "f2": mg.recv[0].cpu().clone()}, out_path)
    finally:
        dist.destroy_process_group()


def test_rccl_map_gather_world1(tmp_path):
    """MapGather's non-host branch on RCCL (world 1 on the one GPU): the async
    all_gather_into_tensor slots hold frames 1 and 2 (frame 2 in the slot frame 0 was
    gathered into, after send(2) waited on that gather) bit-equal to single-process renders."""
    if torch.cuda.device_count() != 1:
        pytest.skip("world-1 RCCL rehearsal is for the one-GPU box")
    out = str(tmp_path / "rccl.pt")
    env_keep = os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"  # dmabuf IPC (the host driver's only mode)
    try:
        assert _run_ranks(_rccl_worker, 1, out, timeout=240) == [0]
    finally:
        if env_keep is None:
            os.environ.pop("HSA_ENABLE_IPC_MODE_LEGACY", None)
        else:
            os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = env_keep
    got = torch.load(out, weights_only=True)
    for f, t in ((1, got["f1"]), (2, got["f2"])):
        ref = torch.empty(R, WIDTH, device="cuda:0")
        _render(f, ref)
        assert tuple(t.shape) == (1, R, WIDTH)
        assert torch.equal(t[0], ref.cpu()), f"frame {f} differs"
