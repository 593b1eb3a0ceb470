#!/usr/bin/env python3
"""bench.py -- rendered rays/s on KITTI-360-shaped frustums (BASELINE.json metric).

Workload (BASELINE.json configs[1]): one 192x640 frame per GPU,
64 samples/ray (7,864,320 points), ViT-S/16-shaped 256x192x640 feature grid,
ResnetFC 295->128->65 (random kaiming init), lindisp stratified sampling, bf16.
A "step" = ImageRaySampler.sample (sd_gen_rays) -> the frame's device-side state
(sd_pack_image, sd_cam_records) -> projected grid P = W_in G + b_in (sd_project_grid) ->
fused render (sd_render_proj: LDS-staged tile kernel + overflow fallback; z sampling,
points, projection, code, P gather, MFMA MLP, colours, alpha compositing).  The C2 step is
timed at two render poses, the encoder view and a 0.5 m lateral / 2 deg yaw offset view
(SURVEY §8(d)); ``value`` is the slower of the two.  For N > 1 every rank renders its own
frame (C3: frames sharded 1-per-GPU) straight into packed [dino | depth | rgb] rows that
are all-gathered over RCCL (all_gather_into_tensor, overlapped with the next frame).
The ViT/DPT encoder is not part of the timed step (separate scope row, ``end_to_end``).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--precision bf16|fp32]
--gpus N > 1 without a torchrun environment launches N rank processes itself
(torch.distributed.run, 127.0.0.1) before touching the GPU; under torchrun WORLD_SIZE must
equal N.  --dist-backend gloo: ranks share one GPU and gather through host memory (a
dry run of the multi-rank path on a one-GPU box).  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

H, W, K_SAMPLES = 192, 640, 64
# diagnostic A/B only (default on: demo_script asks for per-sample weights and alphas)
WANT_SAMPLES = os.environ.get("SCENEDINO_AMD_BENCH_NO_SAMPLES") != "1"
C_GRID, HF, WF = 256, 192, 640
KITTI_K = [[0.7849, 0.0, -0.0312], [0.0, 2.9391, 0.2701], [0.0, 0.0, 1.0]]
PEAK_TFLOPS = {"bf16": 2500.0, "fp16": 2500.0, "fp32": 157.3,   # MI355X dense MFMA
               "fp8": 5000.0}                                    # (MI355X_MICROARCH.md)
D_HIDDEN, D_DINO = 128, 64
D_IN = C_GRID + 39


def mlp_flops_per_point(D=None):
    D = D_DINO if D is None else D
    return 2 * (D_IN * D_HIDDEN + D_HIDDEN * (1 + D))


class FixedGridEncoder(torch.nn.Module):
    def __init__(self, grid):
        super().__init__()
        self.register_buffer("grid", grid)
        self.latent_size = grid.shape[1]
        self.extra_outs = 0

    def forward(self, x, ground_truth=False):
        return [self.grid]


GRID_LAYOUT = "nhwc"  # --grid-layout: the native encoder's DPT writes channels-last grids


def _layout(grid):
    """The synthetic grid in the layout the native encoder delivers (channels-last, a
    (B, C, H, W) view of NHWC storage) or, --grid-layout nchw, the reference's NCHW."""
    return grid.contiguous(memory_format=torch.channels_last) if GRID_LAYOUT == "nhwc" else grid


def make_scene(frame_seed: int, device, precision="bf16", offset_pose=False, grid_hw=None):
    """Synthetic inputs of SURVEY.md §8(d): image U[-1,1) (seed frame), grid N(0,1)
    (seed 1+frame), MLP kaiming (seed 2).  grid_hw: (Hf, Wf) of the feature grid
    (default 192x640, ViT-S/16 + DPT; C5 uses ViT-B/8's 384x1280)."""
    from scenedino_amd.models import BTSNet
    from scenedino_amd.models.prediction_heads import ResnetFC
    from scenedino_amd.common.positional_encoding import PositionalEncoding
    from scenedino_amd.renderer import NeRFRenderer
    from scenedino_amd.common.ray_sampler import ImageRaySampler

    g = torch.Generator().manual_seed(frame_seed)
    images = (torch.rand(1, 1, 3, H, W, generator=g) * 2 - 1).to(device)
    hf, wf = grid_hw if grid_hw is not None else (HF, WF)
    grid = _layout(torch.randn(1, C_GRID, hf, wf,
                               generator=torch.Generator().manual_seed(1 + frame_seed)))
    torch.manual_seed(2)
    head = ResnetFC(d_in=D_IN, d_out=1 + D_DINO, n_blocks=0, d_hidden=D_HIDDEN)
    conf = {"predict_dino": True, "dino_dims": D_DINO, "learn_empty": False, "code_mode": "z",
            "inv_z": True, "z_near": 3, "z_far": 80, "sample_color": True, "precision": precision}
    net = BTSNet(conf, FixedGridEncoder(grid), PositionalEncoding(6, 3, 1.5, True),
                 {"normal_head": head}, final_pred_head="normal_head").to(device).eval()
    Ks = torch.tensor(KITTI_K, device=device).view(1, 1, 3, 3)
    poses = torch.eye(4, device=device).view(1, 1, 4, 4)
    net.encode(images, Ks, poses, ids_encoder=[0], ids_render=[0])
    render_pose = offset_render_pose(poses) if offset_pose else poses.clone()
    renderer = NeRFRenderer(n_coarse=K_SAMPLES, lindisp=True, hard_alpha_cap=False,
                            eval_batch_size=65536)
    wrapper = renderer.bind_parallel(net, gpus=None).eval()
    sampler = ImageRaySampler(z_near=3, z_far=80, height=H, width=W)
    return net, renderer, wrapper, sampler, render_pose, Ks


def end_to_end(args, device, rank):
    """Whole frame through make_model's native encoder (BASELINE configs[1]: DINO
    ViT-S/16 -> DPT -> 256x192x640 grid, random weights) then the C2 render: BTSNet.encode
    (the gt-encoder pass stays deferred, nothing reads grid_l_loss_features at inference)
    + ImageRaySampler + NeRFRenderer.  Reported beside the render-only `value`; SURVEY
    §8(d) prices the encoder separately."""
    from scenedino_amd.models import make_model
    from scenedino_amd.renderer import NeRFRenderer
    from scenedino_amd.common.ray_sampler import ImageRaySampler
    enc = dict(type="dinov2", mode="downsample-prediction", decoder_arch="dpt",
               downsampler_arch="featup", encoder_arch="vit-s", version="v1_16",
               separate_gt_version=None, encoder_freeze=True, flip_avg_gt=False,
               dim_reduction_arch="mlp", num_ch_enc=[64, 64, 128, 256],
               intermediate_features=[3, 6, 9], decoder_out_dim=256, dino_pca_dim=64,
               image_size=[H, W], key_features=False)
    conf = {"arch": "BTSNet", "predict_dino": True, "dino_dims": D_DINO, "learn_empty": False,
            "code_mode": "z", "inv_z": True, "z_near": 3, "z_far": 80, "sample_color": True,
            "encoder": enc, "code": {"num_freqs": 6, "freq_factor": 1.5, "include_input": True},
            "decoder_heads": [{"type": "resnet", "name": "normal_head", "freeze": False,
                               "args": {"n_blocks": 0, "d_hidden": D_HIDDEN}}],
            "final_prediction_head": "normal_head", "precision": args.precision}
    torch.manual_seed(2)
    net = make_model(conf).to(device).eval()
    g = torch.Generator().manual_seed(rank)
    images = (torch.rand(1, 1, 3, H, W, generator=g) * 2 - 1).to(device)
    Ks = torch.tensor(KITTI_K, device=device).view(1, 1, 3, 3)
    poses = torch.eye(4, device=device).view(1, 1, 4, 4)
    wrapper = NeRFRenderer(n_coarse=K_SAMPLES, lindisp=True, hard_alpha_cap=False,
                           eval_batch_size=65536).bind_parallel(net, gpus=None).eval()
    sampler = ImageRaySampler(z_near=3, z_far=80, height=H, width=W)

    def frame():
        net.encode(images, Ks, poses, ids_encoder=[0], ids_render=[0])
        return render_step(net, wrapper, sampler, poses, Ks)

    with torch.no_grad():
        for _ in range(args.warmup):
            frame()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            frame()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
    del net
    torch.cuda.empty_cache()
    return {"encoder": "DINO ViT-S/16 + DPT (make_model native encoder, random weights)",
            "ms_per_frame": dt * 1e3, "rays_per_s": H * W / dt}


def render_step(net, wrapper, sampler, pose, Ks, band=None, want_weights=True, want_alphas=True):
    """One C2 frame: rays of the render pose, then the fused render -- with per-sample
    weights and alphas, as demo_script's render call asks for them
    (demo_utils/utils.py:223).  band = (r0, r1): only rays [r0, r1) of the frame (ray-tile
    sharding; the renderer keys its in-kernel depth jitter by the frame ray index, so the
    band matches the whole-frame render)."""
    net._grid_cache = None  # re-pack / re-project the (freshly encoded) grid every frame
    rays, _ = sampler.sample(None, pose, Ks)
    if band is not None:
        rays = rays[:, band[0]:band[1]]
        wrapper.renderer.ray_offset = band[0]
    return wrapper(rays, want_weights=want_weights, want_alphas=want_alphas)


class KernelTimer:
    """HIP events around named kernel launches (BTSNet.kernel_timer hook), recorded on
    the stream the kernels are launched on (torch's current stream).  Events go around
    the kernels of every ``every``-th timed step (``tick()`` after each step): a timing
    event between two kernels costs the stream a 5-13 us bubble (rocprofv3 trace), which
    sampling keeps out of most timed frames (SCENEDINO_AMD_TIMER_EVERY, default 4)."""

    def __init__(self, every=None):
        self.pairs = {}
        self.on = False
        self.every = max(1, int(every if every is not None
                                else os.environ.get("SCENEDINO_AMD_TIMER_EVERY", "4")))
        self._k = 0

    def tick(self):
        self._k += 1

    @property
    def _live(self):
        return self.on and self._k % self.every == 0

    def start(self, name):
        if self._live:
            e = torch.cuda.Event(enable_timing=True)
            e.record(torch.cuda.current_stream())
            self.pairs.setdefault(name, []).append([e, None])

    def stop(self, name):
        if self._live:
            e = torch.cuda.Event(enable_timing=True)
            e.record(torch.cuda.current_stream())
            self.pairs[name][-1][1] = e

    def mean_ms(self, name):
        ts = [a.elapsed_time(b) for a, b in self.pairs.get(name, [])]
        return sum(ts) / len(ts) if ts else 0.0


def offset_render_pose(pose):
    """The 0.5 m lateral / 2 deg yaw render pose of SURVEY §8(d) (second timed run)."""
    import math
    p = pose.clone()
    a = math.radians(2.0)
    p[..., 0, 0] = math.cos(a); p[..., 0, 2] = math.sin(a)
    p[..., 2, 0] = -math.sin(a); p[..., 2, 2] = math.cos(a)
    p[..., 0, 3] = 0.5
    return p


def host_cpus() -> dict:
    """os.cpu_count(), the affinity mask's CPUs and the cgroup CPU quota (cgroup v2
    cpu.max or v1 cfs quota / period); usable = the smallest of them."""
    import math
    n = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        try:
            q = float(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = float(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    # the job's CPU share as the GPU box states it (OMP_NUM_THREADS is set to it there)
    try:
        share = int(os.environ.get("OMP_NUM_THREADS", "0")) or None
    except ValueError:
        share = None
    usable = min(v for v in (n, aff, math.ceil(quota) if quota else None, share) if v)
    return {"cpu_count": n, "affinity": aff, "quota": quota, "share": share,
            "usable": max(1, usable)}


def cpu_baseline(budget_s: float = 20.0, offset_pose: bool = True):
    """Oracle (pure-PyTorch CPU restatement of the reference, fp32) on the host cores:
    renders whole image rows of the same C2 frame (rays from the offset render pose, as
    the reported GPU value) until ~budget_s of CPU work, on every host CPU this process
    may use (SURVEY §8(d) asks for os.cpu_count(); that is capped by the affinity mask, the
    cgroup CPU quota and the job's CPU share (OMP_NUM_THREADS, 16 on the one-GPU box of
    a 256-CPU host): 256 threads there measured 203 rays/s, oversubscribed, 50x slower
    than 16; SD_CPU_THREADS overrides)."""
    from oracle import render_oracle as O

    threads = int(os.environ.get("SD_CPU_THREADS", host_cpus()["usable"]))
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    images = torch.rand(1, 1, 3, H, W, generator=g) * 2 - 1
    grid = torch.randn(1, C_GRID, HF, WF, generator=torch.Generator().manual_seed(1))
    torch.manual_seed(2)
    from scenedino_amd.models.prediction_heads import ResnetFC
    head = ResnetFC(d_in=D_IN, d_out=1 + D_DINO, n_blocks=0, d_hidden=D_HIDDEN)
    Kn = torch.tensor(KITTI_K)
    pose = torch.eye(4)
    ray_pose = offset_render_pose(pose) if offset_pose else pose
    rays = O.gen_rays(ray_pose.view(1, 4, 4), Kn.view(1, 3, 3), H, W)
    w2c = torch.inverse(pose).view(1, 4, 4)
    imgs = (images * 0.5 + 0.5)
    args = (grid, w2c, Kn.view(1, 3, 3), imgs, w2c.view(1, 1, 4, 4), Kn.view(1, 1, 3, 3),
            head.lin_in.weight.detach(), head.lin_in.bias.detach(), head.lin_out.weight.detach(),
            head.lin_out.bias.detach())
    rows_per_chunk = 4
    done_rays = 0
    # warm-up on one chunk
    u = torch.rand(rows_per_chunk * W, K_SAMPLES, generator=torch.Generator().manual_seed(3))
    with torch.no_grad():
        O.render(rays[: rows_per_chunk * W], u, *args, sb=1)
        t0 = time.perf_counter()
        row = 0
        while row < H and time.perf_counter() - t0 < budget_s:
            sl = slice(row * W, (row + rows_per_chunk) * W)
            O.render(rays[sl], u, *args, sb=1)
            done_rays += rows_per_chunk * W
            row += rows_per_chunk
        dt = time.perf_counter() - t0
        # the same oracle on os.cpu_count() threads (SURVEY §8(d)'s count), one image row:
        # reported beside the main number, which uses the CPUs the job may actually use
        at_count = None
        ncpu = os.cpu_count() or 1
        if ncpu != threads and os.environ.get("SD_CPU_COUNT_RUN", "1") != "0":
            torch.set_num_threads(ncpu)
            sl = slice(0, W)
            t1 = time.perf_counter()
            O.render(rays[sl], u[:W], *args, sb=1)
            d1 = time.perf_counter() - t1
            at_count = {"value": W / d1, "unit": "rays/s", "cores": ncpu,
                        "sample": f"{W} rays (1 row), {d1:.1f} s on {ncpu} threads"}
            torch.set_num_threads(threads)
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    hc = host_cpus()
    return {"value": done_rays / dt, "unit": "rays/s", "cores": threads, "kind": "port",
            "cpu_count": hc["cpu_count"], "affinity_cpus": hc["affinity"],
            "cgroup_cpu_quota": hc["quota"], "job_cpu_share": hc["share"],
            "sample": f"{done_rays} rays ({row} of {H} rows) of the same 192x640x64 frame"
                      f"{' (offset render pose)' if offset_pose else ''}, "
                      f"fp32 torch-CPU oracle restatement, {dt:.1f} s on {threads} threads "
                      f"({cpu}); encoder excluded",
            "at_os_cpu_count": at_count}


def _traffic_from_profile(pose):
    """HBM bytes per frame of the rendering kernels at one render pose, from the committed
    rocprofv3 PMC summary of this bench command (profiles/*_traffic_<pose>.json written by
    tools/traffic_json.py; PMC counters cannot be read from inside the timed process)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_traffic_{pose}.json")))
    if not files:
        return None
    try:
        d = json.load(open(files[-1]))
        tot = sum(v["hbm_bytes"] for k, v in d["kernels"].items()
                  if k in ("k_project", "k_render_tile", "k_render_proj", "k_head_hc"))
    except (KeyError, TypeError, ValueError):
        return None
    return tot, os.path.relpath(files[-1], ROOT) + " (rocprofv3 PMC, per frame)"


SEG_FLOPS_ALGO = 2 * (64 * 128 + 128 * 768) + 2 * (768 * 64 + 768 * 768 + 768 * 64) + 2 * 19 * 64
# executed MFMA work per voxel: W1, the Gram norm (G = W2^T W2 as hi + lo), L, M, Wn2 and
# the k-means tile (32 clusters x 64, three hi/lo products); the fp8 record's norm is the
# 768 x 128 W2 product instead of the Gram form
SEG_FLOPS_EXEC = 2 * (64 * 128 + 2 * 128 * 128 + 64 * 128 + 768 * 128 + 64 * 768 + 3 * 32 * 64)
SEG_FLOPS_EXEC_FP8 = SEG_FLOPS_EXEC - 2 * 2 * 128 * 128 + 2 * 768 * 128
SEG_FLOPS_FP8_PART = 2 * 768 * 128  # the norm product |W2 h + b2| on fp8 MFMA


C5_GRID_HW = (384, 1280)  # ViT-B/8 + DPT feature grid


def c5_scene(device, precision, frame_seed=0):
    """The C5 scene (BASELINE configs[4]): make_scene on the ViT-B/8-shaped 256x384x1280
    grid, random-init MlpDimReduction(768, 64, 128) + SemanticHead(19, 19, 768, 64) (seed 5),
    the SSCBench voxel centres.  precision "fp8": bf16 field, fp8 norm product in the seg
    head.  Returns (net, pts (n_vox, 3), dims)."""
    from scenedino_amd import sscbench
    from scenedino_amd.models.backbones.dino import MlpDimReduction
    from scenedino_amd.downstream_head import SemanticHead
    seg_fp8 = precision == "fp8"
    net, _, _, _, _, _ = make_scene(frame_seed, device, "bf16" if seg_fp8 else precision,
                                    grid_hw=C5_GRID_HW)
    net.seg_precision = "fp8" if seg_fp8 else "bf16"
    torch.manual_seed(5)
    net.encoder.dim_reduction = MlpDimReduction(768, 64, 128).to(device).eval()
    net.downstream_head = SemanticHead(19, 19, 768, 64).to(device).eval()
    net.gt_classes = 19
    dims = sscbench.grid_dims()
    pts = sscbench.generate_point_grid(sscbench.read_calib()["Tr"], device=device)
    return net, pts, dims


def main_c5(args, world, rank, local_rank, dist, device, host_stage=False):
    """C5 (BASELINE configs[4]): SSCBench voxel query, one 256x256x32 voxel grid per frame:
    voxel centres (sd_voxel_points, once per run as the reference does) -> per frame:
    grid packing (sd_pack_grid) + field query without colours (sd_field_query) + folded
    transform_expand / stego / k-means head with the alpha-weighted class pick
    (sd_seg_query) + 3x3x3 density grow.  ViT-B/8-shaped 256x384x1280 grid, d_full 768.
    N > 1: the frame's voxels are split into x-slabs [256 g / N, 256 (g+1) / N) (one halo
    plane each side for the grow), every rank queries its slab and the sigma / class slabs
    are all-gathered (strong scaling of one frame)."""
    from scenedino_amd import sscbench
    seg_fp8 = args.precision == "fp8"  # configs[4]: fp8 MFMA in the voxel MLP chain
    net, pts, dims = c5_scene(device, args.precision, 0 if dist else rank)
    n_vox = pts.shape[0]
    timer = KernelTimer()
    net.kernel_timer = timer

    def predict(p):
        sig, seg = net.predict_voxels(p.reshape(1, -1, 3), voxel_size=sscbench.VOXEL_SIZE)
        return sig.reshape(-1), seg.reshape(-1)

    def step():
        net._grid_cache = None
        if not dist:
            return sscbench.query_voxels(net, pts, dims)
        sig, seg = sscbench.query_voxels_slab(predict, pts, dims, rank, world)
        if host_stage:
            return sscbench.gather_slabs(sig.cpu(), seg.cpu(), dims)
        return sscbench.gather_slabs(sig, seg, dims)

    with torch.no_grad():
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        if dist:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        timer.on = True
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
            timer.tick()
        torch.cuda.synchronize()
        if dist:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
    seg_ms, field_ms = timer.mean_ms("seg"), timer.mean_ms("field")
    if dist:
        t = torch.tensor([elapsed, seg_ms, field_ms], device=device, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed, seg_ms, field_ms = (float(v) for v in t)
    if rank == 0:
        n_launch = n_vox  # voxels per k_seg_head launch (dist: this rank's slab + halo planes)
        if dist:
            x0, x1 = sscbench.slab_range(dims[0], rank, world)
            n_launch = (min(x1 + 1, dims[0]) - max(x0 - 1, 0)) * dims[1] * dims[2]
        algo = n_launch * SEG_FLOPS_ALGO  # the reference's unfolded head
        # HBM bytes per k_seg_head launch (1-GPU launch shape) from the committed PMC
        # summary (tools/c5_traffic.sh: FETCH_SIZE x 2 + WRITE_SIZE, separate passes)
        seg_traffic, seg_tsrc = None, None
        for tn in ("r6_c5_traffic.json", "r5_c5_traffic.json", "r3_c5_traffic.json"):
            tf = os.path.join(ROOT, "profiles", tn)
            if dist or not os.path.exists(tf):
                continue
            try:
                seg_traffic = json.load(open(tf))["kernels"]["k_seg_head"]["hbm_bytes"]
                seg_tsrc = f"profiles/{tn} (rocprofv3 PMC, per launch)"
                break
            except (KeyError, TypeError, ValueError):
                seg_traffic = None
        # the roofline is priced on the folded algorithm the kernel runs: its
        # MFMA FLOPs per voxel, each product at its own dense peak (the fp8 norm product at
        # 5 PF, the rest at 2.5 PF) -- the reference's FLOPs over the same time exceed the
        # peak because the fold removes three quarters of them
        exe = n_launch * (SEG_FLOPS_EXEC_FP8 if seg_fp8 else SEG_FLOPS_EXEC)
        f8 = n_launch * SEG_FLOPS_FP8_PART if seg_fp8 else 0
        peak_eff = exe / ((exe - f8) / PEAK_TFLOPS["bf16"] + f8 / PEAK_TFLOPS["fp8"])
        ach = exe / (seg_ms * 1e-3) / 1e12
        line = {
            "metric": "SSCBench voxel-grid query, voxels/sec (256x256x32 grid per frame)",
            "value": n_vox * args.steps / elapsed, "unit": "voxels/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None,
            "dtype": ("fp8 e4m3 (k_seg_head norm product) + bf16" if seg_fp8 else args.precision),
            "data": "synthetic (seeded image, N(0,1) 256x384x1280 grid, random-init ResnetFC / "
                    "MlpDimReduction / SemanticHead)",
            "config": {"workload": "C5: SSCBench 256x256x32 voxel query, ViT-B/8-shaped "
                                   "256x384x1280 grid, d_full 768, stego_kmeans, alpha-weighted "
                                   "class pick + grow", "voxels_per_frame": n_vox,
                       "parallelism": (f"xslab{world}+allgather" if world > 1 else "1 frame")},
            "roofline": {
                "kernel": "k_seg_head (sd_seg_query)", "bound": "mfma",
                "achieved": ach, "peak": peak_eff, "unit": "TFLOP/s", "frac": ach / peak_eff,
                "peak_note": ("fp8 norm product at 5 PF, other products at 2.5 PF (FLOP-"
                              "weighted)" if seg_fp8 else "bf16 dense MFMA"),
                "traffic": seg_traffic, "traffic_source": seg_tsrc, "kernel_ms": seg_ms,
                "algorithmic_flops_per_launch": exe,
                "algorithm": "folded head (M = Wn1 W2, L = Wl W2, Gram-form norm; DESIGN §5)",
                "reference_flops_per_launch": algo,
                "reference_equivalent_tflops": algo / (seg_ms * 1e-3) / 1e12,
                "field_query_ms": field_ms,
                "field_query_tflops": n_launch * mlp_flops_per_point() / (field_ms * 1e-3) / 1e12,
            },
        }
        if not seg_fp8:  # configs[4] names fp8 MFMA; measured, and not the default
            line["fp8"] = {
                "used": False,
                "reason": "slower and below the label bar: --precision fp8 (the norm product "
                          "on block-scaled fp8 MFMA) runs 1.41 ms vs 1.27-1.29 ms bf16 "
                          "(profiles/r5_c5/bench_c5_fp8.log), and fp8 for the M / Wn2 chain "
                          "keeps < 99 % of the labels at any block scale "
                          "(profiles/r5_seg_fp8_emul.txt); fp8 for the field MLP's first "
                          "layer (the projected grid P in e4m3, per-tensor power-of-two "
                          "scale) keeps sigma within 1.4e-2 rel-L2 but only 98.16 % of the "
                          "labels, against 99.69 % between the accepted fp16 and bf16 modes "
                          "(profiles/r5_field_fp8_emul.txt)"}
        print(json.dumps(line), flush=True)


def vit_flops(T, C, L, p, Np, mlp=4):
    """Algorithmic FLOPs of one ViT pass: per block qkv + proj + MLP GEMMs and the two
    attention products (L T (24 C^2 + 4 T C) at mlp ratio 4), + patch embed."""
    return L * T * (2 * C * 3 * C + 2 * C * C + 2 * 2 * C * mlp * C + 4 * T * C) + 2 * Np * 3 * p * p * C


def main_vit(args, world, rank, device):
    """a19: the DINO encoder's ViT forward (DINOv2Encoder -> _ViT) on one 192x640 frame:
    ViT-S/16 (481 tokens, BASELINE configs[1]) and ViT-B/8 (1921 tokens, the released
    SceneDINO checkpoints), random weights.  Timed: patchify + 12 blocks + final norm +
    token grids, all libsdhip.so kernels."""
    from scenedino_amd.models.backbones.dino.vit import DINOv2Encoder
    results = {}
    models = {"vit-s16": ("vit-s", "v1_16"), "vit-b8": ("vit-b", "v1"),
              "dinov2-b14": ("vit-b", "v2")}  # C4 (configs[3]): 192x640 resized to 168x560
    if args.models:
        models = {k: models[k] for k in args.models.split(",")}
    for name, (arch, ver) in models.items():
        torch.manual_seed(0)
        enc = DINOv2Encoder(arch, (H, W), [3, 6, 9], False, ver).to(device).eval()
        img = (torch.rand(1, 3, H, W, generator=torch.Generator().manual_seed(rank)) * 2 - 1).to(device)
        with torch.no_grad():
            for _ in range(args.warmup):
                enc(img)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                enc(img)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / args.steps
        vit = enc.model.vit
        p, C = vit.patch_size, vit.embed_dim
        rh, rw = enc.resize if enc.resize is not None else (H, W)
        Np = (rh // p) * (rw // p)
        fl = vit_flops(Np + 1, C, len(vit.blocks), p, Np)
        results[name] = {"ms_per_pass": dt * 1e3, "tokens": Np + 1, "dim": C, "patch": p,
                         "gflop_per_pass": fl / 1e9, "tflops": fl / dt / 1e12,
                         "frac_bf16_peak": fl / dt / 1e12 / PEAK_TFLOPS["bf16"]}
    first = next(iter(results))
    roof = "vit-b8" if "vit-b8" in results else first
    if rank == 0:
        print(json.dumps({
            "metric": "DINO ViT encoder passes/sec (192x640 frame, 12 blocks)",
            "value": 1e3 / results[first]["ms_per_pass"], "unit": "passes/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "higher_is_better": True, "dtype": "bf16", "data": "synthetic, random weights",
            "config": {"workload": "a19 ViT encoder forward (DINOv2Encoder, no DPT decoder)"},
            "models": results,
            "roofline": {"kernel": f"k_gemm + k_attn ({roof})", "bound": "mfma",
                         "achieved": results[roof]["tflops"], "peak": PEAK_TFLOPS["bf16"],
                         "unit": "TFLOP/s", "frac": results[roof]["frac_bf16_peak"]},
        }), flush=True)


def dpt_flops(head, gh, gw):
    """Algorithmic FLOPs of one DPTHead pass on a (gh, gw) token grid (2 MACs per
    multiply-add; convolutions as their dense products, ConvTranspose(k, k) as k^2 C_in
    C_out per input pixel, bilinear resizes not counted)."""
    post, d = head.post_process_channels, head.d_out
    C = head.reassemble_blocks.projects[0].in_channels
    c3 = lambda h, w, ci, co: 2 * h * w * 9 * ci * co
    fl = sum(2 * gh * gw * C * c for c in post)
    fl += 2 * gh * gw * post[0] ** 2 * 16 + 2 * gh * gw * post[1] ** 2 * 4
    h3, w3 = (gh + 1) // 2, (gw + 1) // 2
    fl += c3(h3, w3, post[3], post[3])
    sizes = [(4 * gh, 4 * gw), (2 * gh, 2 * gw), (gh, gw), (h3, w3)]
    fl += sum(c3(h, w, c, d) for (h, w), c in zip(sizes, post))
    h, w = h3, w3
    for i in range(len(head.fusion_blocks)):
        fl += (2 if i == 0 else 4) * c3(h, w, d, d)  # rcu2 (+ rcu1)
        h, w = 2 * h, 2 * w
        fl += 2 * h * w * d * d  # project 1x1
    fl += 2 * c3(h, w, d, d)  # project + head0
    fl += 2 * h * w * d * d * 4  # head1 ConvTranspose(2, 2)
    return fl + c3(2 * h, 2 * w, d, d)  # head2


def main_encode(args, world, rank, device):
    """The SceneDINO image encoder's prediction pass (DINOv2Module.forward: ViT -> DPT ->
    NCHW f32 feature grid) on one 192x640 frame, random weights, as configs/model/
    dino_downsampler.yaml builds it (ViT-B/8, DPT num_ch_enc [64, 64, 128, 256], d_out 256)
    and with the ViT-S/16 of BASELINE configs[1].  One HIP graph per pass, output cloned
    (the reference's fresh tensor)."""
    from scenedino_amd.models.backbones import make_backbone
    results = {}
    models = {"vit-s16": ("vit-s", "v1_16"), "vit-b8": ("vit-b", "v1"),
              "dinov2-b14": ("vit-b", "v2")}  # C4 (configs[3]): 192x640 resized to 168x560
    if args.models:
        models = {k: models[k] for k in args.models.split(",")}
    for name, (arch, ver) in models.items():
        torch.manual_seed(0)
        conf = dict(type="dinov2", mode="downsample-prediction", decoder_arch="dpt",
                    downsampler_arch="featup", encoder_arch=arch, version=ver,
                    separate_gt_version=None, encoder_freeze=True, flip_avg_gt=False,
                    dim_reduction_arch="mlp", num_ch_enc=[64, 64, 128, 256],
                    intermediate_features=[3, 6, 9], decoder_out_dim=256, dino_pca_dim=64,
                    image_size=[H, W], key_features=False)
        m = make_backbone(conf).to(device).eval()
        img = (torch.rand(1, 3, H, W, generator=torch.Generator().manual_seed(rank)) * 2 - 1).to(device)
        with torch.no_grad():
            for _ in range(args.warmup):
                m(img)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                m(img)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / args.steps
            out_shape = list(m(img)[0].shape)
        vit = m.encoder.model.vit
        p, C = vit.patch_size, vit.embed_dim
        rh, rw = m.encoder.resize if m.encoder.resize is not None else (H, W)
        gh, gw = rh // p, rw // p
        fv = vit_flops(gh * gw + 1, C, len(vit.blocks), p, gh * gw)
        fd = dpt_flops(m.decoder, gh, gw)
        results[name] = {"ms_per_pass": dt * 1e3, "out_shape": out_shape,
                         "gflop_vit": fv / 1e9, "gflop_dpt": fd / 1e9,
                         "tflops": (fv + fd) / dt / 1e12,
                         "frac_bf16_peak": (fv + fd) / dt / 1e12 / PEAK_TFLOPS["bf16"]}
        del m
        torch.cuda.empty_cache()
    main = "vit-b8" if "vit-b8" in results else next(iter(results))
    if rank == 0:
        print(json.dumps({
            "metric": "SceneDINO encoder passes/sec (ViT + DPT, 192x640 frame)",
            "value": 1e3 / results[main]["ms_per_pass"], "unit": "passes/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "higher_is_better": True, "dtype": "bf16", "data": "synthetic, random weights",
            "config": {"workload": f"DINOv2Module prediction pass ({main} + DPT, "
                                   "configs/model/dino_downsampler.yaml)"},
            "models": results,
            "roofline": {"kernel": f"k_gemm (+ k_attn), {main} + DPT", "bound": "mfma",
                         "achieved": results[main]["tflops"], "peak": PEAK_TFLOPS["bf16"],
                         "unit": "TFLOP/s", "frac": results[main]["frac_bf16_peak"]},
        }), flush=True)


def train_setup(device, rank=0, NB=4, RB=2048, KT=32, PS=8, amp=True, offset_pose=False,
                capturable=False, world=1):
    """The training scene of ``main_train`` (also built by tests/test_train_graph.py): a
    BTSNet over a fixed N(0, 1) grid leaf, NeRFRenderer(n_coarse KT, hard_alpha_cap),
    PatchRaySampler (RB rays per frame in PS x PS snapped patches), random targets and a fused
    Adam on the head.  ``body(patches)`` is one step from the device sampler on: rays and
    targets from the drawn patches (sd_patch_rays), depth jitter into ``zj`` (drawn when
    draw_jitter, else the values already in zj), forward, loss, backward, Adam."""
    from types import SimpleNamespace
    from scenedino_amd import distributed as sdd
    from scenedino_amd.models import BTSNet
    from scenedino_amd.models.prediction_heads import ResnetFC
    from scenedino_amd.common.positional_encoding import PositionalEncoding
    from scenedino_amd.renderer import NeRFRenderer
    from scenedino_amd.common.ray_sampler import PatchRaySampler
    g = torch.Generator(device=device).manual_seed(rank)
    grid = _layout(torch.randn(NB, C_GRID, HF, WF, device=device, generator=g))
    torch.manual_seed(2)
    head = ResnetFC(d_in=D_IN, d_out=1 + D_DINO, n_blocks=0, d_hidden=D_HIDDEN)
    conf = {"predict_dino": True, "dino_dims": D_DINO, "learn_empty": False, "code_mode": "z",
            "inv_z": True, "z_near": 3, "z_far": 80, "sample_color": True, "precision": "fp32"}
    net = BTSNet(conf, FixedGridEncoder(grid), PositionalEncoding(6, 3, 1.5, True),
                 {"normal_head": head}, final_pred_head="normal_head").to(device)
    images = torch.rand(NB, 1, 3, H, W, device=device, generator=g) * 2 - 1
    Ks = torch.tensor(KITTI_K, device=device).view(1, 1, 3, 3).expand(NB, 1, 3, 3).contiguous()
    poses = torch.eye(4, device=device).view(1, 1, 4, 4).expand(NB, 1, 4, 4).contiguous()
    with torch.no_grad():
        net.encode(images, Ks, poses, ids_encoder=[0], ids_render=[0])
    leaf = net.grid_f_features[0].detach().clone().requires_grad_(True)
    net.grid_f_features[0] = leaf
    net.train()
    renderer = NeRFRenderer(n_coarse=KT, lindisp=True, hard_alpha_cap=True, eval_batch_size=65536)
    wrapper = renderer.bind_parallel(net, gpus=None).train()
    ray_poses = poses
    if offset_pose:  # rays from a 0.5 m lateral / 2 deg yaw view: samples of a ray
        import math   # project onto different texels of the encoder grid
        a = math.radians(2.0)
        ray_poses = poses.clone()
        ray_poses[:, 0, 0, 0] = math.cos(a); ray_poses[:, 0, 0, 2] = math.sin(a)
        ray_poses[:, 0, 2, 0] = -math.sin(a); ray_poses[:, 0, 2, 2] = math.cos(a)
        ray_poses[:, 0, 0, 3] = 0.5
    # training/scenedino.yaml + train_scenedino_kitti_360.yaml: patch 8, 2048 rays, snapped
    sampler = PatchRaySampler(3, 80, RB, PS, snap_to_grid=True, dino_upscaled=False)
    dino_gt_map = torch.randn(NB, 1, D_DINO, H // PS, W // PS, device=device, generator=g)
    # the grid is an activation (the encoder's output): its gradient is computed, the
    # optimizer steps the head (a frozen-encoder config; encoder backward is not ours).
    # Adam as one fused kernel over the head's parameters (torch's fused implementation, the
    # same update as the reference's Adam: base_trainer.py optimizer)
    opt = torch.optim.Adam(head.parameters(), lr=1e-4, fused=True, capturable=capturable)
    npatch = RB // (PS * PS)
    zj = torch.empty(NB * RB, KT, device=device)

    def loss_of(out, rgb_gt, dino_gt):
        pd = out["dino_features"].float().view(NB, npatch, PS * PS, D_DINO).mean(2)
        return ((pd - dino_gt) ** 2).mean() + (out["rgb"].float() - (rgb_gt * 0.5 + 0.5)).abs().mean()

    def body(patches, draw_jitter=True):
        rays, rgb_gt, dino_gt = sampler.sample_patches(patches, images, ray_poses, Ks,
                                                       dino_features=dino_gt_map)
        if draw_jitter:
            zj.uniform_()
        renderer.z_jitter = zj
        with torch.autocast("cuda", dtype=torch.float16, enabled=amp, cache_enabled=False):
            out = wrapper(rays, want_weights=True)["coarse"]
            loss = loss_of(out, rgb_gt, dino_gt)
        opt.zero_grad(set_to_none=True)
        leaf.grad = None
        loss.backward()
        if world > 1:  # data-parallel head: one RCCL all-reduce of the gradient bucket
            sdd.allreduce_grads(head.parameters())
        opt.step()
        renderer.z_jitter = None
        return loss

    return SimpleNamespace(net=net, head=head, leaf=leaf, renderer=renderer, wrapper=wrapper,
                           sampler=sampler, images=images, ray_poses=ray_poses, Ks=Ks,
                           dino_gt_map=dino_gt_map, opt=opt, zj=zj, body=body, loss_of=loss_of,
                           NB=NB, RB=RB, KT=KT, PS=PS, npatch=npatch)


def main_train(args, world, rank, device):
    """Training step through the render path (train_scenedino_kitti_360
    .yaml: batch_size 4, n_coarse 32, hard_alpha_cap, training/scenedino.yaml ray_batch_size
    2048 in 8x8 patches): per step 4 frames x 2048 rays x 32 samples through BTSNet.forward
    (sd_field_gather -> ResnetFC -> softplus) + sd_composite, an L2 loss on the rendered
    DINO / colour maps, and loss.backward() (sd_composite_bwd, ResnetFC GEMM backward,
    sd_field_gather_bwd into the 4 x 256 x 192 x 640 grid gradient).  The encoder backward is
    not part of the step (the grid is the leaf)."""
    from scenedino_amd import autograd as sda
    from scenedino_amd import distributed as sdd
    NB, RB, KT, PS = 4, 2048, 32, 8
    # graph mode (the default on one GPU; --no-graph: eager): everything after the host's patch draws -- the device
    # sampler, forward, loss, backward, Adam -- replayed as one captured HIP graph per step,
    # so the host only draws patches and launches the graph (round 3 measured the eager step
    # host-paced: ~1.3 ms of issue against ~1.0 ms of GPU work)
    graph_mode = world == 1 and args.graph
    amp = not args.no_amp  # train_scenedino_kitti_360.yaml: with_amp: true (fp16 autocast)
    ts = train_setup(device, rank, NB, RB, KT, PS, amp=amp, offset_pose=args.offset_pose,
                     capturable=graph_mode, world=world)
    head, leaf, renderer, wrapper, sampler = ts.head, ts.leaf, ts.renderer, ts.wrapper, ts.sampler
    images, ray_poses, Ks, dino_gt_map, opt = ts.images, ts.ray_poses, ts.Ks, ts.dino_gt_map, ts.opt

    host = {} if os.environ.get("SCENEDINO_AMD_HOST_PROFILE") == "1" else None

    def mark(name, t0):  # diagnostic: host issue time per phase (no device sync)
        if host is not None:
            t1 = time.perf_counter()
            host[name] = host.get(name, 0.0) + (t1 - t0)
            return t1
        return t0

    def step():
        t0 = time.perf_counter()
        # PatchRaySampler batch (device rays + rgb / per-patch DINO targets)
        rays, rgb_gt, dino_gt = sampler.sample(images, ray_poses, Ks, dino_features=dino_gt_map)
        t0 = mark("sample", t0)
        with torch.autocast("cuda", dtype=torch.float16, enabled=amp):
            out = wrapper(rays, want_weights=True)["coarse"]
            t0 = mark("forward", t0)
            loss = ts.loss_of(out, rgb_gt, dino_gt)
        t0 = mark("loss", t0)
        opt.zero_grad(set_to_none=True)
        leaf.grad = None
        loss.backward()
        t0 = mark("backward", t0)
        if world > 1:  # data-parallel head: one RCCL all-reduce of the gradient bucket
            sdd.allreduce_grads(head.parameters())
        opt.step()
        mark("optimizer", t0)
        return loss

    eager_step = step

    timer = KernelTimer()
    sda.kernel_timer = timer
    if not graph_mode:  # (graph mode warms up on the capture's side stream below)
        for _ in range(args.warmup):
            step()
    torch.cuda.synchronize()
    if graph_mode:
        # the step from the device sampler on, captured twice (two pinned host slots for the
        # drawn patches: the host fills one while the other graph's copy may still be queued).
        # The depth jitter is drawn on the device inside the graph (torch.rand_like, as
        # nerf.py:134 does), so every replay samples new depths; the kernel timer is off
        # during capture (its events would be frozen into the graph).
        sda.kernel_timer = None
        shape = sampler.draw(images, dino_gt_map).shape
        host_slots = [torch.empty(shape, dtype=torch.int32, pin_memory=True) for _ in range(2)]
        dev_slots = [torch.empty(shape, dtype=torch.int32, device=device) for _ in range(2)]

        def body(k):
            return ts.body(dev_slots[k])

        side = torch.cuda.Stream(device=device)
        side.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(side):  # warm-up of the captured code path (allocations, packing)
            for i in range(max(3, args.warmup)):
                host_slots[i & 1].copy_(sampler.draw(images, dino_gt_map))
                dev_slots[i & 1].copy_(host_slots[i & 1], non_blocking=True)
                body(i & 1)
                torch.cuda.current_stream(device).synchronize()
        torch.cuda.current_stream(device).wait_stream(side)
        torch.cuda.synchronize()
        graphs, pool = [], None
        for k in range(2):
            gph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gph, pool=pool):
                body(k)
            pool = gph.pool()
            graphs.append(gph)
        torch.cuda.synchronize()
        done = [None, None]
        nstep = [0]

        def step():  # noqa: F811 -- the graphed steady-state step
            t0 = time.perf_counter()
            k = nstep[0] & 1
            nstep[0] += 1
            if done[k] is not None:
                done[k].synchronize()  # the copy out of host slot k two steps ago has run
            host_slots[k].copy_(sampler.draw(images, dino_gt_map))
            t0 = mark("sample", t0)
            dev_slots[k].copy_(host_slots[k], non_blocking=True)  # into the graph's input slot
            graphs[k].replay()
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(device))
            done[k] = ev
            mark("replay", t0)

        for _ in range(2):
            step()
        torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    timer.on = not graph_mode
    if host is not None:
        host.clear()  # steady state only
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        timer.tick()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    timer.on = False
    if graph_mode:
        # the kernels' own durations (roofline fields) from eager steps after the timed region
        sda.kernel_timer = timer
        timer.on = True
        for _ in range(4):  # (on the default stream: no autograd state outlives a step)
            eager_step()
            timer.tick()
        torch.cuda.synchronize()
        timer.on = False
    sda.kernel_timer = None
    if host is not None and rank == 0:
        n = args.steps
        print("host issue ms per step: " + ", ".join(f"{k} {1e3 * v / n:.3f}" for k, v in host.items()),
              file=sys.stderr, flush=True)
    ms = {k: timer.mean_ms(k) for k in ("gather", "gather_bwd", "composite_bwd", "mlp_bwd")}
    if world > 1:
        t = torch.tensor([elapsed] + [ms[k] for k in ms], device=device, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t[0])
        ms = {k: float(v) for k, v in zip(ms, t[1:])}
    n_pts = NB * RB * KT
    chunk = n_pts  # points per backward launch (training path: one per pass)
    fused = amp and sda.FUSED_SCATTER
    if fused:
        # k_mlp_bwd with the grid_sample backward fused (ml_scatter): per point it reads
        # d_sigma, sigma (4 + 4), d_dino (4 D), the saved H row (2 x 136) and xyz (12), and
        # writes the dY (2 x 72) and dH (2 x 128) rows of the weight-gradient GEMMs = 948 B;
        # the grid-gradient atomics depend on the geometry and are left out of the floor
        kname, kkey, tkey = "k_mlp_bwd + fused grid_sample backward (sd_mlp_train_bwd)", \
            "mlp_bwd", "k_mlp_bwd"
        bwd_bytes = chunk * (8 + 4 * D_DINO + 2 * 136 + 12 + 2 * 72 + 2 * 128)
    else:
        # compulsory HBM bytes of one scatter launch: the C feature columns of the dX rows
        # (4 C B per point) + the touched grid-gradient pixels written once (4 taps x 4 C B
        # per texel quad; depends on the geometry) -- counted as the dX reads only, the floor
        kname, kkey, tkey = "k_field_gather_bwd (sd_field_gather_bwd)", "gather_bwd", \
            "k_field_gather_bwd"
        bwd_bytes = chunk * 4 * C_GRID
    traffic, tsrc = None, None
    for tf in ("r5_train_traffic.json", "r4_train_traffic.json", "r3_train_traffic.json"):
        try:
            traffic = json.load(open(os.path.join(ROOT, "profiles", tf)))["kernels"][tkey]["hbm_bytes"]
            tsrc = f"profiles/{tf} (rocprofv3 PMC, per launch)"
            break
        except (OSError, KeyError, TypeError, ValueError):
            traffic = None
    line = {
        "metric": "training rays/sec (render forward + backward into grid and ResnetFC)",
        "value": world * NB * RB * args.steps / elapsed, "unit": "rays/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "step_issue": ("one captured HIP graph per step (host: patch draws + replay)"
                       if graph_mode else "eager"),
        "dtype": "fp16 autocast MLP, fp32 gather / compositing" if amp else "fp32",
        "data": "synthetic (N(0,1) 4x256x192x640 grid, U[-1,1) images, random targets)",
        "config": {"workload": "train: 4 frames x 2048 rays (PatchRaySampler: 32 snapped 8x8 "
                               "patches) x 32 samples, "
                               "hard_alpha_cap, ResnetFC 295-128-65, Adam step on the head, "
                               "grid gradient computed" +
                               (", rays from an offset view" if args.offset_pose else
                                ", rays from the encoder view"),
                   "points_per_step": n_pts,
                   "parallelism": f"dp{world} (4 frames per GPU, head gradients all-reduced)"},
        "roofline": {"kernel": kname, "bound": "hbm",
                     "algorithmic_bytes_per_launch": bwd_bytes,
                     "achieved": bwd_bytes / (ms[kkey] * 1e-3) / 1e9 if ms[kkey] else None,
                     "peak": 8000.0, "unit": "GB/s",
                     "frac": bwd_bytes / (ms[kkey] * 1e-3) / 1e9 / 8000.0 if ms[kkey] else None,
                     "traffic": traffic, "traffic_source": tsrc, "kernel_ms": ms[kkey],
                     "gather_ms": ms["gather"], "composite_bwd_ms": ms["composite_bwd"],
                     "mlp_bwd_ms": ms["mlp_bwd"], "gather_bwd_ms": ms["gather_bwd"]},
    }
    if rank == 0:
        print(json.dumps(line), flush=True)


def _launch_ranks(args) -> int:
    """--gpus N outside torchrun: start N rank processes (this process has not touched
    the GPU: device counting aside, nothing in bench.py initialises HIP before here) and
    return their exit status."""
    import socket
    import subprocess
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
    so.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def reserve_cus(args, world, host_stage) -> int:
    """CUs the persistent kernels leave to RCCL when a collective runs beside them: --reserve-cus,
    or (-1, auto) NCCL_MAX_NCHANNELS (bench.py sets 16 for its RCCL gathers) with N > 1 RCCL."""
    if args.reserve_cus >= 0:
        return args.reserve_cus
    if world <= 1 or host_stage:
        return 0
    return int(os.environ.get("NCCL_MAX_NCHANNELS", "16"))


def c2_pose_run(args, world, rank, device, dist, offset_pose, host_stage):
    """Time the C2 step at one render pose (all ranks; max over ranks)."""
    from scenedino_amd import distributed as sdd
    rows = dist and args.shard == "rows"
    # frames: frame r on rank r (weak scaling); rows: every rank encodes the same frame and
    # renders its band of rows [H g / N, H (g + 1) / N) (strong scaling of one frame)
    net, renderer, wrapper, sampler, pose, Ks = make_scene(0 if rows else rank, device,
                                                          args.precision, offset_pose)
    R = H * W
    band = None
    if rows:
        y0, y1 = sdd.row_band(H, rank, world)
        if (y1 - y0) != H // world or H % world:
            raise ValueError(f"--shard rows needs H ({H}) divisible by the world size ({world})")
        band = (y0 * W, y1 * W)
    Rr = band[1] - band[0] if band else R
    # frames are independent units; by default (BASELINE configs[2]) every
    # rank's maps are all-gathered over RCCL under the next frame's render, --gather none
    # leaves them on each rank's GPU.  Row bands of one frame are gathered into the frame
    # (that IS the frame's assembly).
    use_gather = dist and (rows or args.gather == "allgather")
    gather = sdd.MapGather(Rr, 1 + D_DINO + 3, device, host_stage=host_stage) if use_gather else None
    # RCCL's all-gather of frame i runs beside frame i+1's projection and render: the
    # persistent grids leave its CUs free (sd_reserve_cus, one CU per RCCL channel), else the
    # workgroups whose CUs it holds start only after it
    from scenedino_amd import _lib as sdl
    sdl.reserve_cus(reserve_cus(args, world, host_stage) if use_gather else 0)
    net.fused_mode = args.mode
    timer = KernelTimer()
    net.kernel_timer = timer

    def step(i):
        if gather is not None:  # frame f on rank f; maps rendered into the gather send slot
            net.render_into = gather.send(i)
        out = render_step(net, wrapper, sampler, pose, Ks, band, want_weights=WANT_SAMPLES,
                          want_alphas=WANT_SAMPLES)
        if gather is not None:
            gather.start(i)
        return out

    for i in range(args.warmup):
        step(i)
    if gather is not None:
        gather.wait_all()
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    timer.on = True
    t0 = time.perf_counter()
    host_ms = 0.0
    for i in range(args.steps):
        th = time.perf_counter()
        step(args.warmup + i)
        host_ms += 1e3 * (time.perf_counter() - th)
        timer.tick()
    if os.environ.get("SCENEDINO_AMD_HOST_PROFILE") == "1" and rank == 0:
        print(f"host issue ms per frame: {host_ms / args.steps:.3f}", file=sys.stderr, flush=True)
    if gather is not None:
        gather.wait_all()
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    timer.on = False
    render_ms, proj_ms = timer.mean_ms("render"), timer.mean_ms("project")
    if dist:
        t = torch.tensor([elapsed, render_ms, proj_ms], device=device, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed, render_ms, proj_ms = float(t[0]), float(t[1]), float(t[2])
    proj = net._use_proj()
    res = {"value": (R if rows else world * R) * args.steps / elapsed,
           "ms_per_step": 1e3 * elapsed / args.steps,
           "render_kernel_ms": render_ms, "project_kernel_ms": proj_ms, "proj": proj}
    if gather is not None and rank == 0:
        res["gathered_maps"] = list(gather.recv[0].shape)
    net.render_into = None
    del net, wrapper, renderer, gather
    torch.cuda.empty_cache()
    return res


def main_c2(args, world, rank, device, dist, host_stage):
    poses = {"identity": False, "offset": True}
    if args.offset_pose:
        poses = {"offset": True}
    elif args.identity_pose:
        poses = {"identity": False}
    runs = {name: c2_pose_run(args, world, rank, device, dist, off, host_stage)
            for name, off in poses.items()}
    alt = None
    if args.precision == "bf16" and not args.no_fp16_line and args.config in ("c1", "c2"):
        # the library's default precision (fp16: within SURVEY §8(c)'s 1e-2 m depth contract,
        # DESIGN §4), timed at the same poses beside the configs[1] (bf16) value
        a16 = argparse.Namespace(**dict(vars(args), precision="fp16"))
        r16 = {name: c2_pose_run(a16, world, rank, device, dist, off, host_stage)
               for name, off in poses.items()}
        s16 = min(r16, key=lambda k: r16[k]["value"])
        alt = {"dtype": "fp16", "note": "BTSNet's default precision (meets the 1e-2 m depth "
               "contract); same kernels as the bf16 value", "pose": s16,
               "value": r16[s16]["value"], "ms_per_step": r16[s16]["ms_per_step"],
               "poses": {k: {kk: v[kk] for kk in ("value", "ms_per_step", "render_kernel_ms",
                                                  "project_kernel_ms")} for k, v in r16.items()}}
    rows = dist and args.shard == "rows"
    slow = min(runs, key=lambda k: runs[k]["value"])
    nog = None
    if dist and not rows and args.gather == "allgather":
        # the labelled variant: the same frames and pose with no data-path collective, so
        # the line shows what the all-gather costs on top of the independent frames
        an = argparse.Namespace(**dict(vars(args), gather="none"))
        rn = c2_pose_run(an, world, rank, device, dist, poses[slow], host_stage)
        nog = {"parallelism": f"frames{world}", "pose": slow, "value": rn["value"],
               "ms_per_step": rn["ms_per_step"], "render_kernel_ms": rn["render_kernel_ms"],
               "note": "same workload with every rank's maps left on its GPU (no collective)"}
    if rank != 0:
        return
    r = runs[slow]
    R = H * W
    # SURVEY §8(d) algorithmic work: 92,160 FLOP per point (the reference MLP), over the
    # kernels that turn the encoded grid into rendered maps
    kern_ms = r["render_kernel_ms"] + r["project_kernel_ms"]
    flops = R * K_SAMPLES * mlp_flops_per_point()
    achieved = flops / (kern_ms * 1e-3) / 1e12
    peak = PEAK_TFLOPS[args.precision]
    if r["proj"]:
        # what the matrix cores execute per 16-sample item (k_render_tile): blend 16 x
        # 16x16x32, code 8 x 16x16x32 + 8 x 16x16x16, sigma 4 x 16x16x32; DINO head per
        # 8-ray group D/16 x 4 x 16x16x32; plus the projection P = W G (k_project)
        mac_item = 16 * 8192 + 8 * 8192 + 8 * 4096 + 4 * 8192
        exec_flops = (HF * WF * 2 * C_GRID * D_HIDDEN
                      + (R * K_SAMPLES // 16) * 2 * mac_item
                      + (R // 8) * (D_DINO // 16) * 4 * 2 * 8192)
    else:
        exec_flops = flops
    line = {
        "metric": f"rendered rays/sec, KITTI-360 192x640x{K_SAMPLES}-sample frustum",
        "value": r["value"],
        "unit": "rays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": r["ms_per_step"],
        "ms_per_frame": r["ms_per_step"] / (1 if rows else world),
        "higher_is_better": True,
        "scaling": "strong" if rows else "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic (seeded U[-1,1) image, N(0,1) 256x192x640 feature grid, "
                "kaiming-init ResnetFC; no dataset/checkpoint offline)",
        "config": {
            "workload": ("C2: KITTI-360 192x640 frustum, 64 samples/ray, ViT-S/16-shaped "
                         "256x192x640 DPT feature grid, ResnetFC 295-128-65, lindisp"
                         if args.config == "c2" else
                         "C1 shape: 192x640 frustum, 32 samples/ray (configs/renderer/"
                         "pixelnerf.yaml), 256x192x640 DPT feature grid, ResnetFC 295-128-65, "
                         "lindisp"
                         if args.config == "c1" else
                         "C4: KITTI-360 192x640 frustum, 128 samples/ray, DINOv2-B/14-shaped "
                         "256x192x640 DPT feature grid, ResnetFC 295-128-385 (384-d field), "
                         "lindisp") +
                        f"; render poses {'/'.join(runs)}, value = the slower ({slow})",
            "frames_per_gpu": 1, "rays_per_frame": R, "samples_per_ray": K_SAMPLES,
            "grid": [C_GRID, HF, WF],
            "parallelism": (f"rows{world}" if rows else f"frames{world}") +
            (f"+{'rccl' if not host_stage else 'gloo-host'}_allgather"
             if world > 1 and (rows or args.gather == "allgather") else ""),
            "dist_world_size": world,
        },
        "poses": {k: {kk: v[kk] for kk in ("value", "ms_per_step", "render_kernel_ms",
                                          "project_kernel_ms")} for k, v in runs.items()},
        "roofline": {
            "kernel": ("k_project + k_render_tile (+ k_render_proj overflow) "
                       "(sd_project_grid + sd_render_proj)" if r["proj"] else
                       "k_render (sd_render_fused)"),
            "pose": slow,
            "bound": "mfma",
            # achieved / frac: the MFMA work the executed algorithm issues (projection
            # P = W_in G once per grid pixel + per-sample blend / code / sigma + the per-ray
            # DINO head) over the kernels' time -- the matrix cores' utilisation.
            # SURVEY §8(d)'s reference-equivalent count (92,160 FLOP per point, the unfolded
            # MLP) over the same time is kept beside it; it exceeds the executed work
            # because the projected grid and the hidden-space head are exact rewrites.
            "achieved": exec_flops / (kern_ms * 1e-3) / 1e12,
            "peak": peak,
            "unit": "TFLOP/s",
            "frac": exec_flops / (kern_ms * 1e-3) / 1e12 / peak,
            "frac_basis": "executed MFMA work",
            "traffic": None,
            "kernel_ms": kern_ms,
            "render_kernel_ms": r["render_kernel_ms"],
            "project_kernel_ms": r["project_kernel_ms"],
            "executed_mfma_flops_per_launch": exec_flops,
            "reference_flops_per_launch": flops,
            "reference_equivalent_tflops": achieved,
            "reference_equivalent_frac": achieved / peak,
        },
    }
    if "gathered_maps" in r:
        line["config"]["gathered_maps"] = r["gathered_maps"]
        line["config"]["reserved_cus"] = reserve_cus(args, world, host_stage)
        line["config"]["nccl_max_nchannels"] = os.environ.get("NCCL_MAX_NCHANNELS")
        line["config"]["gather_bytes_per_rank_per_step"] = 4 * r["gathered_maps"][1] * \
            r["gathered_maps"][2] * (world - 1)
    if nog is not None:
        line["no_gather"] = nog
    if alt is not None:
        line["fp16_default"] = alt
    tr = _traffic_from_profile(slow) if args.config == "c2" else None
    if tr is not None:
        line["roofline"]["traffic"] = tr[0]
        line["roofline"]["traffic_source"] = tr[1]
    if args.config == "c2" and not args.no_end_to_end and world == 1:
        line["end_to_end"] = end_to_end(args, device, rank)
    if not args.no_cpu_baseline and world == 1:
        line["cpu_baseline"] = cpu_baseline(args.cpu_budget, offset_pose=(slow == "offset"))
    print(json.dumps(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp16", "fp32", "fp8"],
                    help="fp8: --config c5 only (fp8 MFMA norm product in k_seg_head)")
    ap.add_argument("--offset-pose", action="store_true",
                    help="c2/c4: time only the offset render pose (default: both poses)")
    ap.add_argument("--shard", default="frames", choices=["frames", "rows"],
                    help="c2 with N > 1: frames (frame r on rank r, configs[2]) or rows (one "
                         "frame's row bands across ranks, the north star's ray tiles)")
    ap.add_argument("--gather", default="allgather", choices=["none", "allgather"],
                    help="c2 --shard frames with N > 1: allgather (default, BASELINE configs[2]: "
                         "RCCL all-gather of every rank's rendered maps, overlapped with the "
                         "next frame's render; the same pose is then also timed without the "
                         "collective and reported as no_gather on the same line) or none (value "
                         "timed with no data-path collective)")
    ap.add_argument("--reserve-cus", type=int, default=-1,
                    help="c2 with an RCCL gather: CUs the persistent kernels leave free for RCCL's "
                         "channels (-1: NCCL_MAX_NCHANNELS, set to 16 by bench.py if unset)")
    ap.add_argument("--identity-pose", action="store_true",
                    help="c2: time only the identity render pose (profiling runs)")
    ap.add_argument("--mode", default="proj", choices=["proj", "grid"],
                    help="16-bit render kernel: projected grid (default) or per-sample grid")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--grid-layout", default="nhwc", choices=["nhwc", "nchw"],
                    help="synthetic feature-grid layout: nhwc = channels-last, what the native "
                         "encoder writes (default); nchw = the reference's contiguous layout")
    ap.add_argument("--config", default="c2", choices=["c1", "c2", "c4", "c5", "vit", "encode", "train"],
                    help="c1: BASELINE configs[0] render shape (K=32, the demo's sampler); "
                         "c2: BASELINE configs[1] (K=64, D=64, the metric's config); c4: "
                         "configs[3] render shape (K=128, 384-d feature field); c5: "
                         "configs[4] SSCBench voxel query (voxels/s); vit: the DINO ViT "
                         "encoder forward (a19); encode: ViT + DPT decoder (DINOv2Module); "
                         "train: render forward + backward (training step)")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--no-graph", dest="graph", action="store_false",
                    help="--config train: issue the step eagerly instead of replaying it as a "
                         "captured HIP graph (host: patch draws + one graph launch; the default "
                         "on one GPU, round 4: 0.964 vs 0.983 ms per step)")
    ap.add_argument("--no-amp", action="store_true",
                    help="--config train: fp32 MLP instead of the reference's fp16 autocast")
    ap.add_argument("--no-fp16-line", action="store_true",
                    help="c1/c2 at bf16: skip the fp16 (library default precision) timing "
                         "reported beside value")
    ap.add_argument("--no-end-to-end", action="store_true",
                    help="c2: skip the encode + render frame timing reported beside value")
    ap.add_argument("--models", default="", help="--config encode/vit: comma list of "
                    "vit-s16, vit-b8, dinov2-b14 (default all)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: ranks share GPU 0 and exchange through host memory (dry run)")
    args = ap.parse_args()
    if args.precision == "fp8" and args.config != "c5":
        ap.error("--precision fp8 is the C5 voxel MLP chain (--config c5)")
    global K_SAMPLES, D_DINO, GRID_LAYOUT
    GRID_LAYOUT = args.grid_layout
    if args.config == "c4":
        K_SAMPLES, D_DINO = 128, 384
    elif args.config == "c1":
        K_SAMPLES = 32

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    dist = world > 1
    host_stage = dist and args.dist_backend == "gloo"
    dev_index = local_rank
    if host_stage:  # dry run: every rank on one shared GPU
        dev_index = local_rank % max(torch.cuda.device_count(), 1)
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(dev_index)
        if host_stage:
            tdist.init_process_group("gloo")
        else:
            # the render's persistent grids leave NCCL_MAX_NCHANNELS CUs to the all-gather
            # beside them (reserve_cus): bound RCCL's channels -- one workgroup each -- to that
            os.environ.setdefault("NCCL_MAX_NCHANNELS", "16")
            tdist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        if tdist.get_world_size() != args.gpus:
            raise SystemExit("bench.py: process-group size differs from --gpus")
    device = torch.device("cuda", dev_index)

    from scenedino_amd import _lib
    _lib.load()
    if args.config == "train":
        main_train(args, world, rank, device)
    elif args.config == "c5":
        main_c5(args, world, rank, local_rank, dist, device, host_stage)
    elif args.config == "vit":
        main_vit(args, world, rank, device)
    elif args.config == "encode":
        main_encode(args, world, rank, device)
    else:
        main_c2(args, world, rank, device, dist, host_stage)
    if dist:
        tdist.barrier()
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
