"""Generate golden input/output vectors from the reference (tum-vision/scenedino).

Run ONLY in the build container, where the read-only reference lives at
/root/reference:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports the reference's own Python modules (renderer, BTSNet, ray sampler,
pinhole camera, positional encoding, ResnetFC) with a handful of tiny stub
modules for third-party packages that are absent here and irrelevant to the
hot path (dotmap, cv2, torchvision, omegaconf), runs them on CPU in fp32 on
seeded inputs, and writes the inputs and outputs as ``.npz`` fixtures next to
this script.  Nothing from the reference is copied: the fixtures are data
(arrays), and this script only *calls* the reference.

Fixtures written (all float32 unless noted):
  gen_rays_small.npz      ImageRaySampler.sample at 24x80, two poses, 2 frames
  gen_rays_full.json      sha256 of the raw bytes of the 192x640 rays (bit-exact)
  sample_z.npz            NeRFRenderer.sample_coarse with injected jitter u
  field_query.npz         BTSNet.forward on raw points (sigma, dino, rgb, invalid)
  render_*.npz            NeRFRenderer(...).forward through BTSNet, 24x80 frames
  render_full_digest.json summary statistics of a 192x640x64 reference render
  ssc_scoring.json        SSCBench FOV mask digest + per-frame counts (fx_ssc_scoring)
"""
from __future__ import annotations

import contextlib
import hashlib
import json
import os
import sys
import types

import numpy as np
import torch

REF = os.environ.get("SCENEDINO_REF", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))

KITTI_K = [[0.7849, 0.0, -0.0312], [0.0, 2.9391, 0.2701], [0.0, 0.0, 1.0]]


# ----------------------------------------------------------------------------
# reference import harness
# ----------------------------------------------------------------------------
def _install_stubs():
    class DotMap(dict):
        def __getattr__(self, k):
            if k.startswith("__"):
                raise AttributeError(k)
            if k not in self:
                self[k] = DotMap()
            return self[k]

        def __setattr__(self, k, v):
            self[k] = v

        def toDict(self):
            out = {}
            for k, v in self.items():
                out[k] = v.toDict() if isinstance(v, DotMap) else v
            return out

    dm = types.ModuleType("dotmap")
    dm.DotMap = DotMap
    sys.modules["dotmap"] = dm

    cv2 = types.ModuleType("cv2")
    cv2.COLORMAP_HOT = 11
    sys.modules["cv2"] = cv2

    tv = types.ModuleType("torchvision")
    tvt = types.ModuleType("torchvision.transforms")
    tv.transforms = tvt
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.transforms"] = tvt

    oc = types.ModuleType("omegaconf")
    oc.ListConfig = list
    sys.modules["omegaconf"] = oc

    sys.path.insert(0, REF)
    import scenedino  # noqa: F401  (real package, light __init__)

    for sub in ("scenedino.models", "scenedino.models.prediction_heads"):
        m = types.ModuleType(sub)
        m.__path__ = [os.path.join(REF, *sub.split("."))]
        sys.modules[sub] = m


@contextlib.contextmanager
def _no_cuda_ones():
    orig = torch.ones

    def ones(*a, **kw):
        kw.pop("device", None)
        return orig(*a, **kw)

    torch.ones = ones
    try:
        yield
    finally:
        torch.ones = orig


def load_reference():
    _install_stubs()
    from scenedino.renderer.nerf import NeRFRenderer
    from scenedino.common.ray_sampler import ImageRaySampler
    from scenedino.common import util
    from scenedino.common.positional_encoding import PositionalEncoding
    from scenedino.models.prediction_heads.resnetfc import ResnetFC

    with _no_cuda_ones():
        from scenedino.models.bts import BTSNet
    return types.SimpleNamespace(
        NeRFRenderer=NeRFRenderer,
        ImageRaySampler=ImageRaySampler,
        util=util,
        PositionalEncoding=PositionalEncoding,
        ResnetFC=ResnetFC,
        BTSNet=BTSNet,
    )


class FakeEncoder(torch.nn.Module):
    """Stands in for DINOv2Module: returns a fixed feature grid (the ViT/DPT
    encoder is a separate row of the scope table)."""

    def __init__(self, grid):
        super().__init__()
        self.grid = grid  # (n*nv, C, h, w)
        self.latent_size = grid.shape[1]
        self.extra_outs = 0

    def forward(self, x, ground_truth=False):
        return [self.grid]


def make_pose(yaw_deg, tx, ty=0.0, tz=0.0):
    a = np.deg2rad(yaw_deg)
    p = np.eye(4, dtype=np.float32)
    p[0, 0], p[0, 2], p[2, 0], p[2, 2] = np.cos(a), np.sin(a), -np.sin(a), np.cos(a)
    p[:3, 3] = [tx, ty, tz]
    return torch.from_numpy(p)


def build_net(ref, grid, n_views_enc=1, dino_dims=64, d_hidden=128, seed=2, learn_empty=False):
    conf = {
        "predict_dino": True,
        "dino_dims": dino_dims,
        "learn_empty": learn_empty,
        "code_mode": "z",
        "inv_z": True,
        "z_near": 3,
        "z_far": 80,
        "sample_color": True,
    }
    torch.manual_seed(seed)
    code = ref.PositionalEncoding(num_freqs=6, d_in=3, freq_factor=1.5, include_input=True)
    enc = FakeEncoder(grid)
    d_in = enc.latent_size + code.d_out
    head = ref.ResnetFC(d_in=d_in, d_out=1 + dino_dims, n_blocks=0, d_hidden=d_hidden)
    # ResnetFC initialises biases to zero; perturb them so parity covers the bias path.
    with torch.no_grad():
        g = torch.Generator().manual_seed(seed + 100)
        head.lin_in.bias.copy_(0.1 * torch.randn(d_hidden, generator=g))
        head.lin_out.bias.copy_(0.1 * torch.randn(1 + dino_dims, generator=g))
    net = ref.BTSNet(conf, enc, code, {"normal_head": head}, final_pred_head="normal_head")
    if learn_empty:  # bts.py:90-93 draws it from the global RNG; make it seeded
        with torch.no_grad():
            net.empty_feature.copy_(torch.randn(enc.latent_size,
                                                generator=torch.Generator().manual_seed(seed + 7)))
    return net.eval()


def np32(t):
    return t.detach().cpu().numpy()


# ----------------------------------------------------------------------------
# fixtures
# ----------------------------------------------------------------------------
def fx_gen_rays(ref):
    out = {}
    K = torch.tensor(KITTI_K)
    poses = torch.stack([torch.eye(4), make_pose(2.0, 0.5, 0.1, 0.3)])  # (2,4,4)
    projs = torch.stack([K, K * torch.tensor([[1.05, 1, 1], [1, 0.97, 1], [1, 1, 1]])])
    sampler = ref.ImageRaySampler(z_near=3, z_far=80, height=24, width=80)
    rays, _ = sampler.sample(None, poses.view(1, 2, 4, 4), projs.view(1, 2, 3, 3))
    out["poses"] = np32(poses)
    out["projs"] = np32(projs)
    out["rays"] = np32(rays)  # (1, 2*24*80, 11)
    np.savez_compressed(os.path.join(HERE, "gen_rays_small.npz"), **out)

    digests = {}
    for name, P in (("identity", torch.eye(4)), ("offset", make_pose(2.0, 0.5, 0.1, 0.3))):
        s = ref.ImageRaySampler(z_near=3, z_far=80, height=192, width=640)
        r, _ = s.sample(None, P.view(1, 1, 4, 4), K.view(1, 1, 3, 3))
        digests[name] = {
            "pose": np32(P).tolist(),
            "shape": list(r.shape),
            "sha256": hashlib.sha256(np.ascontiguousarray(np32(r)).tobytes()).hexdigest(),
        }
    with open(os.path.join(HERE, "gen_rays_full.json"), "w") as f:
        json.dump({"K": KITTI_K, "near": 3, "far": 80, "H": 192, "W": 640, "cases": digests}, f, indent=1)


@contextlib.contextmanager
def injected_rand(u):
    orig = torch.rand_like

    def rl(x, *a, **kw):
        assert x.shape == u.shape, (x.shape, u.shape)
        return u.clone()

    torch.rand_like = rl
    try:
        yield
    finally:
        torch.rand_like = orig


def fx_sample_z(ref):
    g = torch.Generator().manual_seed(3)
    rays = np.load(os.path.join(HERE, "gen_rays_small.npz"))["rays"][0][:512]
    rays = torch.from_numpy(rays)
    out = {"rays": np32(rays)}
    for K in (8, 32, 64, 128):
        u = torch.rand(rays.shape[0], K, generator=g)
        for lindisp in (True, False):
            r = ref.NeRFRenderer(n_coarse=K, lindisp=lindisp)
            with injected_rand(u):
                z = r.sample_coarse(rays)
            out[f"u_{K}"] = np32(u)
            out[f"z_{K}_{int(lindisp)}"] = np32(z)
    np.savez_compressed(os.path.join(HERE, "sample_z.npz"), **out)

    # full-size bit-exact digest at 192x640x64 with seeded u
    K = torch.tensor(KITTI_K)
    s = ref.ImageRaySampler(z_near=3, z_far=80, height=192, width=640)
    full, _ = s.sample(None, torch.eye(4).view(1, 1, 4, 4), K.view(1, 1, 3, 3))
    full = full[0]
    u = torch.rand(full.shape[0], 64, generator=torch.Generator().manual_seed(7))
    r = ref.NeRFRenderer(n_coarse=64, lindisp=True)
    with injected_rand(u):
        z = r.sample_coarse(full)
    with open(os.path.join(HERE, "sample_z_full.json"), "w") as f:
        json.dump({"seed": 7, "K": 64, "lindisp": True,
                   "u_sha256": hashlib.sha256(np32(u).tobytes()).hexdigest(),
                   "z_sha256": hashlib.sha256(np32(z).tobytes()).hexdigest()}, f, indent=1)


def make_scene(n, nv_render, C, gh, gw, H, W, seed, offset_render=True):
    """Inputs for encode(): images (n, nv, 3, H, W) in [-1,1], Ks, c2w poses.
    view 0 = encoder view; views 0..nv_render-1 are render (colour) views."""
    g = torch.Generator().manual_seed(seed)
    images = torch.rand(n, nv_render, 3, H, W, generator=g) * 2 - 1
    K = torch.tensor(KITTI_K)
    Ks = K.view(1, 1, 3, 3).repeat(n, nv_render, 1, 1)
    poses = torch.eye(4).view(1, 1, 4, 4).repeat(n, nv_render, 1, 1)
    for b in range(n):
        for v in range(nv_render):
            if v > 0 or (b > 0 and offset_render):
                poses[b, v] = make_pose(1.5 * v + 0.7 * b, 0.4 * v + 0.2 * b, 0.05 * v, 0.3 * v)
    grid = torch.randn(n, C, gh, gw, generator=g)
    return images, Ks, poses, grid


def fx_field_query(ref, learn_empty=False):
    """BTSNet.forward on raw world points (the SSCBench / inference_3d call)."""
    n, C, gh, gw, H, W = 1, 256, 12, 40, 24, 80
    images, Ks, poses, grid = make_scene(n, 1, C, gh, gw, H, W, seed=11)
    net = build_net(ref, grid, learn_empty=learn_empty)
    net.encode(images, Ks, poses, ids_encoder=[0], ids_render=[0])
    g = torch.Generator().manual_seed(12)
    P = 4096
    xyz = torch.empty(1, P, 3)
    xyz[..., 0] = (torch.rand(P, generator=g) * 2 - 1) * 25.0
    xyz[..., 1] = (torch.rand(P, generator=g) * 2 - 1) * 4.0
    xyz[..., 2] = torch.rand(P, generator=g) * 90.0 - 5.0  # includes z<=eps and far points
    with torch.no_grad():
        rgb, invalid, sigma, extras, sd = net(xyz)
    head = net.heads["normal_head"]
    extra = {"empty_feature": np32(net.empty_feature)} if learn_empty else {}
    np.savez_compressed(
        os.path.join(HERE, "field_query_empty.npz" if learn_empty else "field_query.npz"), **extra,
        images=np32(images), Ks=np32(Ks), poses=np32(poses), grid=np32(grid),
        W_in=np32(head.lin_in.weight), b_in=np32(head.lin_in.bias),
        W_out=np32(head.lin_out.weight), b_out=np32(head.lin_out.bias),
        xyz=np32(xyz), rgb=np32(rgb), invalid=np32(invalid), sigma=np32(sigma),
        dino=np32(sd["dino_features"]), invalid_features=np32(sd["invalid_features"]),
    )


def fx_render(ref, name, n, nv_render, K, hard_cap, H=24, W=80, gh=12, gw=40, seed=21,
              learn_empty=False, render_offset=None):
    C = 256
    images, Ks, poses, grid = make_scene(n, nv_render, C, gh, gw, H, W, seed=seed)
    net = build_net(ref, grid.view(n, C, gh, gw), learn_empty=learn_empty)
    net.encode(images, Ks, poses, ids_encoder=[0], ids_render=list(range(nv_render)))
    renderer = ref.NeRFRenderer(n_coarse=K, lindisp=True, hard_alpha_cap=hard_cap,
                                eval_batch_size=65536)
    wrapper = renderer.bind_parallel(net, gpus=None).eval()
    sampler = ref.ImageRaySampler(z_near=3, z_far=80, height=H, width=W)
    # render view: view 0 of each batch element (the encoder view), as the demo does
    rpose = poses[:, :1]
    if render_offset is not None:  # render from a moved camera: rays leave the encoder frustum
        rpose = rpose @ make_pose(*render_offset).view(1, 1, 4, 4)
    rays, _ = sampler.sample(None, rpose, Ks[:, :1])
    g = torch.Generator().manual_seed(seed + 1)
    u = torch.rand(rays.shape[0] * rays.shape[1], K, generator=g)
    with torch.no_grad(), injected_rand(u):
        out = wrapper(rays, want_weights=True, want_alphas=True, want_z_samps=True,
                      want_rgb_samps=True)
    c = out["coarse"]
    head = net.heads["normal_head"]
    extra = {"empty_feature": np32(net.empty_feature)} if learn_empty else {}
    np.savez_compressed(
        os.path.join(HERE, f"render_{name}.npz"), **extra,
        images=np32(images), Ks=np32(Ks), poses=np32(poses), grid=np32(grid),
        W_in=np32(head.lin_in.weight), b_in=np32(head.lin_in.bias),
        W_out=np32(head.lin_out.weight), b_out=np32(head.lin_out.bias),
        rays=np32(rays), u=np32(u), K=np.int64(K), hard_cap=np.int64(hard_cap),
        nv_render=np.int64(nv_render),
        rgb=np32(c["rgb"]), depth=np32(c["depth"]), invalid=np32(c["invalid"]),
        ray_info=np32(c["ray_info"]), weights=np32(c["weights"]), alphas=np32(c["alphas"]),
        z_samps=np32(c["z_samps"]), rgb_samps=np32(c["rgb_samps"]),
        dino_features=np32(c["dino_features"]),
        invalid_features=np32(c["invalid_features"]),
        sd_dino=np32(out["state_dict"]["dino_features"]),
    )


def fx_render_full_digest(ref):
    """One 192x640x64 render (the BASELINE C2 shape, fp32 reference) at a small
    grid; store summary statistics + a strided subsample of the outputs."""
    H, W, K = 192, 640, 64
    n, C, gh, gw = 1, 256, 48, 160
    images, Ks, poses, grid = make_scene(n, 1, C, gh, gw, H, W, seed=31)
    net = build_net(ref, grid)
    net.encode(images, Ks, poses, ids_encoder=[0], ids_render=[0])
    renderer = ref.NeRFRenderer(n_coarse=K, lindisp=True, hard_alpha_cap=False,
                                eval_batch_size=65536)
    wrapper = renderer.bind_parallel(net, gpus=None).eval()
    sampler = ref.ImageRaySampler(z_near=3, z_far=80, height=H, width=W)
    rays, _ = sampler.sample(None, poses[:, :1], Ks[:, :1])
    u = torch.rand(rays.shape[1], K, generator=torch.Generator().manual_seed(32))
    with torch.no_grad(), injected_rand(u):
        out = wrapper(rays, want_weights=True, want_alphas=True)
    c = out["coarse"]
    idx = np.arange(0, H * W, 97)
    np.savez_compressed(
        os.path.join(HERE, "render_full_subsample.npz"),
        grid_seed=np.int64(31), u_seed=np.int64(32), idx=idx,
        depth=np32(c["depth"])[0, idx], dino=np32(c["dino_features"])[0, idx],
        rgb=np32(c["rgb"])[0, idx], weights=np32(c["weights"])[0, idx],
        depth_mean=np.float64(c["depth"].double().mean()),
        dino_abs_mean=np.float64(c["dino_features"].double().abs().mean()),
    )


def fx_render_full_offset(ref):
    """The BASELINE C2 shape (192x640x64, fp32 reference) at the full 256x192x640 feature
    grid, rays from the 0.5 m lateral / 2 deg yaw render pose of SURVEY §8(d) (encoder and
    colour view at the identity): strided subsample of every output, digests of the full
    masks, summary statistics."""
    import hashlib
    H, W, K = 192, 640, 64
    n, C, gh, gw = 1, 256, 192, 640
    images, Ks, poses, grid = make_scene(n, 1, C, gh, gw, H, W, seed=61)
    net = build_net(ref, grid)
    net.encode(images, Ks, poses, ids_encoder=[0], ids_render=[0])
    renderer = ref.NeRFRenderer(n_coarse=K, lindisp=True, hard_alpha_cap=False,
                                eval_batch_size=65536)
    wrapper = renderer.bind_parallel(net, gpus=None).eval()
    sampler = ref.ImageRaySampler(z_near=3, z_far=80, height=H, width=W)
    render_pose = make_pose(2.0, 0.5).view(1, 1, 4, 4)
    rays, _ = sampler.sample(None, render_pose, Ks[:, :1])
    u = torch.rand(rays.shape[1], K, generator=torch.Generator().manual_seed(62))
    with torch.no_grad(), injected_rand(u):
        out = wrapper(rays, want_weights=True, want_alphas=True)
    c = out["coarse"]
    idx = np.arange(0, H * W, 61)
    sha = lambda t: hashlib.sha256(np.ascontiguousarray(np32(t)).tobytes()).hexdigest()
    np.savez_compressed(
        os.path.join(HERE, "render_full_offset.npz"),
        scene_seed=np.int64(61), u_seed=np.int64(62), idx=idx,
        render_pose=np32(render_pose),
        depth=np32(c["depth"])[0, idx], dino=np32(c["dino_features"])[0, idx],
        rgb=np32(c["rgb"])[0, idx], weights=np32(c["weights"])[0, idx],
        alphas=np32(c["alphas"])[0, idx],
        invalid_sha256=np.array(sha(c["invalid"])),
        invalid_features_sha256=np.array(sha(c["invalid_features"])),
        invalid_shape=np.array(c["invalid"].shape), invalid_features_shape=np.array(c["invalid_features"].shape),
        depth_mean=np.float64(c["depth"].double().mean()),
        dino_abs_mean=np.float64(c["dino_features"].double().abs().mean()),
        weights_sum_mean=np.float64(c["weights"].double().sum(-1).mean()),
    )



def fx_render_full_offset_k32(ref):
    """BASELINE configs[0]'s sample count (K = 32, configs/renderer/pixelnerf.yaml:1) on the
    scene of fx_render_full_offset (256x192x640 grid, seed 61), whole 192x640 frame from the
    same offset render pose, jitter seed 63: strided subsample of every output (every 61st
    ray), SHA-256 of the whole-frame masks, summary statistics."""
    import hashlib
    H, W, K = 192, 640, 32
    n, C, gh, gw = 1, 256, 192, 640
    images, Ks, poses, grid = make_scene(n, 1, C, gh, gw, H, W, seed=61)
    net = build_net(ref, grid)
    net.encode(images, Ks, poses, ids_encoder=[0], ids_render=[0])
    renderer = ref.NeRFRenderer(n_coarse=K, lindisp=True, hard_alpha_cap=False,
                                eval_batch_size=65536)
    wrapper = renderer.bind_parallel(net, gpus=None).eval()
    sampler = ref.ImageRaySampler(z_near=3, z_far=80, height=H, width=W)
    render_pose = make_pose(2.0, 0.5).view(1, 1, 4, 4)
    rays, _ = sampler.sample(None, render_pose, Ks[:, :1])
    u = torch.rand(rays.shape[1], K, generator=torch.Generator().manual_seed(63))
    with torch.no_grad(), injected_rand(u):
        out = wrapper(rays, want_weights=True, want_alphas=True)
    c = out["coarse"]
    idx = np.arange(0, H * W, 61)
    sha = lambda t: hashlib.sha256(np.ascontiguousarray(np32(t)).tobytes()).hexdigest()
    np.savez_compressed(
        os.path.join(HERE, "render_full_offset_k32.npz"),
        scene_seed=np.int64(61), u_seed=np.int64(63), K=np.int64(K), idx=idx,
        render_pose=np32(render_pose),
        depth=np32(c["depth"])[0, idx], dino=np32(c["dino_features"])[0, idx],
        rgb=np32(c["rgb"])[0, idx], weights=np32(c["weights"])[0, idx],
        alphas=np32(c["alphas"])[0, idx],
        invalid_sha256=np.array(sha(c["invalid"])),
        invalid_features_sha256=np.array(sha(c["invalid_features"])),
        invalid_shape=np.array(c["invalid"].shape),
        invalid_features_shape=np.array(c["invalid_features"].shape),
        depth_mean=np.float64(c["depth"].double().mean()),
        dino_abs_mean=np.float64(c["dino_features"].double().abs().mean()),
        weights_sum_mean=np.float64(c["weights"].double().sum(-1).mean()),
    )


def fx_render_c4_offset(ref):
    """BASELINE configs[3]'s render shape: 128 samples per ray and a 384-d feature field
    (ResnetFC 295 -> 128 -> 385, configs/model/*: dino_dims 384) over the 256x192x640 grid of
    fx_render_full_offset's scene (seed 61), rays from the same offset render pose.  The
    reference renders a strided subsample of the frame's rays only (every 61st ray, 2 015
    rays x 128 samples -- the whole frame would hold 24 GB of per-sample 384-d features on
    the CPU); the rays are independent, so the GPU test renders the WHOLE frame with the
    same per-ray jitter rows (seed 64 over all 122 880 rays) and compares these rays.  The
    head's weights are stored (d_out 385 changes the kaiming draw)."""
    H, W, K, D = 192, 640, 128, 384
    n, C, gh, gw = 1, 256, 192, 640
    images, Ks, poses, grid = make_scene(n, 1, C, gh, gw, H, W, seed=61)
    net = build_net(ref, grid, dino_dims=D)
    net.encode(images, Ks, poses, ids_encoder=[0], ids_render=[0])
    renderer = ref.NeRFRenderer(n_coarse=K, lindisp=True, hard_alpha_cap=False,
                                eval_batch_size=65536)
    wrapper = renderer.bind_parallel(net, gpus=None).eval()
    sampler = ref.ImageRaySampler(z_near=3, z_far=80, height=H, width=W)
    render_pose = make_pose(2.0, 0.5).view(1, 1, 4, 4)
    rays, _ = sampler.sample(None, render_pose, Ks[:, :1])
    u = torch.rand(rays.shape[1], K, generator=torch.Generator().manual_seed(64))
    idx = np.arange(0, H * W, 61)
    it = torch.from_numpy(idx)
    with torch.no_grad(), injected_rand(u[it]):
        out = wrapper(rays[:, it], want_weights=True, want_alphas=True)
    c = out["coarse"]
    head = net.heads["normal_head"]
    np.savez_compressed(
        os.path.join(HERE, "render_c4_offset.npz"),
        scene_seed=np.int64(61), u_seed=np.int64(64), K=np.int64(K), D=np.int64(D), idx=idx,
        render_pose=np32(render_pose),
        W_in=np32(head.lin_in.weight), b_in=np32(head.lin_in.bias),
        W_out=np32(head.lin_out.weight), b_out=np32(head.lin_out.bias),
        depth=np32(c["depth"])[0], dino=np32(c["dino_features"])[0], rgb=np32(c["rgb"])[0],
        weights=np32(c["weights"])[0], alphas=np32(c["alphas"])[0],
        invalid=np32(c["invalid"])[0].astype(np.uint8),
        invalid_features=np32(c["invalid_features"])[0].astype(np.uint8),
    )

def load_reference_seg():
    """The reference's MlpDimReduction and SemanticHead pieces (CPU).  semantic_head.py
    imports the CRF helper (pydensecrf, torchvision.transforms.functional: absent here,
    unused by the inference path) -> stub modules; SemanticHead.__init__ allocates its
    training buffers on "cuda", so the head object is assembled with its reference
    sub-modules and its own (unbound) forward is called."""
    for name in ("pydensecrf", "pydensecrf.densecrf", "pydensecrf.utils",
                 "torchvision.transforms.functional"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["pydensecrf"].densecrf = sys.modules["pydensecrf.densecrf"]
    sys.modules["pydensecrf"].utils = sys.modules["pydensecrf.utils"]
    for sub in ("scenedino.models.backbones", "scenedino.models.backbones.dino"):
        m = types.ModuleType(sub)
        m.__path__ = [os.path.join(REF, *sub.split("."))]
        sys.modules[sub] = m
    from scenedino.models.backbones.dino.dim_reduction import MlpDimReduction
    from scenedino.downstream_head import semantic_head as sh
    return MlpDimReduction, sh


def fx_seg_head():
    """transform_expand (dim_reduction.py:22-25) + SemanticHead.forward "stego_kmeans"
    (semantic_head.py:107-111) on seeded 64-d DINO codes; d_full 768 (ViT-B) and 384
    (ViT-S, configs/downstream/semantic.yaml input_dim)."""
    MlpDimReduction, sh = load_reference_seg()
    out = {}
    for d_full in (768, 384):
        torch.manual_seed(60 + d_full)
        dr = MlpDimReduction(d_full, 64, latent_channels=128).eval()
        stego = sh.StegoClusterHead(d_full, 64).eval()
        clus = sh.KMeansParamHead(19, 19, 64).eval()
        with torch.no_grad():
            clus.pseudo_assignment.copy_((torch.arange(19) * 7 + 3) % 19)
        head = torch.nn.Module()
        head.stego_head, head.stego_cluster_head = stego, clus
        g = torch.Generator().manual_seed(61)
        P = 2048
        x = torch.randn(P, 64, generator=g) * 0.5
        x[:16] *= 40.0     # large codes
        x[16:32] *= 1e-3   # tiny codes
        x[32] = 0.0        # zero code -> relu(b1) path
        with torch.no_grad():
            full = dr.transform_expand(x.view(1, P, 64))
            seg = sh.SemanticHead.forward(head, full, mode="stego_kmeans")
        t = f"_{d_full}"
        out.update({
            "x" + t: np32(x), "full" + t: np32(full[0, :256]), "labels" + t: seg[0].numpy(),
            "W1" + t: np32(dr.linear_in.weight), "b1" + t: np32(dr.linear_in.bias),
            "W2" + t: np32(dr.linear_out.weight), "b2" + t: np32(dr.linear_out.bias),
            "Wl" + t: np32(stego.linear_path[0].weight), "bl" + t: np32(stego.linear_path[0].bias),
            "Wn1" + t: np32(stego.nonlinear_path[0].weight),
            "bn1" + t: np32(stego.nonlinear_path[0].bias),
            "Wn2" + t: np32(stego.nonlinear_path[2].weight),
            "bn2" + t: np32(stego.nonlinear_path[2].bias),
            "centres" + t: np32(clus.cluster_centers), "assign" + t: clus.pseudo_assignment.numpy(),
        })
    np.savez_compressed(os.path.join(HERE, "seg_head.npz"), **out)


def fx_voxel_points():
    """SSCBench voxel-centre grid (evaluate_model_sscbench.py:270-278 -> point_utils.py:17-82).
    numba is absent here, so TSDFVolume.vox2world (fusion.py:203-219: float32 inputs, f64
    arithmetic in a numba loop, float32 store) is restated in numpy with explicit f64
    promotion; rigid_transform (fusion.py:407-411) is the reference's own numpy call
    sequence (hstack + np.dot with the f64 transform, a BLAS dgemm); .float() rounds once.
    T = read_calib()["Tr"] (point_utils.py:84-137), restated from its constants."""
    cam2velo = np.array([0.04307104361, -0.08829286498, 0.995162929, 0.8043914418,
                         -0.999004371, 0.007784614041, 0.04392796942, 0.2993489574,
                         -0.01162548558, -0.9960641394, -0.08786966659, -0.1770225824]).reshape(3, 4)
    C2V = np.concatenate([cam2velo, np.array([0, 0, 0, 1]).reshape(1, 4)], axis=0)
    T = np.identity(4)
    T[:3, :4] = np.linalg.inv(C2V)[:3, :]
    origin = np.array([0, -25.6, -2])
    dims = np.ceil(np.array([51.2, 51.2, 6.4]) / 0.2).astype(int)
    xv, yv, zv = np.meshgrid(range(dims[0]), range(dims[1]), range(dims[2]), indexing="ij")
    coords = np.stack([xv.reshape(-1), yv.reshape(-1), zv.reshape(-1)], 1).astype(np.float32)
    o32 = origin.astype(np.float32).astype(np.float64)
    cam = ((o32[None] + 0.2 * coords.astype(np.float64)) + 0.2 * 0.5).astype(np.float32)
    xyz_h = np.hstack([cam, np.ones((len(cam), 1), dtype=np.float32)])
    pts = torch.tensor(np.dot(T, xyz_h.T).T[:, :3]).float().numpy()
    sel = np.arange(0, len(pts), 2049)
    with open(os.path.join(HERE, "voxel_points.json"), "w") as f:
        json.dump({"origin": origin.tolist(), "voxel_size": 0.2, "dims": dims.tolist(),
                   "T": T.tolist(), "sha256": hashlib.sha256(pts.tobytes()).hexdigest(),
                   "slice_stride": 2049, "slice": pts[sel].tolist()}, f)


def _ref_functions(path, names, ns, cls=None):
    """Execute the named top-level (or ``cls`` static-method) function definitions of a
    reference file, decorators dropped, in namespace ``ns``; returns ns.  Used where the
    module itself cannot be imported here (hydra, matplotlib, numba, skimage at import)."""
    import ast
    src = open(path).read()
    tree = ast.parse(src)
    body = tree.body
    if cls is not None:
        body = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == cls][0].body
    defs = []
    for n in body:
        if isinstance(n, ast.FunctionDef) and n.name in names:
            n.decorator_list = []
            defs.append(n)
    assert {d.name for d in defs} == set(names), (path, names)
    exec(compile(ast.Module(body=defs, type_ignores=[]), path, "exec"), ns)
    return ns


def fx_ssc_scoring():
    """SSCBench scoring (sscbench/evaluate_model_sscbench.py): the FOV mask from the
    reference's generate_point_grid (point_utils.py:17-82) with its cam2pix (fusion.py:222-232,
    the numba loop run as plain Python: f64 arithmetic either way) and rigid_transform
    (fusion.py:407-411); vox2world (numba; numpy 2 scalar promotion would differ) is the
    restatement pinned by voxel_points.json.  Then, on the seeded frames of
    tests/_ssc_inputs.py, the reference's own convert_voxels / identify_additional_invalids /
    compute_occupancy_numbers(_segmentation) / compute_occupancy_recall_segmentation, glued
    as the main loop does (:366-367, 452-456, 492, 496-507)."""
    import yaml
    sys.path.insert(0, os.path.dirname(HERE))
    from _ssc_inputs import make_frame
    ssc = os.path.join(REF, "sscbench")
    fus = _ref_functions(os.path.join(ssc, "fusion.py"), ["rigid_transform"], {"np": np})
    fus = _ref_functions(os.path.join(ssc, "fusion.py"), ["cam2pix"], dict(fus, prange=range),
                         cls="TSDFVolume")

    def vox2world(vol_origin, vox_coords, vox_size, offsets=(0.5, 0.5, 0.5)):
        o32 = np.asarray(vol_origin).astype(np.float32).astype(np.float64)
        c = vox_coords.astype(np.float32).astype(np.float64)
        return ((o32[None] + vox_size * c) + vox_size * 0.5).astype(np.float32)

    tsdf = types.SimpleNamespace(vox2world=vox2world, cam2pix=fus["cam2pix"])
    pu = _ref_functions(os.path.join(ssc, "point_utils.py"),
                        ["generate_point_grid", "read_calib"],
                        {"np": np, "TSDFVolume": tsdf, "rigid_transform": fus["rigid_transform"]})
    gps = _ref_functions(os.path.join(ssc, "generate_ply_sequence.py"), ["get_cam_k"], {"np": np})
    calib = pu["read_calib"]()
    _, fov = pu["generate_point_grid"](vox_origin=np.array([0, -25.6, -2]),
                                       scene_size=(51.2, 51.2, 6.4), voxel_size=0.2,
                                       cam_E=calib["Tr"], cam_k=gps["get_cam_k"]())
    fov = fov.reshape(256, 256, 32)
    ev = _ref_functions(os.path.join(ssc, "evaluate_model_sscbench.py"),
                        ["convert_voxels", "identify_additional_invalids",
                         "compute_occupancy_numbers", "compute_occupancy_numbers_segmentation",
                         "compute_occupancy_recall_segmentation"], {"np": np})
    with open(os.path.join(ssc, "label_maps.yaml")) as f:
        label_maps = yaml.safe_load(f)
    frames = []
    for seed in (0, 1):
        sigmas, segs, gt = make_frame(seed)
        segs = ev["convert_voxels"](segs.astype(np.float64), label_maps["cityscapes_to_label"])
        target = ev["convert_voxels"](gt.astype(int), label_maps["sscbench_to_label"])
        invalids = ev["identify_additional_invalids"](target)
        target[invalids == 1] = 255
        segs[sigmas < 0.2] = 0
        per = {}
        for size in (12.8, 25.6, 51.2):
            n = int(size // 0.2)
            sl = (slice(None, n), slice(128 - n // 2, 128 + n // 2), slice(None))
            tp, fp, tn, fn = ev["compute_occupancy_numbers"](
                y_pred=segs[sl], y_true=target[sl], fov_mask=fov[sl])
            tps, fps, tns, fns, conf = ev["compute_occupancy_numbers_segmentation"](
                y_pred=segs[sl], y_true=target[sl], fov_mask=fov[sl], labels=label_maps["labels"])
            tpr, sumr = ev["compute_occupancy_recall_segmentation"](
                y_pred=segs[sl], y_true=target[sl], fov_mask=fov[sl], labels=label_maps["labels"])
            per[str(size)] = {"tp": int(tp), "fp": int(fp), "tn": int(tn), "fn": int(fn),
                              "tp_seg": tps.astype(int).tolist(), "fp_seg": fps.astype(int).tolist(),
                              "tn_seg": tns.astype(int).tolist(), "fn_seg": fns.astype(int).tolist(),
                              "confusion_seg": conf.astype(int).tolist(),
                              "tp_recall_seg": tpr.astype(int).tolist(),
                              "sum_recall_seg": sumr.astype(int).tolist()}
        frames.append({"seed": seed, "n_additional_invalids": int(invalids.sum()), "sizes": per})
    with open(os.path.join(HERE, "ssc_scoring.json"), "w") as f:
        json.dump({"fov_sha256": hashlib.sha256(fov.astype(np.uint8).tobytes()).hexdigest(),
                   "fov_count": int(fov.sum()), "label_maps": label_maps, "frames": frames}, f)


def fx_patch_sampler(ref):
    """PatchRaySampler.sample (ray_sampler.py:136-287) with snap_to_grid: three cases on
    seeded inputs, the global torch RNG seeded before each call (its randint draws pick
    the patches)."""
    from scenedino.common.ray_sampler import PatchRaySampler
    g = torch.Generator().manual_seed(71)
    n, v, c, h, w = 2, 2, 3, 24, 80
    images = torch.rand(n, v, c, h, w, generator=g) * 2 - 1
    K = torch.tensor(KITTI_K)
    Ks = K.view(1, 1, 3, 3).repeat(n, v, 1, 1)
    poses = torch.stack([torch.stack([make_pose(3.0 * b + 1.1 * vv, 0.3 * vv, 0.1 * b)
                                      for vv in range(v)]) for b in range(n)])
    dino = torch.randn(n, v, 16, 3, 10, generator=g)
    dino_up = torch.randn(n, v, 8, h, w, generator=g)
    cases = {
        "grid": dict(ps=8, rb=512, up=False, shift=None, seed=5),
        "shift": dict(ps=8, rb=512, up=False, shift=(-3, 5), seed=6),
        "upscaled": dict(ps=(4, 8), rb=64, up=True, shift=None, seed=7),
    }
    out = {"images": np32(images), "Ks": np32(Ks), "poses": np32(poses), "dino": np32(dino),
           "dino_up": np32(dino_up)}
    for name, cs in cases.items():
        smp = PatchRaySampler(3.0, 80.0, cs["rb"], cs["ps"], snap_to_grid=True,
                              dino_upscaled=cs["up"])
        torch.manual_seed(cs["seed"])
        shift = torch.tensor(cs["shift"]) if cs["shift"] is not None else None
        rays, rgb, dg = smp.sample(images, poses, Ks, dino_features=dino_up if cs["up"] else dino,
                                   loss_feature_grid_shift=shift)
        out[f"{name}_rays"], out[f"{name}_rgb"], out[f"{name}_dino"] = np32(rays), np32(rgb), np32(dg)
        out[f"{name}_meta"] = np.array([cs["rb"], *(cs["ps"] if isinstance(cs["ps"], tuple) else (cs["ps"],) * 2),
                                        int(cs["up"]), cs["seed"],
                                        *(cs["shift"] if cs["shift"] else (0, 0)),
                                        int(cs["shift"] is not None)], np.int64)
    np.savez_compressed(os.path.join(HERE, "patch_sampler.npz"), **out)


def fx_salience_downsampler():
    """PatchSalienceDownsampler (models/backbones/dino/downsampler.py:31-98), featup with
    normalize_features=True as build_downsampler makes it (dinov2_module.py:59-62): forward
    (patch mode) and the autograd gradients of a seeded linear loss of its output."""
    _install_stubs()
    for sub in ("scenedino.models.backbones", "scenedino.models.backbones.dino"):
        m = types.ModuleType(sub)  # bare packages: skip the heavy backbone __init__ imports
        m.__path__ = [os.path.join(REF, *sub.split("."))]
        sys.modules[sub] = m
    from scenedino.models.backbones.dino.downsampler import PatchSalienceDownsampler
    out = {}
    for name, (n, p, ps, c) in {"p8c64": (2, 5, 8, 64), "p14c768": (1, 3, 14, 768)}.items():
        torch.manual_seed(81)
        m = PatchSalienceDownsampler(c, ps, True)
        g = torch.Generator().manual_seed(82)
        x = torch.randn(n, p, ps, ps, 1, c, generator=g).requires_grad_(True)
        gout = torch.randn(n, p, 1, c, generator=g)
        res, sal, wmap, pwb = m(x, "patch")
        (res * gout).sum().backward()
        out.update({f"{name}_x": np32(x), f"{name}_gout": np32(gout),
                    f"{name}_conv_w": np32(m.conv.weight), f"{name}_conv_b": np32(m.conv.bias),
                    f"{name}_pw": np32(m.patch_weight), f"{name}_pb": np32(m.patch_bias),
                    f"{name}_out": np32(res), f"{name}_sal": np32(sal), f"{name}_wmap": np32(wmap),
                    f"{name}_gx": np32(x.grad), f"{name}_gconv_w": np32(m.conv.weight.grad),
                    f"{name}_gconv_b": np32(m.conv.bias.grad), f"{name}_gpw": np32(m.patch_weight.grad),
                    f"{name}_gpb": np32(m.patch_bias.grad)})
    np.savez_compressed(os.path.join(HERE, "salience_downsampler.npz"), **out)


def fx_visualization():
    """VisualizationModule (models/backbones/dino/visualization.py:9-153), the encoder's
    PCA / k-means colouring API (dinov2_module.py:156,194-201): fit_pca under a seeded global
    RNG (torch.pca_lowrank draws its sketch from it), transform_pca in every mode the callers
    use, and fit_transform_kmeans_batch.  pykeops is absent: its ``LazyTensor`` is stubbed by
    the dense equivalent of the two operations the k-means loop uses (``x_i | c_j`` = the
    (N, K) dot products, ``.argmax(dim=1)``), so the loop itself is the reference's."""
    import importlib.util
    pk = types.ModuleType("pykeops")
    pkt = types.ModuleType("pykeops.torch")

    class LazyTensor:  # dense stand-in for the two LazyTensor ops of visualization.py:142-143
        def __init__(self, t):
            self.t = t

        def __or__(self, other):
            return LazyTensor((self.t * other.t).sum(-1))

        def argmax(self, dim):
            return self.t.argmax(dim=dim)

    pkt.LazyTensor = LazyTensor
    pk.torch = pkt
    sys.modules["pykeops"], sys.modules["pykeops.torch"] = pk, pkt
    spec = importlib.util.spec_from_file_location(
        "ref_visualization", os.path.join(REF, "scenedino/models/backbones/dino/visualization.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    g = torch.Generator().manual_seed(91)
    feats = torch.randn(600, 64, generator=g) @ torch.randn(64, 64, generator=g) * 0.3 + 0.1
    feats[[5, 77, 301]] = float("nan")
    img = torch.randn(6, 10, 64, generator=g) + 0.2
    vis = mod.VisualizationModule(768)
    torch.manual_seed(92)
    vis.fit_pca(feats, refit=True)
    out = {"feats": np32(feats), "img": np32(img), "mean": np32(vis.batch_rgb_mean),
           "comp": np32(vis.batch_rgb_comp)}
    for fd in (0, 3, 6):
        for norm in (False, True):
            out[f"t_{fd}_{int(norm)}"] = np32(vis.transform_pca(img, norm, fd))
    km_in = torch.randn(3, 40, 1, 64, generator=g)
    km_in[:, :, :, :4] += 2.0 * torch.randn(3, 40, 1, 4, generator=g).sign()
    out["km_in"] = np32(km_in)
    out["km_map"] = np32(vis.fit_transform_kmeans_batch(km_in))
    out["km_centers"] = np32(vis.kmeans_cluster_centers)
    np.savez_compressed(os.path.join(HERE, "visualization.npz"), **out)


def det_fill(module, seed):
    """Deterministic parameter fill by sorted state_dict name (shared with tests/test_dpt.py):
    weights N(0, 1/fan) with fan = numel of one output slice, vectors N(0, 0.05^2)."""
    g = torch.Generator().manual_seed(seed)
    sd = module.state_dict()
    with torch.no_grad():
        for name in sorted(sd):
            t = sd[name]
            if t.dim() > 1:
                t.copy_(torch.randn(t.shape, generator=g) / float(t[0].numel()) ** 0.5)
            else:
                t.copy_(0.05 * torch.randn(t.shape, generator=g))


def fx_dpt():
    """The reference's DPTHead (dpt_head.py:179-236, only torch imports) with the shipped
    decoder shape (embed 384 = ViT-S, post_process_channels [64, 64, 128, 256], d_out 256,
    configs/model/dino_downsampler.yaml:22-25) on a 2 x 4 token grid."""
    sys.path.insert(0, REF)
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "ref_dpt_head", os.path.join(REF, "scenedino/models/backbones/dino/dpt_head.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    head = mod.DPTHead(embed_dims=384, post_process_channels=[64, 64, 128, 256],
                       readout_type="ignore", patch_size=16, d_out=256, expand_channels=False).eval()
    det_fill(head, 70)
    g = torch.Generator().manual_seed(71)
    inputs = [torch.randn(1, 384, 2, 4, generator=g) for _ in range(4)]
    with torch.no_grad():
        out = head(inputs)[0]
    np.savez_compressed(os.path.join(HERE, "dpt_head.npz"),
                        **{f"in{i}": np32(x) for i, x in enumerate(inputs)},
                        out=np32(out).astype(np.float16), out_norm=np.float64(out.double().norm()))


def fx_state_dict_manifest(ref):
    """Key -> shape manifest of the reference modules whose parameters the build must load
    unchanged (checkpoint.pt, load_state_dict(strict=False), demo_utils/utils.py:52-55):
    ResnetFC / BTSNet heads (models/__init__.py:30-44, configs/model/dino_downsampler.yaml),
    NeRFRenderer buffers (nerf.py:106-111), DPTHead for ViT-S and ViT-B embeddings
    (dpt_head.py:179-236), MlpDimReduction (dim_reduction.py:15-25) and SemanticHead
    (semantic_head.py:40-100, both head variants).  Shapes only -- no weights."""
    import importlib.util
    man = {}
    sd_shapes = lambda m, drop=(): {k: list(v.shape) for k, v in m.state_dict().items()
                                     if not k.startswith(drop)}
    head = ref.ResnetFC(d_in=295, d_out=65, n_blocks=0, d_hidden=128)
    man["resnetfc"] = sd_shapes(head)
    net = build_net(ref, torch.zeros(1, 256, 4, 8))
    man["btsnet"] = sd_shapes(net, drop=("encoder.",))
    man["nerf_renderer"] = sd_shapes(ref.NeRFRenderer(n_coarse=32, lindisp=True))
    spec = importlib.util.spec_from_file_location(
        "ref_dpt_head", os.path.join(REF, "scenedino/models/backbones/dino/dpt_head.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    for embed, name in ((384, "dpt_head_vits"), (768, "dpt_head_vitb")):
        dpt = mod.DPTHead(embed_dims=embed, post_process_channels=[64, 64, 128, 256],
                          readout_type="ignore", patch_size=16, d_out=256, expand_channels=False)
        man[name] = sd_shapes(dpt)
    MlpDimReduction, sh = load_reference_seg()
    man["mlp_dim_reduction"] = sd_shapes(MlpDimReduction(768, 64, latent_channels=128))
    zeros, tensor_to = torch.zeros, torch.Tensor.to
    torch.zeros = lambda *a, **kw: zeros(*a, **{k: v for k, v in kw.items() if k != "device"})
    torch.Tensor.to = lambda self, *a, **kw: self if a and a[0] == "cuda" else tensor_to(self, *a, **kw)
    try:
        for mlp, name in ((False, "semantic_head"), (True, "semantic_head_mlp")):
            head = sh.SemanticHead(19, 19, 768, 64, buffer_size=2, patch_sample_size=4,
                                   knn_neighbors=4, mode="3d", mlp_head=mlp, apply_crf=False)
            man[name] = sd_shapes(head)
    finally:
        torch.zeros, torch.Tensor.to = zeros, tensor_to
    with open(os.path.join(HERE, "state_dict_manifest.json"), "w") as f:
        json.dump(man, f, indent=0, sort_keys=True)


def _reconstruct_input(n=2, v=1, H=8, W=16, K=5, vr=1, ch=3, D=6, ps=4, upscaled=False):
    """A render dict shaped as the renderer returns it (SB = n super-batches of v*H*W rays),
    values = arange (views keep them), with every key ImageRaySampler.reconstruct handles."""
    R = v * H * W
    t = lambda *s: torch.arange(int(np.prod(s)), dtype=torch.float32).view(*s)
    part = {"rgb": t(n, R, vr * ch), "weights": t(n, R, K), "depth": t(n, R),
            "invalid": t(n, R, K, vr), "invalid_features": t(n, R, K, vr), "alphas": t(n, R, K),
            "z_samps": t(n, R, K), "rgb_samps": t(n, R, K, vr * ch), "ray_info": t(n, R, 3),
            "extras": t(n, R, 2), "dino_features": t(n, R, D)}
    gh = H if upscaled else H // ps
    gw = W if upscaled else W // ps
    return {"coarse": part, "rgb_gt": t(n, R, ch), "dino_gt": t(n, v * gh * gw, D),
            "dino_artifacts": t(n, v * gh * gw, D)}


def fx_reconstruct(ref):
    """ImageRaySampler.reconstruct (ray_sampler.py:515-607) output shapes, including the
    dino_gt / dino_artifacts patch-grid branch (:587-605), for patch and upscaled targets."""
    out = {}
    for upscaled in (False, True):
        s = ref.ImageRaySampler(z_near=3, z_far=80, height=8, width=16, channels=3,
                                dino_upscaled=upscaled)
        d = s.reconstruct(_reconstruct_input(upscaled=upscaled))
        shapes = {k: list(v.shape) for k, v in d.items() if torch.is_tensor(v)}
        shapes.update({"coarse." + k: list(v.shape) for k, v in d["coarse"].items()})
        out["upscaled" if upscaled else "patch"] = shapes
    with open(os.path.join(HERE, "reconstruct_shapes.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)


def main():
    torch.set_num_threads(8)
    if os.environ.get("GOLDEN_ONLY") == "dpt":
        fx_dpt()
        print("dpt fixture written to", HERE)
        return
    if os.environ.get("GOLDEN_ONLY") == "salience":
        fx_salience_downsampler()
        print("salience downsampler fixture written to", HERE)
        return
    if os.environ.get("GOLDEN_ONLY") == "ssc":
        fx_ssc_scoring()
        print("ssc scoring fixture written to", HERE)
        return
    if os.environ.get("GOLDEN_ONLY") == "visualization":
        fx_visualization()
        print("visualization fixture written to", HERE)
        return
    if os.environ.get("GOLDEN_ONLY") == "seg":
        _install_stubs()
        fx_seg_head()
        fx_voxel_points()
        print("seg / voxel fixtures written to", HERE)
        return
    ref = load_reference()
    if os.environ.get("GOLDEN_ONLY") == "patch":
        fx_patch_sampler(ref)
        print("patch sampler fixture written to", HERE)
        return
    if os.environ.get("GOLDEN_ONLY") == "empty":
        fx_field_query(ref, learn_empty=True)
        fx_render(ref, "sb2_k32_empty", n=2, nv_render=1, K=32, hard_cap=False, H=16, W=48,
                  seed=61, learn_empty=True, render_offset=(12.0, 1.5))
        print("learn_empty fixtures written to", HERE)
        return
    if os.environ.get("GOLDEN_ONLY") == "full_offset":
        fx_render_full_offset(ref)
        print("full offset-pose fixture written to", HERE)
        return
    if os.environ.get("GOLDEN_ONLY") == "configs03":
        fx_render_full_offset_k32(ref)
        fx_render_c4_offset(ref)
        print("configs[0] / configs[3] full-frame fixtures written to", HERE)
        return
    if os.environ.get("GOLDEN_ONLY") == "reconstruct":
        fx_reconstruct(ref)
        print("reconstruct fixture written to", HERE)
        return
    if os.environ.get("GOLDEN_ONLY") == "manifest":
        fx_state_dict_manifest(ref)
        print("state_dict manifest written to", HERE)
        return
    fx_gen_rays(ref)
    fx_sample_z(ref)
    fx_field_query(ref)
    fx_render(ref, "k32_cap0", n=1, nv_render=1, K=32, hard_cap=False)
    fx_render(ref, "k64_cap1", n=1, nv_render=1, K=64, hard_cap=True, H=16, W=48, seed=41)
    fx_render(ref, "sb2_nv2_k16", n=2, nv_render=2, K=16, hard_cap=False, H=16, W=48, seed=51)
    if os.environ.get("GOLDEN_FULL", "1") == "1":
        fx_render_full_digest(ref)
        fx_render_full_offset(ref)
        fx_render_full_offset_k32(ref)
        fx_render_c4_offset(ref)
    fx_state_dict_manifest(ref)
    fx_reconstruct(ref)
    fx_field_query(ref, learn_empty=True)
    fx_render(ref, "sb2_k32_empty", n=2, nv_render=1, K=32, hard_cap=False, H=16, W=48,
              seed=61, learn_empty=True, render_offset=(12.0, 1.5))
    fx_ssc_scoring()
    fx_patch_sampler(ref)
    fx_salience_downsampler()
    fx_visualization()
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
