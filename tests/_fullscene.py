"""Rebuild the scenes of the full-size golden renders (tests/golden/make_golden.py
fx_render_full_digest / fx_render_full_offset) on the build's API."""
import torch

KITTI_K = [[0.7849, 0.0, -0.0312], [0.0, 2.9391, 0.2701], [0.0, 0.0, 1.0]]


def full_scene(seed, gh, gw, precision, dev, H=192, W=640, C=256):
    """make_golden.make_scene(1, 1, C, gh, gw, H, W, seed) + build_net(ref, grid) (kaiming
    ResnetFC at seed 2, biases 0.1 N(0, 1) at seed 102) on the build's BTSNet, encoded at the
    identity pose.  Returns (net, Kn (1, 1, 3, 3) on dev)."""
    from _helpers import build_net
    from scenedino_amd.models.prediction_heads import ResnetFC
    g = torch.Generator().manual_seed(seed)
    images = torch.rand(1, 1, 3, H, W, generator=g) * 2 - 1
    grid = torch.randn(1, C, gh, gw, generator=g)
    torch.manual_seed(2)
    head = ResnetFC(d_in=C + 39, d_out=65, n_blocks=0, d_hidden=128)
    gb = torch.Generator().manual_seed(102)
    with torch.no_grad():
        head.lin_in.bias.copy_(0.1 * torch.randn(128, generator=gb))
        head.lin_out.bias.copy_(0.1 * torch.randn(65, generator=gb))
    net = build_net(grid, head.lin_in.weight, head.lin_in.bias, head.lin_out.weight,
                    head.lin_out.bias, precision, dev)
    Kn = torch.tensor(KITTI_K).view(1, 1, 3, 3).to(dev)
    poses = torch.eye(4).view(1, 1, 4, 4).to(dev)
    net.encode(images.to(dev), Kn, poses, ids_encoder=[0], ids_render=[0])
    return net, Kn


def render_full_offset(d, precision, dev="cuda", nets=None, K=64):
    """The golden's 192x640x64 offset-pose render on the build (jitter injected).  nets: a
    list the BTSNet is appended to (tests that read its render scratch); K != 64: the same
    scene at K samples per ray (no golden: self-consistency tests)."""
    from scenedino_amd.renderer import NeRFRenderer
    from scenedino_amd.common.ray_sampler import ImageRaySampler
    net, Kn = full_scene(int(d["scene_seed"]), 192, 640, precision, dev)
    if nets is not None:
        nets.append(net)
    pose = torch.as_tensor(d["render_pose"]).to(dev)
    rays, _ = ImageRaySampler(3, 80, 192, 640).sample(None, pose, Kn)
    u = torch.rand(rays.shape[1], K, generator=torch.Generator().manual_seed(int(d["u_seed"])))
    r = NeRFRenderer(n_coarse=K, lindisp=True, hard_alpha_cap=False, eval_batch_size=65536)
    r.z_jitter = u.to(dev)
    with torch.no_grad():
        return r.bind_parallel(net).eval()(rays, want_weights=True, want_alphas=True)["coarse"]


def scene_arrays(seed, gh=192, gw=640, H=192, W=640, C=256, D=64, weights=None):
    """The CPU arrays of make_golden.make_scene(1, 1, C, gh, gw, H, W, seed) + its head:
    (images (1, 1, 3, H, W), grid (1, C, gh, gw), (W_in, b_in, W_out, b_out)).  weights: a
    fixture holding W_in / b_in / W_out / b_out (d_out != 65 changes the kaiming draw), else
    build_net's seeded head."""
    from scenedino_amd.models.prediction_heads import ResnetFC
    g = torch.Generator().manual_seed(seed)
    images = torch.rand(1, 1, 3, H, W, generator=g) * 2 - 1
    grid = torch.randn(1, C, gh, gw, generator=g)
    if weights is not None:
        T = lambda k: torch.as_tensor(weights[k])
        return images, grid, (T("W_in"), T("b_in"), T("W_out"), T("b_out"))
    torch.manual_seed(2)
    head = ResnetFC(d_in=C + 39, d_out=1 + D, n_blocks=0, d_hidden=128)
    gb = torch.Generator().manual_seed(102)
    with torch.no_grad():
        head.lin_in.bias.copy_(0.1 * torch.randn(128, generator=gb))
        head.lin_out.bias.copy_(0.1 * torch.randn(1 + D, generator=gb))
    return images, grid, tuple(t.detach() for t in (head.lin_in.weight, head.lin_in.bias,
                                                    head.lin_out.weight, head.lin_out.bias))


def render_offset_fixture(d, precision, dev="cuda", whole_frame=True):
    """make_golden.fx_render_full_offset_k32 / fx_render_c4_offset on the build: the seed-61
    scene (head from the fixture if it holds one), rays of the fixture's render pose, the
    fixture's jitter rows (seed u_seed over all 122 880 rays x K).  whole_frame: render every
    ray of the frame (the tile kernel's full-frame grouping); else only the fixture's rays."""
    from _helpers import build_net
    from scenedino_amd.renderer import NeRFRenderer
    from scenedino_amd.common.ray_sampler import ImageRaySampler
    K = int(d["K"])
    D = int(d["D"]) if "D" in d else 64
    images, grid, (W_in, b_in, W_out, b_out) = scene_arrays(
        int(d["scene_seed"]), D=D, weights=d if "W_in" in d else None)
    net = build_net(grid, W_in, b_in, W_out, b_out, precision, dev)
    Kn = torch.tensor(KITTI_K).view(1, 1, 3, 3).to(dev)
    net.encode(images.to(dev), Kn, torch.eye(4).view(1, 1, 4, 4).to(dev), ids_encoder=[0],
               ids_render=[0])
    pose = torch.as_tensor(d["render_pose"]).to(dev)
    rays, _ = ImageRaySampler(3, 80, 192, 640).sample(None, pose, Kn)
    u = torch.rand(rays.shape[1], K, generator=torch.Generator().manual_seed(int(d["u_seed"])))
    if not whole_frame:
        it = torch.from_numpy(d["idx"])
        rays, u = rays[:, it.to(dev)], u[it]
    r = NeRFRenderer(n_coarse=K, lindisp=True, hard_alpha_cap=False, eval_batch_size=65536)
    r.z_jitter = u.to(dev)
    with torch.no_grad():
        return r.bind_parallel(net).eval()(rays, want_weights=True, want_alphas=True)["coarse"]
