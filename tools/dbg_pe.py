"""Diagnostic: 16-bit render vs the CPU oracle with the code columns of W_in masked."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch
from _helpers import build_net, rel_l2
from oracle import render_oracle as O
from scenedino_amd.renderer import NeRFRenderer
from scenedino_amd.common.ray_sampler import ImageRaySampler
dev = "cuda:0"
g = torch.Generator().manual_seed(0)
H, W, K, C = 16, 48, 32, 256
images = torch.rand(1, 1, 3, H, W, generator=g) * 2 - 1
grid = torch.randn(1, C, 8, 24, generator=g)
W_in0 = torch.randn(128, C + 39, generator=g) * 0.08
b_in = torch.randn(128, generator=g) * 0.1
W_out = torch.randn(65, 128, generator=g) * 0.1
b_out = torch.randn(65, generator=g) * 0.1
Kn = torch.tensor([[0.7849, 0.0, -0.0312], [0.0, 2.9391, 0.2701], [0.0, 0.0, 1.0]]).view(1, 1, 3, 3)
pose = torch.eye(4).view(1, 1, 4, 4)
u = torch.rand(H * W, K, generator=g)
MODES = sys.argv[1].split(",") if len(sys.argv) > 1 else None
for name, cols in (("all", list(range(39))), ("none", []), ("raw", [0, 1, 2]), ("f0", [3, 4, 5, 6, 7, 8]),
                   ("f4", [27, 28, 29, 30, 31, 32]), ("x-only", [3, 6, 9, 12, 15, 18, 21, 24, 27, 30, 33, 36])):
    if MODES and name not in MODES:
        continue
    W_in = W_in0.clone()
    mask = torch.zeros(39, dtype=torch.bool); mask[cols] = True
    W_in[:, C:][:, ~mask] = 0
    net = build_net(grid, W_in, b_in, W_out, b_out, "bf16", dev)
    net.encode(images.to(dev), Kn.to(dev), pose.to(dev), ids_encoder=[0], ids_render=[0])
    rays, _ = ImageRaySampler(3, 80, H, W).sample(None, pose.to(dev), Kn.to(dev))
    r = NeRFRenderer(n_coarse=K, lindisp=True)
    r.z_jitter = u.to(dev)
    with torch.no_grad():
        c = r.bind_parallel(net).eval()(rays, want_weights=True)["coarse"]
    w2c = torch.inverse(pose)
    ref = O.render(rays[0].cpu(), u, grid, w2c[:, 0], Kn[:, 0], images * 0.5 + 0.5, w2c, Kn, W_in, b_in, W_out, b_out, sb=1)
    print(name, " ".join(f"{k} {rel_l2(c[k], ref[k]):.3g}" for k in ("depth", "weights", "dino_features")))
