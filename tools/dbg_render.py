"""Diagnostic: per-output errors of the 16-bit render against a golden fixture."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch
from _helpers import load, net_from_fixture, rel_l2
from scenedino_amd.renderer import NeRFRenderer
fx = sys.argv[1] if len(sys.argv) > 1 else "render_k32_cap0.npz"
prec = sys.argv[2] if len(sys.argv) > 2 else "bf16"
d = load(fx)
net = net_from_fixture(d, prec, mode="proj")
K = int(d["K"])
r = NeRFRenderer(n_coarse=K, lindisp=True, hard_alpha_cap=bool(d["hard_cap"]), eval_batch_size=65536)
w = r.bind_parallel(net, gpus=None).eval()
r.z_jitter = torch.as_tensor(d["u"]).cuda()
with torch.no_grad():
    c = w(torch.as_tensor(d["rays"]).cuda(), want_weights=True, want_alphas=True, want_z_samps=True, want_rgb_samps=True)["coarse"]
for k in ("depth", "weights", "alphas", "rgb", "dino_features", "rgb_samps"):
    print(fx, prec, k, "rel-L2 %.3g" % rel_l2(c[k], d[k]), "max %.3g" % float((c[k].cpu() - torch.as_tensor(d[k])).abs().max()))
