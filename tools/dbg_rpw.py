"""Diagnostic: per-ray-slot DINO / depth error of the tile kernel on the K = 32 fixture
(which of a 16-ray group's slots are off)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import torch
from _helpers import load, net_from_fixture
from scenedino_amd.renderer import NeRFRenderer

d = load("render_k32_cap0.npz")
for prec in ("fp16", "bf16"):
    net = net_from_fixture(d, prec, mode="proj")
    K = int(d["K"])
    r = NeRFRenderer(n_coarse=K, lindisp=True, hard_alpha_cap=bool(d["hard_cap"]))
    w = r.bind_parallel(net).eval()
    r.z_jitter = torch.as_tensor(d["u"]).cuda()
    with torch.no_grad():
        c = w(torch.as_tensor(d["rays"]).cuda(), want_weights=True)["coarse"]
    for k in ("dino_features", "depth", "rgb"):
        a = c[k].double().cpu().reshape(c[k].shape[1], -1)
        b = torch.as_tensor(d[k]).double().reshape(a.shape)
        e = (a - b).norm(dim=1) / b.norm(dim=1).clamp_min(1e-9)
        slots = [float(e[s::16].mean()) for s in range(16)]
        print(prec, k, "per-slot mean rel err:", " ".join(f"{v:.1e}" for v in slots))
