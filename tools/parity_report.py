"""Diagnostic: per-output error statistics of every render mode against the golden
fixtures (max |d|, max |d| / (|ref| + 1e-6), rel-L2) -- the numbers the tolerances in
tests/test_gpu_parity.py are set from."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import torch
from _helpers import load, net_from_fixture, rel_l2
from scenedino_amd.renderer import NeRFRenderer

for fx in ["render_k32_cap0.npz", "render_k64_cap1.npz", "render_sb2_nv2_k16.npz"]:
    d = load(fx)
    for prec, mode in (("fp32", "grid"), ("bf16", "proj"), ("fp16", "proj"), ("bf16", "grid")):
        net = net_from_fixture(d, prec, mode=mode)
        K = int(d["K"])
        r = NeRFRenderer(n_coarse=K, lindisp=True, hard_alpha_cap=bool(d["hard_cap"]), eval_batch_size=65536)
        w = r.bind_parallel(net, gpus=None).eval()
        r.z_jitter = torch.as_tensor(d["u"]).cuda()
        with torch.no_grad():
            c = w(torch.as_tensor(d["rays"]).cuda(), want_weights=True, want_alphas=True,
                  want_z_samps=True, want_rgb_samps=True)["coarse"]
        row = []
        for k, rk in (("depth", "depth"), ("weights", "weights"), ("alphas", "alphas"), ("rgb", "rgb"),
                      ("dino_features", "dino_features"), ("rgb_samps", "rgb_samps")):
            a = c[k].double().cpu().reshape(-1); b = torch.as_tensor(d[rk]).double().reshape(-1)
            e = (a - b).abs()
            need = float((e - 1e-5 * b.abs()).max())
            row.append(f"{k}: max {e.max():.2e} rel {(e / (b.abs() + 1e-6)).max():.1e} l2 {rel_l2(a, b):.1e} atol@rtol1e-5 {need:.1e}")
        masks = all(torch.equal(c[m].cpu(), torch.from_numpy(d[m])) for m in ("invalid", "invalid_features"))
        print(fx, prec, mode, "masks", masks)
        for x in row:
            print("    ", x)

import hashlib
from _fullscene import render_full_offset
d = load("render_full_offset.npz")
idx = torch.from_numpy(d["idx"])
for prec in ("fp32", "bf16", "fp16"):
    c = render_full_offset(d, prec)
    print("full_offset", prec, "masks",
          hashlib.sha256(c["invalid"].cpu().numpy().tobytes()).hexdigest() == str(d["invalid_sha256"]),
          hashlib.sha256(c["invalid_features"].cpu().numpy().tobytes()).hexdigest() == str(d["invalid_features_sha256"]))
    for k, rk in (("depth", "depth"), ("weights", "weights"), ("alphas", "alphas"), ("rgb", "rgb"), ("dino_features", "dino")):
        a = c[k][0].double().cpu()[idx].reshape(-1); b = torch.as_tensor(d[rk]).double().reshape(-1)
        e = (a - b).abs()
        need = float((e - 1e-5 * b.abs()).max())
        print("    ", f"{k}: max {e.max():.2e} l2 {rel_l2(a, b):.1e} atol@rtol1e-5 {need:.1e}")
    print("     depth mean diff", abs(float(c["depth"].double().mean()) - float(d["depth_mean"])))
