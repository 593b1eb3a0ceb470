"""Shared test helpers: load golden fixtures, build the scenedino_amd model on them."""
from __future__ import annotations

import os

import numpy as np
import torch

from conftest import GOLDEN


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


class FixedGridEncoder(torch.nn.Module):
    """Stand-in for the DINO/DINOv2 encoder: returns a fixed feature grid (the encoder
    is its own scope row); exposes the attributes BTSNet reads."""

    def __init__(self, grid):
        super().__init__()
        self.register_buffer("grid", grid)
        self.latent_size = grid.shape[1]
        self.extra_outs = 0

    def forward(self, x, ground_truth=False):
        return [self.grid]


MODEL_CONF = {"predict_dino": True, "dino_dims": 64, "learn_empty": False, "code_mode": "z",
              "inv_z": True, "z_near": 3, "z_far": 80, "sample_color": True}


def build_net(grid, W_in, b_in, W_out, b_out, precision="fp32", device="cuda", mode="proj",
              empty_feature=None):
    from scenedino_amd.models import BTSNet
    from scenedino_amd.models.prediction_heads import ResnetFC
    from scenedino_amd.common.positional_encoding import PositionalEncoding

    grid = torch.as_tensor(grid)
    code = PositionalEncoding(6, 3, 1.5, True)
    enc = FixedGridEncoder(grid)
    D = W_out.shape[0] - 1
    head = ResnetFC(d_in=grid.shape[1] + 39, d_out=1 + D, n_blocks=0, d_hidden=128)
    with torch.no_grad():
        head.lin_in.weight.copy_(torch.as_tensor(W_in))
        head.lin_in.bias.copy_(torch.as_tensor(b_in))
        head.lin_out.weight.copy_(torch.as_tensor(W_out))
        head.lin_out.bias.copy_(torch.as_tensor(b_out))
    conf = dict(MODEL_CONF, dino_dims=D, precision=precision, fused_mode=mode,
                learn_empty=empty_feature is not None)
    net = BTSNet(conf, enc, code, {"normal_head": head}, final_pred_head="normal_head")
    if empty_feature is not None:
        with torch.no_grad():
            net.empty_feature.copy_(torch.as_tensor(np.asarray(empty_feature)))
    return net.to(device).eval()


def net_from_fixture(d, precision="fp32", device="cuda", mode="proj"):
    net = build_net(d["grid"], d["W_in"], d["b_in"], d["W_out"], d["b_out"], precision, device,
                    mode, empty_feature=d["empty_feature"] if "empty_feature" in d else None)
    nv = int(d["nv_render"]) if "nv_render" in d else 1
    T = lambda k: torch.as_tensor(d[k]).to(device)
    net.encode(T("images"), T("Ks"), T("poses"), ids_encoder=[0], ids_render=list(range(nv)))
    return net


def rel_l2(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))
