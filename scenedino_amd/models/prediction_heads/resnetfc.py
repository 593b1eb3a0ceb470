"""ResnetFC -- parameter container with the reference's module/parameter names.

Mirror of scenedino.models.prediction_heads.resnetfc.ResnetFC
(/root/reference/scenedino/models/prediction_heads/resnetfc.py:66-237).  Shipped
configs use n_blocks=0 (configs/model/dino_downsampler.yaml:35-41):
``out = lin_out(relu(lin_in(x)))``.  In this package the MLP is evaluated by the
fused gfx950 kernels (BTSNet); ``forward`` here is the plain tensor-op form kept for
API completeness (used by nothing on the hot path).
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import nn


class ResnetBlockFC(nn.Module):
    def __init__(self, size_in, size_out=None, size_h=None, beta=0.0):
        super().__init__()
        size_out = size_in if size_out is None else size_out
        size_h = min(size_in, size_out) if size_h is None else size_h
        self.size_in, self.size_h, self.size_out = size_in, size_h, size_out
        self.fc_0 = nn.Linear(size_in, size_h)
        self.fc_1 = nn.Linear(size_h, size_out)
        nn.init.constant_(self.fc_0.bias, 0.0)
        nn.init.kaiming_normal_(self.fc_0.weight, a=0, mode="fan_in")
        nn.init.constant_(self.fc_1.bias, 0.0)
        nn.init.zeros_(self.fc_1.weight)
        self.activation = nn.Softplus(beta=beta) if beta > 0 else nn.ReLU()
        self.shortcut = None if size_in == size_out else nn.Linear(size_in, size_out, bias=False)

    def forward(self, x):
        net = self.fc_0(self.activation(x))
        dx = self.fc_1(self.activation(net))
        return (x if self.shortcut is None else self.shortcut(x)) + dx


class ResnetFC(nn.Module):
    def __init__(self, d_in, view_number: Optional[int] = None, d_out=4, n_blocks=5, d_latent=0,
                 d_hidden=128, beta=0.0, combine_layer=1000, combine_type="average",
                 use_spade=False):
        super().__init__()
        if d_in > 0:
            self.lin_in = nn.Linear(d_in, d_hidden)
            nn.init.constant_(self.lin_in.bias, 0.0)
            nn.init.kaiming_normal_(self.lin_in.weight, a=0, mode="fan_in")
        self.lin_out = nn.Linear(d_hidden, d_out)
        nn.init.constant_(self.lin_out.bias, 0.0)
        nn.init.kaiming_normal_(self.lin_out.weight, a=0, mode="fan_in")
        self.n_blocks, self.d_latent, self.d_in = n_blocks, d_latent, d_in
        self.view_number, self.d_out, self.d_hidden = view_number, d_out, d_hidden
        self.combine_layer, self.combine_type, self.use_spade = combine_layer, combine_type, use_spade
        self.blocks = nn.ModuleList([ResnetBlockFC(d_hidden, beta=beta) for _ in range(n_blocks)])
        if d_latent != 0:
            n_lin_z = min(combine_layer, n_blocks)
            self.lin_z = nn.ModuleList([nn.Linear(d_latent, d_hidden) for _ in range(n_lin_z)])
            if use_spade:
                self.scale_z = nn.ModuleList([nn.Linear(d_latent, d_hidden) for _ in range(n_lin_z)])
        self.activation = nn.Softplus(beta=beta) if beta > 0 else nn.ReLU()

    def forward(self, sampled_features, combine_inner_dims=(1,), combine_index=None,
                dim_size=None, **kwargs):
        if self.n_blocks or self.d_latent:
            raise NotImplementedError("only n_blocks=0, d_latent=0 (shipped configs)")
        zx = sampled_features if self.view_number is None else sampled_features[..., self.view_number, :]
        return self.lin_out(self.activation(self.lin_in(zx)))

    @classmethod
    def from_conf(cls, conf, d_in, d_out, d_latent=0):
        return cls(d_in=d_in, d_out=d_out, **conf)
