"""Loss-side feature downsamplers (mirror of scenedino/models/backbones/dino/downsampler.py).

``PatchSalienceDownsampler`` (the ``featup`` downsampler, :31-98) keeps the reference's
parameters (``conv``, ``patch_weight``, ``patch_bias``: same checkpoint keys and init) and
runs ``forward_patches`` as the sd_salience_fwd / sd_salience_bwd kernels
(csrc/sdhip_down.hip, autograd in scenedino_amd.autograd.SalienceDownsample).
``BilinearDownsampler`` (:6-28) is one ``F.interpolate`` call, kept as the torch op.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


class BilinearDownsampler(torch.nn.Module):
    """downsampler.py:6-28."""

    def __init__(self, patch_size):
        super().__init__()
        if isinstance(patch_size, int):
            self.patch_size = (patch_size, patch_size)
        elif isinstance(patch_size, tuple):
            self.patch_size = patch_size

    def forward(self, x, mode):
        n, v, h, w, _, c = x.shape
        assert h % self.patch_size[0] == 0
        assert w % self.patch_size[1] == 0
        th, tw = h // self.patch_size[0], w // self.patch_size[1]
        x = x.permute(0, 1, 4, 5, 2, 3).flatten(0, 2)
        x = F.interpolate(x, size=(th, tw), mode="bilinear")
        x = x.reshape(n, v, -1, c, th, tw).permute(0, 1, 4, 5, 2, 3)
        return x.squeeze(2, 3)


class PatchSalienceDownsampler(torch.nn.Module):
    """downsampler.py:31-98."""

    def __init__(self, channels, patch_size, normalize_features):
        super().__init__()
        if isinstance(patch_size, int):
            self.patch_size = (patch_size, patch_size)
        elif isinstance(patch_size, tuple):
            self.patch_size = patch_size
        self.conv = torch.nn.Conv2d(channels, 1, kernel_size=1)
        self.patch_weight = torch.nn.Parameter(torch.ones(self.patch_size))
        self.patch_bias = torch.nn.Parameter(torch.zeros(self.patch_size))
        self.normalize_features = normalize_features
        torch.nn.init.kaiming_normal_(self.conv.weight, a=0, mode="fan_in")
        torch.nn.init.zeros_(self.conv.bias)
        torch.nn.init.normal_(self.patch_weight, mean=1.0, std=0.01)
        torch.nn.init.normal_(self.patch_bias, mean=0.0, std=0.01)

    def forward(self, x, mode):
        if mode == "patch":
            return self.forward_patches(x)
        if mode == "image":  # :62-79
            n, v, h, w, _, c = x.shape
            ph, pw = self.patch_size
            nh, nw = h // ph, w // pw
            patches = x.reshape(n, v, nh, ph, nw, pw, 1, c).swapaxes(3, 4).flatten(1, 3)
            res, sal, wmap, pwb = self.forward_patches(patches)
            res = res.reshape(n, v, nh, nw, 1, c)
            sal = sal.reshape(n, v, nh, nw, ph, pw, 1, 1).swapaxes(3, 4).reshape(n, v, h, w, 1, 1)
            wmap = wmap.reshape(n, v, nh, nw, ph, pw, 1, 1).swapaxes(3, 4).reshape(n, v, h, w, 1, 1)
            return res, sal, wmap, pwb
        return None

    def forward_patches(self, x):
        """:82-98: x (n, p, ph, pw, 1, c) -> (features (n, p, 1, c), salience (n, p, ph, pw,
        1, 1), weights (n, p, ph, pw, 1, 1), cat(patch_weight, patch_bias))."""
        from ....autograd import SalienceDownsample
        n, p, ph, pw, _, c = x.shape
        if x.device.type != "cuda":
            raise RuntimeError("PatchSalienceDownsampler: the salience kernels need CUDA (HIP) "
                               "tensors")
        out, sal, wmap = SalienceDownsample.apply(
            x.reshape(n * p, ph * pw, c), self.conv.weight, self.conv.bias, self.patch_weight,
            self.patch_bias, self.normalize_features)
        return (out.to(x.dtype).reshape(n, p, 1, c), sal.reshape(n, p, ph, pw, 1, 1),
                wmap.reshape(n, p, ph, pw, 1, 1),
                torch.cat([self.patch_weight, self.patch_bias], dim=1))
