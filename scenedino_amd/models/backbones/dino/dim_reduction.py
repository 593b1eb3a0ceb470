"""DINO feature dimension reduction, MI355X build.

Mirror of scenedino/models/backbones/dino/dim_reduction.py:6-25 (same class names,
constructor arguments and parameter names ``linear_in`` / ``linear_out``, so the
reference's ``encoder.dim_reduction.*`` checkpoint keys load unchanged).
``MlpDimReduction.transform_expand`` (64 -> 128 ReLU -> d_full, L2-normalised) runs in
the gfx950 kernel ``sd_seg_query`` (expand-only record, csrc/sdhip_seg.hip).
"""
from __future__ import annotations

import torch
from torch import nn

from .... import _lib  # noqa: F401  (fail loudly on a box without the HIP library)


class NoDimReduction(nn.Module):
    """dim_reduction.py:6-12: identity (full == reduced)."""

    def __init__(self, full_channels, reduced_channels):
        super().__init__()
        if full_channels != reduced_channels:
            raise ValueError("NoDimReduction needs full_channels == reduced_channels")

    def forward(self, features):
        return features

    def transform_expand(self, features):
        return features


class MlpDimReduction(nn.Module):
    """dim_reduction.py:15-25."""

    def __init__(self, full_channels, reduced_channels, latent_channels):
        super().__init__()
        self.linear_in = nn.Linear(reduced_channels, latent_channels)
        self.linear_out = nn.Linear(latent_channels, full_channels)
        self.relu = nn.ReLU()
        self._packed = None

    def _rec(self):
        from ....seg_pack import PackedSegHead, seg_key
        key = seg_key(self)
        if self._packed is None or self._packed[0] != key:
            self._packed = (key, PackedSegHead(self))
        return self._packed[1]

    def transform_expand(self, features: torch.Tensor) -> torch.Tensor:
        """features (..., reduced) -> F.normalize(linear_out(relu(linear_in(x))), dim=-1)."""
        if torch.is_grad_enabled() and self.training:
            raise NotImplementedError("scenedino_amd: transform_expand has no backward kernel; "
                                      "use eval() / torch.no_grad()")
        from ....seg_pack import seg_key
        lead = features.shape[:-1]
        x = features.reshape(-1, features.shape[-1]).float().contiguous()
        _, _, full = _lib.seg_query(x, self._rec().rec, want_labels=False, want_full=True)
        out = full.view(*lead, -1)
        # provenance for SemanticHead.forward: the expanded features of these codes, so the
        # 2-D demo's head call on them (demo_utils/utils.py:228-232) runs the folded
        # stego / k-means kernel on the 64-d codes instead of library GEMMs on 768-d rows
        out._sd_expand = (x, self, seg_key(self), out._version)
        return out
