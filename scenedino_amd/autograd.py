"""Differentiable (training) field path: autograd Functions over the sdhip_train.hip kernels.

The inference path (sd_render_proj / sd_render_fused) fuses everything into one kernel and
keeps no per-sample state; training (``train.py`` renders through the field and
back-propagates into the feature grid and the ResnetFC, base_trainer.py:223,251) runs

  FieldGather  (sd_field_gather / sd_field_gather_bwd)   a8-a10, a12, a15  -> X = [feat | code]
  ResnetFC     torch.nn.Linear (library GEMMs, autograd)  a13
  softplus     torch                                       a14
  Composite    (sd_composite / sd_composite_bwd)           a16

so that ``loss.backward()`` reaches ``grid_f_features`` (and through it whatever encoder
produced the grid) and the head parameters, as in the reference's
``BTSNet.forward`` -> ``NeRFRenderer.composite`` (bts.py:476-595, nerf.py:343-405).
No CPU fallback: every op here is a HIP kernel or a torch GPU op.
"""
from __future__ import annotations

import torch

from . import _lib


class FieldGather(torch.autograd.Function):
    """X = [grid_sample(grid, project(xyz)) | positional_code(xyz)], differentiable in the
    grid (bts.py:271-328).  grid_nhwc (B, Hf, Wf, C) f32; xyz (B, P, 3) (no gradient: the
    reference's sample points come from rays and depths without grad)."""

    @staticmethod
    def forward(ctx, grid_nhwc, xyz, cam_f, img, cam_c, colors):
        x, invf, rgb, inv = _lib.field_gather(xyz, grid_nhwc, cam_f, img, cam_c, colors)
        ctx.save_for_backward(xyz, cam_f)
        ctx.grid_shape = tuple(grid_nhwc.shape)
        outs = [t for t in (invf, rgb, inv) if t is not None]
        ctx.mark_non_differentiable(*outs)
        return x, invf, rgb, inv

    @staticmethod
    def backward(ctx, gx, *_):
        xyz, cam_f = ctx.saved_tensors
        dgrid = None
        if ctx.needs_input_grad[0] and gx is not None:
            _, Hf, Wf, C = ctx.grid_shape
            dgrid = _lib.field_gather_bwd(xyz, gx, cam_f, Hf, Wf, C)
        return dgrid, None, None, None, None, None


class Composite(torch.autograd.Function):
    """Alpha compositing (nerf.py:376-405) with the sd_composite_bwd backward.
    z, sigma (R, K); feat (R, K, F) | None; rgb (R, K, Cc) | None.  Returns
    (weights, alphas, depth, feat_out, rgb_out).  z carries no gradient (the reference's
    depths are sampled without grad)."""

    @staticmethod
    def forward(ctx, z, sigma, feat, rgb, hard_alpha_cap):
        z = z.float().contiguous()
        sigma = sigma.float().contiguous()
        feat = feat.float().contiguous() if feat is not None else None
        rgb = rgb.float().contiguous() if rgb is not None else None
        w, a, d, fo, ro = _lib.composite(z, sigma, feat, rgb, hard_alpha_cap)
        ctx.save_for_backward(z, sigma, feat, rgb)
        ctx.hard = bool(hard_alpha_cap)
        return w, a, d, fo, ro

    @staticmethod
    def backward(ctx, g_w, g_a, g_d, g_f, g_r):
        z, sigma, feat, rgb = ctx.saved_tensors
        d_sigma, d_feat, d_rgb = _lib.composite_bwd(
            z, sigma, feat, rgb, ctx.hard, g_d, g_f, g_r, g_w, g_a,
            need_feat=ctx.needs_input_grad[2], need_rgb=ctx.needs_input_grad[3])
        return (None, d_sigma if ctx.needs_input_grad[1] else None, d_feat, d_rgb, None)


def composite(z, sigma, feat, rgb, hard_alpha_cap):
    """Differentiable when any input requires grad and grad mode is on; otherwise the plain
    sd_composite launch (no saved state)."""
    if torch.is_grad_enabled() and any(t is not None and t.requires_grad
                                       for t in (sigma, feat, rgb)):
        return Composite.apply(z, sigma, feat, rgb, hard_alpha_cap)
    return _lib.composite(z.float().contiguous(), sigma.float().contiguous(),
                          feat.float().contiguous() if feat is not None else None,
                          rgb.float().contiguous() if rgb is not None else None, hard_alpha_cap)
