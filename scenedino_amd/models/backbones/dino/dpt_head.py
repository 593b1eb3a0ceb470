"""DPT decoder, MI355X build.

Mirror of scenedino/models/backbones/dino/dpt_head.py:10-236 (``DPTHead``,
``ReassembleBlocks``, ``PreActResidualConvUnit``, ``FeatureFusionBlock``, ``OutputHead``):
same constructor arguments and parameter names (``reassemble_blocks.projects.{i}``,
``reassemble_blocks.resize_layers.{0,1,3}``, ``convs.{i}``,
``fusion_blocks.{i}.{project,res_conv_unit1,res_conv_unit2}.{conv1,conv2}``, ``project``,
``output_head.head_modules.{0,1,2}``), so the ``encoder.decoder.*`` keys of a SceneDINO
checkpoint load unchanged.  The forward pass runs on the gfx950 GEMM kernel of
csrc/sdhip_vit.hip with NHWC bf16 activations:
  * 1x1 convolutions: plain GEMMs over pixels;
  * ConvTranspose2d(k, stride k): one GEMM to k^2 Cout columns whose epilogue scatters
    every column block to its sub-pixel (SD_EPI_SHUF);
  * 3x3 convolutions (stride 1 / 2, padding 1): implicit GEMM, the im2col done by the
    A-tile loader (out-of-image taps read as zeros through the buffer bounds), the
    pre-activation ReLU of the residual units applied as the tile is loaded, the residual
    additions in the epilogue;
  * bilinear x2 (align_corners=True): sd_upsample2x;
  * the last convolution writes the NCHW f32 grid BTSNet samples (SD_EPI_NCHW).
Parity: tests/golden/dpt_head.npz, produced by the reference's own DPTHead on CPU.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F
from torch import nn

from .... import _lib
from .vit import _param_key

# FeatureFusionBlock's 1x1 projection applied before its x2 upsampling (the reference order,
# dpt_head.py:156-157, is upsample then project; exact in real arithmetic, one bf16 rounding
# moved); SCENEDINO_AMD_DPT_PROJECT_FIRST=0 restores the reference order (A/B runs)
PROJECT_FIRST = os.environ.get("SCENEDINO_AMD_DPT_PROJECT_FIRST", "1") != "0"
# levels 0 / 1: the reassemble projection (1x1 conv) folded into the ConvTranspose(k, stride k)
# behind it -- both linear, no padding, so W_t W_p x + (W_t b_p + b_t) is the same map in one
# GEMM (weights multiplied in fp32 on the host, one bf16 rounding of the product instead of
# one of the intermediate activations); SCENEDINO_AMD_DPT_FOLD_UP=0: two GEMMs (A/B runs)
FOLD_UP = os.environ.get("SCENEDINO_AMD_DPT_FOLD_UP", "1") != "0"


class ReassembleBlocks(nn.Module):
    def __init__(self, in_channels=768, out_channels=None, readout_type="ignore", patch_size=16):
        super().__init__()
        out_channels = [96, 192, 384, 384] if out_channels is None else out_channels
        if readout_type != "ignore":
            raise NotImplementedError("readout_type 'ignore' only (dpt_head.py:41)")
        self.readout_type = readout_type
        self.patch_size = patch_size
        self.projects = nn.ModuleList([nn.Conv2d(in_channels, c, kernel_size=1) for c in out_channels])
        self.resize_layers = nn.ModuleList([
            nn.ConvTranspose2d(out_channels[0], out_channels[0], kernel_size=4, stride=4, padding=0),
            nn.ConvTranspose2d(out_channels[1], out_channels[1], kernel_size=2, stride=2, padding=0),
            nn.Identity(),
            nn.Conv2d(out_channels[3], out_channels[3], kernel_size=3, stride=2, padding=1),
        ])


class PreActResidualConvUnit(nn.Module):
    def __init__(self, in_channels, stride=1, dilation=1, bn=False):
        super().__init__()
        if bn or stride != 1 or dilation != 1:
            raise NotImplementedError("PreActResidualConvUnit(bn=False, stride 1, dilation 1) only")
        self.bn = bn
        self.act = nn.ReLU()
        self.conv1 = nn.Conv2d(in_channels, in_channels, 3, stride=stride, padding=dilation,
                               dilation=dilation, bias=True)
        self.conv2 = nn.Conv2d(in_channels, in_channels, 3, padding=1, bias=True)


class FeatureFusionBlock(nn.Module):
    def __init__(self, in_channels, expand=False, align_corners=True):
        super().__init__()
        self.in_channels = in_channels
        self.expand = expand
        self.align_corners = align_corners
        self.out_channels = in_channels // 2 if expand else in_channels
        self.project = nn.Conv2d(self.in_channels, self.out_channels, kernel_size=1)
        self.res_conv_unit1 = PreActResidualConvUnit(in_channels=self.in_channels)
        self.res_conv_unit2 = PreActResidualConvUnit(in_channels=self.in_channels)


class OutputHead(nn.Module):
    def __init__(self, latent_size=768):
        super().__init__()
        self.head_modules = nn.ModuleList([
            nn.Conv2d(latent_size, latent_size, kernel_size=3, stride=1, padding=1),
            nn.ConvTranspose2d(latent_size, latent_size, kernel_size=2, stride=2, padding=0),
            nn.Conv2d(latent_size, latent_size, kernel_size=3, stride=1, padding=1),
        ])


def _pack_conv3(conv):
    w = conv.weight.detach()  # (Cout, Cin, 3, 3) -> (Cout, ky, kx, ci)
    return (w.permute(0, 2, 3, 1).reshape(w.shape[0], -1).to(torch.bfloat16).contiguous(),
            conv.bias.detach().float().contiguous() if conv.bias is not None else None)


def _pack_conv1(conv):
    w = conv.weight.detach()
    return (w.reshape(w.shape[0], -1).to(torch.bfloat16).contiguous(),
            conv.bias.detach().float().contiguous() if conv.bias is not None else None)


def _pack_proj_convT(proj, conv):
    """Conv2d(C, c, 1) followed by ConvTranspose2d(c, c', k, stride k) as one GEMM operand:
    (k k c', C) with column n = (dy k + dx) c' + co (_pack_convT's order), bias per column."""
    wp = proj.weight.detach().double().reshape(proj.weight.shape[0], -1)  # (c, C)
    bp = proj.bias.detach().double()
    w = conv.weight.detach().double()  # (c, c', k, k)
    cin, cout, k, _ = w.shape
    wt = w.permute(2, 3, 1, 0).reshape(k * k * cout, cin)  # (k k c', c)
    bt = conv.bias.detach().double().repeat(k * k)
    return ((wt @ wp).to(torch.bfloat16).contiguous(), (wt @ bp + bt).float().contiguous(), k)


def _pack_convT(conv):
    """ConvTranspose2d(k, stride k): weight (Cin, Cout, k, k) -> (k k Cout, Cin) with column
    n = (dy k + dx) Cout + co; bias repeated per sub-pixel."""
    w = conv.weight.detach()
    cin, cout, k, _ = w.shape
    wp = w.permute(2, 3, 1, 0).reshape(k * k * cout, cin)
    b = conv.bias.detach().float().repeat(k * k)
    return wp.to(torch.bfloat16).contiguous(), b.contiguous(), k


class DPTHead(nn.Module):
    """dpt_head.py:179-236.  ``forward(inputs)``: the reference contract (list of 4 NCHW
    feature grids -> [NCHW f32 grid]); ``forward_nhwc`` takes NHWC bf16 inputs directly
    (the ViT's token layout, no transposition)."""

    def __init__(self, embed_dims=768, post_process_channels=None, readout_type="ignore",
                 patch_size=16, d_out=384, expand_channels=False):
        super().__init__()
        post = list(post_process_channels) if post_process_channels else [96, 192, 384, 768]
        self.post_process_channels = [min(d_out, c) for c in post]
        self.d_out = d_out
        self.expand_channels = expand_channels
        self.reassemble_blocks = ReassembleBlocks(embed_dims, self.post_process_channels,
                                                  readout_type, patch_size)
        self.convs = nn.ModuleList([nn.Conv2d(c, d_out, kernel_size=3, padding=1, bias=False)
                                    for c in self.post_process_channels])
        self.fusion_blocks = nn.ModuleList([FeatureFusionBlock(d_out) for _ in self.convs])
        self.fusion_blocks[0].res_conv_unit1 = None
        self.project = nn.Conv2d(d_out, d_out, kernel_size=3, padding=1)
        self.output_head = OutputHead(d_out)
        self._packed = None

    def _pack(self, key=None):
        """Packed weights, re-packed when the parameters changed (``key``: this module's
        _param_key if the caller has it already)."""
        key = _param_key(self) if key is None else key
        if self._packed is not None and self._packed[0] == key:
            return self._packed[1]
        rb = self.reassemble_blocks
        P = {
            "proj": [_pack_conv1(c) for c in rb.projects],
            "up0": _pack_convT(rb.resize_layers[0]), "up1": _pack_convT(rb.resize_layers[1]),
            "projup": [_pack_proj_convT(rb.projects[i], rb.resize_layers[i]) for i in (0, 1)],
            "down3": _pack_conv3(rb.resize_layers[3]),
            "convs": [_pack_conv3(c) for c in self.convs],
            "fusion": [{
                "rcu1": (None if fb.res_conv_unit1 is None else
                         (_pack_conv3(fb.res_conv_unit1.conv1), _pack_conv3(fb.res_conv_unit1.conv2))),
                "rcu2": (_pack_conv3(fb.res_conv_unit2.conv1), _pack_conv3(fb.res_conv_unit2.conv2)),
                "project": _pack_conv1(fb.project),
            } for fb in self.fusion_blocks],
            "project": _pack_conv3(self.project),
            "head0": _pack_conv3(self.output_head.head_modules[0]),
            "head1": _pack_convT(self.output_head.head_modules[1]),
            "head2": _pack_conv3(self.output_head.head_modules[2]),
        }
        self._packed = (key, P)
        return P

    def forward_level(self, i, x):
        """The per-level front of the head for NHWC bf16 tokens x of level i: the
        reassemble projection (+ its resize layer) and ``convs[i]`` (dpt_head.py:56-92,
        226-229).  The four levels are independent, so a caller may run them on side
        streams as their token grids appear (DINOv2Module._decode)."""
        L = _lib
        P = self._pack()
        if FOLD_UP and (i == 0 or i == 1):
            wf, bf, k = P["projup"][i]
            return L.conv3x3(L.linear_nhwc(x, wf, bf, shuf=k), *P["convs"][i])
        w, b = P["proj"][i]
        y = L.linear_nhwc(x, w, b)
        if i == 0 or i == 1:
            wt, bt, k = P["up0" if i == 0 else "up1"]
            y = L.linear_nhwc(y, wt, bt, shuf=k)
        elif i == 3:
            w3, b3 = P["down3"]
            y = L.conv3x3(y, w3, b3, stride=2)
        return L.conv3x3(y, *P["convs"][i])

    def forward_nhwc(self, xs, last: bool = True, levels=None):
        """xs: 4 NHWC bf16 tensors (B, h, w, embed) -> [f32 (B, d_out, H, W), channels-last].
        ``last=False`` stops before the final convolution and returns its NHWC bf16 input
        (``forward_last`` applies it: the graph-captured pass leaves that one launch out,
        so its output is a fresh tensor instead of a copy of a graph-owned buffer).
        ``levels``: forward_level outputs already computed (None entries are computed
        here)."""
        if torch.is_grad_enabled() and self.training:
            raise NotImplementedError("scenedino_amd DPT: no backward kernels; use no_grad / eval")
        L = _lib
        P = self._pack()
        levels = list(levels) if levels is not None else [None] * len(xs)
        f = [levels[i] if levels[i] is not None else self.forward_level(i, x) for i, x in enumerate(xs)]

        def rcu(x, pk, extra=None):
            (w1, b1), (w2, b2) = pk
            t = L.conv3x3(x, w1, b1, relu_in=True)
            return L.conv3x3(t, w2, b2, relu_in=True, res=x, res2=extra)  # conv2(..) + x (+ extra)

        def fusion(i, x, res=None):
            fp = P["fusion"][i]
            if res is not None:
                if res.shape != x.shape:  # dpt_head.py:152-154 (not hit by 192x640 frames)
                    res = F.interpolate(res.permute(0, 3, 1, 2).float(), size=x.shape[1:3],
                                        mode="bilinear", align_corners=False)
                    res = res.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()
                x = rcu(res, fp["rcu1"], extra=x)                   # x + rcu1(res)
            x = rcu(x, fp["rcu2"])
            w, b = fp["project"]
            if PROJECT_FIRST:
                # project (1x1 conv) before the x2 upsampling: both are linear and the
                # align_corners bilinear weights sum to one (the bias passes through), so
                # upsample(project(x)) = project(upsample(x)) -- on a quarter of the pixels
                return L.upsample2x(L.linear_nhwc(x, w, b))
            x = L.upsample2x(x)
            return L.linear_nhwc(x, w, b)

        out = fusion(0, f[-1])
        for i in range(1, len(self.fusion_blocks)):
            out = fusion(i, out, f[-(i + 1)])
        out = L.conv3x3(out, *P["project"])
        out = L.conv3x3(out, *P["head0"])
        wt, bt, k = P["head1"]
        out = L.linear_nhwc(out, wt, bt, shuf=k)
        return self.forward_last(out) if last else out

    def forward_last(self, x, key=None):
        """output_head.head_modules[2] (3x3 conv) on NHWC bf16 -> [(B, C, H, W) f32 grid].
        The grid is written channels-last (the GEMM's natural, coalesced output rows) and
        returned as its (B, C, H, W) permuted view: the reference's shape and values, and
        the layout every grid consumer here reads without a transposition
        (sd_project_grid_nhwc, sd_cast_grid, the training gather)."""
        w2, b2 = self._pack(key)["head2"]
        return [_lib.conv3x3(x, w2, b2, epi=_lib.SD_EPI_F32).permute(0, 3, 1, 2)]

    def forward(self, inputs):
        """dpt_head.py:226-236: list of 4 NCHW grids -> [NCHW f32 grid]."""
        xs = [x.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous() for x in inputs]
        return self.forward_nhwc(xs)
