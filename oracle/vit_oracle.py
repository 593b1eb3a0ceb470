"""vit_oracle -- TEST INFRASTRUCTURE ONLY (the checker, never shipped).

PyTorch CPU fp32 restatement of the ViT forward the reference runs through timm
(scenedino/models/backbones/dino/vit.py:48-62 timm.create_model, :112-189 _ViT with the
FX feature extractor; dinov2_module.py:225-227 _normalize_input, :258-288
DINOv2Encoder.forward).  timm itself is absent from this container and unpinned by the
reference (environment.yml:29), and its weights come from the HF hub, so this block is
restated from timm's published VisionTransformer: patch-embed convolution, class token,
+ pos_embed, pre-LN blocks x + ls1 * proj(attn(norm1 x)), x + ls2 * fc2(gelu(fc1(norm2
x))) with LayerNorm eps 1e-6, fused-qkv bias, softmax(q k^T * hd^-0.5), exact-erf GELU,
then the final norm.  PARITY UNPINNED by reference fixtures: the tests pin
the HIP kernels to this restatement on random weights.

Parameters are read from a scenedino_amd VisionTransformer container (timm's names).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

MEAN = torch.tensor([0.485, 0.456, 0.406])
STD = torch.tensor([0.229, 0.224, 0.225])


def normalize_input(x):
    """dinov2_module.py:225-227: Normalize(mean, std)(x / 2 + 0.5)."""
    x = x / 2 + 0.5
    return (x - MEAN.view(1, 3, 1, 1)) / STD.view(1, 3, 1, 1)


def block(x, b, nh):
    B, T, C = x.shape
    hd = C // nh
    y = F.layer_norm(x, (C,), b.norm1.weight, b.norm1.bias, 1e-6)
    qkv = F.linear(y, b.attn.qkv.weight, b.attn.qkv.bias).reshape(B, T, 3, nh, hd).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    attn = ((q * hd ** -0.5) @ k.transpose(-2, -1)).softmax(dim=-1)
    o = (attn @ v).transpose(1, 2).reshape(B, T, C)
    o = F.linear(o, b.attn.proj.weight, b.attn.proj.bias)
    x = x + (o * b.ls1.gamma if b.ls1 is not None else o)
    y = F.layer_norm(x, (C,), b.norm2.weight, b.norm2.bias, 1e-6)
    y = F.linear(F.gelu(F.linear(y, b.mlp.fc1.weight, b.mlp.fc1.bias)), b.mlp.fc2.weight, b.mlp.fc2.bias)
    return x + (y * b.ls2.gamma if b.ls2 is not None else y)


@torch.no_grad()
def encoder_forward(vit, images, intermediate):
    """images (B,3,H,W) in [-1,1] -> [grids of blocks in ``intermediate``, L2-normalised
    final tokens] each (B, C, gh, gw) (DINOv2Encoder.forward order)."""
    x = normalize_input(images.float())
    B = x.shape[0]
    C, nh, p = vit.embed_dim, vit.num_heads, vit.patch_size
    gh, gw = x.shape[-2] // p, x.shape[-1] // p
    t = F.conv2d(x, vit.patch_embed.proj.weight, vit.patch_embed.proj.bias, stride=p)
    t = t.flatten(2).transpose(1, 2)
    t = torch.cat([vit.cls_token.expand(B, -1, -1), t], 1) + vit.pos_embed
    grids = []
    to_grid = lambda z: z[:, 1:].transpose(1, 2).reshape(B, C, gh, gw)
    for i, b in enumerate(vit.blocks):
        t = block(t, b, nh)
        if i in intermediate:
            grids.append(to_grid(t))
    f = F.layer_norm(t, (C,), vit.norm.weight, vit.norm.bias, 1e-6)
    f = F.normalize(f[:, 1:], p=2, dim=2)                       # vit.py:188
    f = F.normalize(f.transpose(1, 2), dim=1).reshape(B, C, gh, gw)  # dinov2_module.py:281-286
    return grids + [f]
