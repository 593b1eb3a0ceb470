"""DINO / DINOv2 ViT encoder, MI355X build.

Mirror of scenedino/models/backbones/dino/vit.py (``_ViT`` :112-189 and the ``dino_*`` /
``dinov2_*`` factories :264-365) and of ``DINOv2Encoder`` (dinov2_module.py:230-339).
The reference wraps a timm ``VisionTransformer`` (pretrained weights fetched from the HF
hub at construction) in a torchvision FX feature extractor; this build holds the same
parameters under the same names (``vit.cls_token``, ``vit.pos_embed``,
``vit.patch_embed.proj``, ``vit.blocks.{i}.{norm1,attn.qkv,attn.proj,ls1.gamma,norm2,
mlp.fc1,mlp.fc2,ls2.gamma}``, ``vit.norm``), so the encoder keys of a SceneDINO
``checkpoint.pt`` load unchanged; it never downloads anything (weights come from the
checkpoint) and runs the forward pass in the gfx950 kernels of csrc/sdhip_vit.hip:
patchify + patch-embed GEMM, per block LayerNorm -> qkv GEMM (scattered into the
attention layouts) -> flash attention -> proj GEMM (+ residual, layer scale) ->
LayerNorm -> fc1 GEMM + GELU -> fc2 GEMM (+ residual), final LayerNorm, token -> grid.

timm's arithmetic (pre-LN block, LayerNorm eps 1e-6, qkv bias, scale head_dim^-1/2,
exact-erf GELU, DINOv2 LayerScale) is restated from the timm version the reference
imports (unpinned, environment.yml:29; timm is absent here): parity is pinned against
oracle/vit_oracle.py, a PyTorch fp32 restatement of that block.
"""
from __future__ import annotations

import os

from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F
from torch import nn

from .... import _lib

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


class _LayerScale(nn.Module):
    def __init__(self, dim, init_values=1e-5):
        super().__init__()
        self.gamma = nn.Parameter(init_values * torch.ones(dim))


class _Attention(nn.Module):
    def __init__(self, dim, num_heads):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.scale = self.head_dim ** -0.5
        self.qkv = nn.Linear(dim, 3 * dim, bias=True)
        self.proj = nn.Linear(dim, dim)


class _Mlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.fc2 = nn.Linear(hidden, dim)


class _Block(nn.Module):
    def __init__(self, dim, num_heads, mlp_ratio=4.0, layer_scale=False):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = _Attention(dim, num_heads)
        self.ls1 = _LayerScale(dim) if layer_scale else None
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = _Mlp(dim, int(dim * mlp_ratio))
        self.ls2 = _LayerScale(dim) if layer_scale else None


class _PatchEmbed(nn.Module):
    def __init__(self, patch_size, dim):
        super().__init__()
        self.proj = nn.Conv2d(3, dim, kernel_size=patch_size, stride=patch_size)


class VisionTransformer(nn.Module):
    """Parameter container with timm's VisionTransformer names (class token, no
    registers, global_pool '' / num_classes 0 as _load_vit builds it)."""

    def __init__(self, img_size: Tuple[int, int], patch_size: int, embed_dim: int, depth: int,
                 num_heads: int, layer_scale: bool = False):
        super().__init__()
        self.patch_size = patch_size
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        gh, gw = img_size[0] // patch_size, img_size[1] // patch_size
        self.grid_size = (gh, gw)
        self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
        self.pos_embed = nn.Parameter(torch.randn(1, gh * gw + 1, embed_dim) * 0.02)
        self.patch_embed = _PatchEmbed(patch_size, embed_dim)
        self.blocks = nn.ModuleList(
            [_Block(embed_dim, num_heads, layer_scale=layer_scale) for _ in range(depth)])
        self.norm = nn.LayerNorm(embed_dim, eps=1e-6)


class _Packed:
    """bf16 GEMM operands of a VisionTransformer, built once per parameter version."""

    def __init__(self, vit: VisionTransformer):
        bf = torch.bfloat16
        p = vit.patch_size
        C = vit.embed_dim
        k = 3 * p * p
        self.Kp = (k + 31) // 32 * 32
        w = vit.patch_embed.proj.weight.detach().reshape(C, k)
        self.w_pe = F.pad(w, (0, self.Kp - k)).to(bf).contiguous()
        self.b_pe = vit.patch_embed.proj.bias.detach().float().contiguous()
        self.cls = vit.cls_token.detach().float().reshape(C).contiguous()
        self.pos = vit.pos_embed.detach().float().reshape(-1, C).contiguous()
        f = lambda t: t.detach().float().contiguous()
        self.blocks = []
        for b in vit.blocks:
            self.blocks.append({
                "n1w": f(b.norm1.weight), "n1b": f(b.norm1.bias),
                "qkv_w": b.attn.qkv.weight.detach().to(bf).contiguous(), "qkv_b": f(b.attn.qkv.bias),
                "proj_w": b.attn.proj.weight.detach().to(bf).contiguous(), "proj_b": f(b.attn.proj.bias),
                "ls1": f(b.ls1.gamma) if b.ls1 is not None else None,
                "n2w": f(b.norm2.weight), "n2b": f(b.norm2.bias),
                "fc1_w": b.mlp.fc1.weight.detach().to(bf).contiguous(), "fc1_b": f(b.mlp.fc1.bias),
                "fc2_w": b.mlp.fc2.weight.detach().to(bf).contiguous(), "fc2_b": f(b.mlp.fc2.bias),
                "ls2": f(b.ls2.gamma) if b.ls2 is not None else None,
            })
        self.nw, self.nb = f(vit.norm.weight), f(vit.norm.bias)


def _param_key(m: nn.Module):
    """(storage, version) of every parameter: changes on load_state_dict, in-place edits,
    .to() and Parameter replacement.  The module list is collected once (a recursive
    m.parameters() walk costs ~0.3 ms of host time per encode for ViT + DPT, enough to
    starve the launch queue); re-structuring a module after its first forward is not
    tracked."""
    mods = m.__dict__.get("_sd_modules")
    if mods is None:
        mods = list(m.modules())
        m.__dict__["_sd_modules"] = mods
    return tuple((t.data_ptr(), t._version) for x in mods for t in x._parameters.values()
                 if t is not None)


# fuse the block norms into the qkv / fc1 GEMMs (sd_ln_gemm); SCENEDINO_AMD_LN_GEMM=0 keeps
# the separate sd_layernorm launches (A/B runs)
LN_GEMM = os.environ.get("SCENEDINO_AMD_LN_GEMM", "1") != "0"
LN_GEMM_ALL = os.environ.get("SCENEDINO_AMD_LN_GEMM", "1") == "all"  # also C = 768 (A/B runs)
# SCENEDINO_AMD_LN_TAIL=1: the block norms written by the preceding residual GEMM's last
# workgroup per row band (sd_gemm_resid_ln): no LayerNorm launch, a plain GEMM for qkv /
# fc1.  Bit-equal, but measured slower (ViT-S/16 0.588 -> 0.88 ms, DINOv2-B/14 0.876 ->
# 1.23: the band's write-through stores, ticket and read-back cost 11-16 us per residual
# GEMM against the 5 us LayerNorm launch they replace, profiles/r4_ln_tail_ab.txt): off
LN_TAIL = os.environ.get("SCENEDINO_AMD_LN_TAIL", "0") == "1"
# the DPT's intermediate token grids written by fc2's residual epilogue (no tokens_to_nhwc
# launches); SCENEDINO_AMD_FC2_GRID=0 restores the separate launches (A/B runs)
FC2_GRID = os.environ.get("SCENEDINO_AMD_FC2_GRID", "1") != "0"
# the MLP half of a C = 384 block as one launch (sd_vit_mlp: norm2 + fc1 + GELU + fc2 +
# residual, f32 atomics into the residual stream): 5 launches per block -> 4, but measured
# SLOWER (ViT-S/16 0.519 -> 0.611 ms, profiles/r5_vit_mlp_ab.txt: 96 workgroups each stream
# 393 KB of fc1 / fc2 weights, against the two GEMMs' 384 + 192 small tiles) and not
# bit-reproducible (atomics: graph vs eager outputs differ by 5e-4 rel-L2); off by default,
# SCENEDINO_AMD_VIT_MLP=1 selects it (A/B runs)
VIT_MLP = os.environ.get("SCENEDINO_AMD_VIT_MLP", "0") == "1"


def vit_forward(vit: VisionTransformer, images: torch.Tensor, packed: _Packed,
                intermediate: List[int], nhwc: bool = False, on_grid=None):
    """images (B, 3, H, W) in [-1, 1] (DINOv2Encoder input, before _normalize_input) ->
    (intermediate block outputs as (B, C, gh, gw) f32 grids, final-norm tokens
    L2-normalised as a grid).  ``nhwc=True`` returns (B, gh, gw, C) bf16 grids instead: the
    DPT decoder's operand layout, written straight from the token rows.  ``on_grid(i, g)``
    is called as each intermediate grid is written (the caller may start consuming it on
    another stream while the later blocks run).  Every arithmetic step is a libsdhip.so
    kernel."""
    if torch.is_grad_enabled() and vit.training:
        raise NotImplementedError("scenedino_amd ViT: no backward kernels; use no_grad / eval")
    B, _, H, W = images.shape
    p, C, nh = vit.patch_size, vit.embed_dim, vit.num_heads
    gh, gw = H // p, W // p
    Np = gh * gw
    T = Np + 1
    if packed.pos.shape[0] != T:
        raise ValueError(f"pos_embed holds {packed.pos.shape[0]} tokens, the image gives {T}")
    hd = C // nh
    if hd != 64:
        raise NotImplementedError("sd_attention implements head_dim 64 (ViT-S/B, DINO/DINOv2)")
    dev = images.device
    bf = torch.bfloat16
    Tp = (T + 63) // 64 * 64
    img = images.float().contiguous()
    x = torch.empty(B * T, C, device=dev)
    patches = torch.empty(B * Np, packed.Kp, device=dev, dtype=bf)
    _lib.patchify(img, p, packed.Kp, IMAGENET_MEAN, IMAGENET_STD, patches, packed.cls,
                  packed.pos, x)
    _lib.gemm(patches, packed.w_pe, packed.b_pe, _lib.SD_EPI_PATCH, out=x, pos=packed.pos,
              patches=Np)
    xn = torch.empty(B * T, C, device=dev, dtype=bf)
    q = torch.empty(B, nh, T, hd, device=dev, dtype=bf)
    # K / V^T with their token padding (rows / columns T .. Tp - 1) zero: allocated and zeroed
    # once per shape and kept on the packed weights -- the qkv epilogue writes only the
    # first T tokens, so the padding stays zero, and a captured pass holds no memset launches
    # (two ~5 us fills per pass).  One pass at a time per model, as the LayerNorm-tail
    # tickets below.
    kv = getattr(packed, "_kv", None)
    kkey = (B, nh, T, Tp, hd, str(dev))
    if kv is None or kv[0] != kkey:
        kv = packed._kv = (kkey, torch.zeros(B, nh, Tp, hd, device=dev, dtype=bf),
                           torch.zeros(B, nh, hd, Tp, device=dev, dtype=bf))
    k, vt = kv[1], kv[2]
    ao = torch.empty(B * T, C, device=dev, dtype=bf)
    hid = torch.empty(B * T, packed.blocks[0]["fc1_w"].shape[0], device=dev, dtype=bf)
    grids = []
    to_grid = _lib.tokens_to_nhwc if nhwc else _lib.tokens_to_grid
    scale = hd ** -0.5
    # norm1 / norm2 fused into the qkv / fc1 GEMM prologues (sd_ln_gemm: 32 x 128 tiles) for
    # ViT-S at small token counts (481 tokens: 0.61 -> 0.57 ms per pass); measured slower
    # for C = 768 (DINOv2-B/14: 0.90 -> 0.99 ms against sd_layernorm + the 64 x 64-tile
    # sd_gemm) and at 1921 tokens (the narrow tile re-reads the weights per row tile)
    fuse_ln = (C == 384 or LN_GEMM_ALL) and LN_GEMM and B * T <= 1024
    # the LayerNorm tails: the token-global residual stream is normalised by the residual
    # GEMM that produced it (one ticket word per 32-row band, self-resetting, per model)
    tail = LN_TAIL and C <= 1024 and C % 4 == 0
    ws = None
    if tail:
        ws = getattr(packed, "_ln_ws", None)
        if ws is None or ws.device != dev or ws.numel() < (B * T + 31) // 32:
            ws = packed._ln_ws = torch.zeros((B * T + 31) // 32, device=dev, dtype=torch.int32)
    nblk = len(packed.blocks)
    hidden = packed.blocks[0]["fc1_w"].shape[0]
    fused_mlp = VIT_MLP and not tail and C == 384 and hidden % 256 == 0
    xc = torch.empty_like(x) if fused_mlp else None  # x after the attention half (LN2 input)
    xn_ready = False  # xn holds this block's norm1 (the previous fc2's tail)
    for i, blk in enumerate(packed.blocks):
        if xn_ready:
            _lib.gemm(xn, blk["qkv_w"], blk["qkv_b"], _lib.SD_EPI_QKV, qkv=(q, k, vt), tokens=T,
                      heads=nh)
        elif fuse_ln:
            _lib.ln_gemm(x, blk["n1w"], blk["n1b"], 1e-6, blk["qkv_w"], blk["qkv_b"],
                         _lib.SD_EPI_QKV, qkv=(q, k, vt), tokens=T, heads=nh)
        else:
            _lib.layernorm(x, blk["n1w"], blk["n1b"], 1e-6, xn)
            _lib.gemm(xn, blk["qkv_w"], blk["qkv_b"], _lib.SD_EPI_QKV, qkv=(q, k, vt), tokens=T,
                      heads=nh)
        _lib.attention(q, k, vt, scale, ao)
        if fused_mlp:  # proj (+ the f32 copy), then norm2 .. fc2 + residual in one launch
            _lib.gemm(ao, blk["proj_w"], blk["proj_b"], _lib.SD_EPI_RESID, out=x, gamma=blk["ls1"],
                      copy_out=xc)
            _lib.vit_mlp(xc, x, blk["n2w"], blk["n2b"], 1e-6, blk["fc1_w"], blk["fc1_b"],
                         blk["fc2_w"], blk["fc2_b"], gamma=blk["ls2"])
            if i in intermediate:
                grids.append(to_grid(x, B, T, C, 1, gh, gw, False))
                if on_grid is not None:
                    on_grid(len(grids) - 1, grids[-1])
            continue
        if tail:  # proj + norm2 -> xn, then fc1 as a plain GEMM
            _lib.gemm(ao, blk["proj_w"], blk["proj_b"], _lib.SD_EPI_RESID, out=x, gamma=blk["ls1"],
                      ln=(blk["n2w"], blk["n2b"], 1e-6, xn, ws))
            _lib.gemm(xn, blk["fc1_w"], blk["fc1_b"], _lib.SD_EPI_GELU, out=hid)
        else:
            _lib.gemm(ao, blk["proj_w"], blk["proj_b"], _lib.SD_EPI_RESID, out=x, gamma=blk["ls1"])
            if fuse_ln:
                _lib.ln_gemm(x, blk["n2w"], blk["n2b"], 1e-6, blk["fc1_w"], blk["fc1_b"],
                             _lib.SD_EPI_GELU, out=hid)
            else:
                _lib.layernorm(x, blk["n2w"], blk["n2b"], 1e-6, xn)
                _lib.gemm(xn, blk["fc1_w"], blk["fc1_b"], _lib.SD_EPI_GELU, out=hid)
        nxt = packed.blocks[i + 1] if tail and i + 1 < nblk else None
        ln = (nxt["n1w"], nxt["n1b"], 1e-6, xn, ws) if nxt is not None else None
        if i in intermediate and nhwc and FC2_GRID:  # the DPT's bf16 token grid from fc2's epilogue
            grid = torch.empty(B, gh, gw, C, device=dev, dtype=bf)
            _lib.gemm(hid, blk["fc2_w"], blk["fc2_b"], _lib.SD_EPI_RESID, out=x, gamma=blk["ls2"],
                      tokens=T, grid_out=grid, ln=ln)
            grids.append(grid)
        else:
            _lib.gemm(hid, blk["fc2_w"], blk["fc2_b"], _lib.SD_EPI_RESID, out=x, gamma=blk["ls2"],
                      ln=ln)
            if i in intermediate:
                grids.append(to_grid(x, B, T, C, 1, gh, gw, False))
        xn_ready = nxt is not None
        if i in intermediate:
            if on_grid is not None:
                on_grid(len(grids) - 1, grids[-1])
    if nhwc and FC2_GRID:  # final norm + L2-normalised bf16 grid in one launch
        return grids, _lib.layernorm_nhwc(x, packed.nw, packed.nb, 1e-6, B, T, C, 1, gh, gw, True)
    xf = torch.empty(B * T, C, device=dev)
    _lib.layernorm(x, packed.nw, packed.nb, 1e-6, xf)
    final = to_grid(xf, B, T, C, 1, gh, gw, True)
    return grids, final


class _ViT(nn.Module):
    """vit.py:112-189: holds ``self.vit``; forward(images) -> output dict with
    ``features_normalized`` (B, N, C) and ``intermediate_features.{idx}`` (B, N, C), class
    token removed.  Unlike the reference (which gets ImageNet-normalised images), the
    kernels fold the input normalisation into the patchify step: ``forward_grids`` takes
    the raw [-1, 1] images."""

    def __init__(self, vit: VisionTransformer, patch_size: int, registers: bool = False,
                 class_token: bool = True, intermediate_features: Optional[List[int]] = None):
        super().__init__()
        if registers or not class_token:
            raise NotImplementedError("register-token / no-class-token ViTs are not in the "
                                      "shipped configs")
        self.patch_size = patch_size
        self.registers = registers
        self.class_token = class_token
        self.intermediate = list(intermediate_features or [])
        self.vit = vit
        self._packed = None
        self._graph = None
        self.use_graph = True

    def packed(self):
        key = _param_key(self.vit)
        if self._packed is None or self._packed[0] != key:
            self._packed = (key, _Packed(self.vit))
        return self._packed[1]

    def forward_grids(self, images_pm1):
        """HIP-graph replay of the whole encoder (patchify, 12 x 7 kernels, final norm,
        grids): captured once per (input shape, parameter version), then replayed -- the
        ~90 launches of a pass cost one graph launch.  ``use_graph = False`` launches
        eagerly."""
        if not self.use_graph or not images_pm1.is_cuda:
            return vit_forward(self.vit, images_pm1, self.packed(), self.intermediate)
        key = (tuple(images_pm1.shape), str(images_pm1.device), _param_key(self.vit))
        if self._graph is None or self._graph[0] != key:
            self._graph = None
            packed = self.packed()
            static_in = images_pm1.detach().float().contiguous().clone()
            side = torch.cuda.Stream(device=images_pm1.device)
            side.wait_stream(torch.cuda.current_stream(images_pm1.device))
            with torch.cuda.stream(side):  # warm-up outside the capture
                vit_forward(self.vit, static_in, packed, self.intermediate)
            torch.cuda.current_stream(images_pm1.device).wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                outs = vit_forward(self.vit, static_in, packed, self.intermediate)
            self._graph = (key, graph, static_in, outs)
        _, graph, static_in, (grids, final) = self._graph
        static_in.copy_(images_pm1)
        graph.replay()
        return [g.clone() for g in grids], final.clone()

    def forward(self, images_pm1) -> Dict[str, torch.Tensor]:
        grids, final = self.forward_grids(images_pm1)
        out = {"features_normalized": final.flatten(2).transpose(1, 2)}
        for idx, g in enumerate(grids):
            out[f"intermediate_features.{idx}"] = g.flatten(2).transpose(1, 2)
        return out


_ARCH = {"vit-s": (384, 6), "vit-b": (768, 12)}
_PATCH = {"v1": 8, "v1_16": 16, "v2": 14}


def _make(backbone, version, image_size, intermediate_features):
    dim, heads = _ARCH[backbone]
    p = _PATCH[version]
    vit = VisionTransformer(image_size, p, dim, 12, heads, layer_scale=(version == "v2"))
    return _ViT(vit, p, class_token=True, intermediate_features=intermediate_features)


def dino_small(image_size=(224, 224), intermediate_features=None):
    """vit_small_patch16_224.dino (vit.py:264-278)."""
    return _make("vit-s", "v1_16", image_size, intermediate_features)


def dino_small8(image_size=(224, 224), intermediate_features=None):
    """vit_small_patch8_224.dino (vit.py:281-295)."""
    return _make("vit-s", "v1", image_size, intermediate_features)


def dino_base(image_size=(224, 224), intermediate_features=None):
    """vit_base_patch16_224.dino (vit.py:298-312)."""
    return _make("vit-b", "v1_16", image_size, intermediate_features)


def dino_base8(image_size=(224, 224), intermediate_features=None):
    """vit_base_patch8_224.dino (vit.py:315-329)."""
    return _make("vit-b", "v1", image_size, intermediate_features)


def dinov2_small(image_size=(224, 224), intermediate_features=None):
    """vit_small_patch14_dinov2.lvd142m (vit.py:332-347)."""
    return _make("vit-s", "v2", image_size, intermediate_features)


def dinov2_base(image_size=(224, 224), intermediate_features=None):
    """vit_base_patch14_dinov2.lvd142m (vit.py:350-365)."""
    return _make("vit-b", "v2", image_size, intermediate_features)


class DINOv2Encoder(nn.Module):
    """dinov2_module.py:230-339: ``forward(x)`` (x in [-1, 1]) -> [grid of block i for i in
    intermediate_features (B, C, h, w), L2-normalised final tokens (B, C, h, w)]."""

    def __init__(self, backbone, image_size, intermediate_features, key_features, version):
        super().__init__()
        if key_features:
            raise NotImplementedError("key_features=True is not used by the shipped configs")
        if version not in ("v1", "v1_16", "v2"):
            raise NotImplementedError(f"DINO version {version!r} (fit3d / reg need registers "
                                      "or a hub download)")
        self.image_size = tuple(image_size)
        self.backbone = backbone
        self.version = version
        self.key_features = key_features
        if version == "v2":  # internal patch 14, external 16 (dinov2_module.py:235-240)
            self.patch_size = 16
            adjusted = (image_size[0] * 14 // 16, image_size[1] * 14 // 16)
            self.resize = adjusted
        else:
            self.patch_size = _PATCH[version]
            adjusted = tuple(image_size)
            self.resize = None
        factory = {("vit-s", "v1"): dino_small8, ("vit-b", "v1"): dino_base8,
                   ("vit-s", "v1_16"): dino_small, ("vit-b", "v1_16"): dino_base,
                   ("vit-s", "v2"): dinov2_small, ("vit-b", "v2"): dinov2_base}
        self.model = factory[(backbone, version)](image_size=adjusted,
                                                  intermediate_features=intermediate_features)
        self.latent_size = _ARCH[backbone][0]

    def forward(self, x):
        if self.resize is not None:
            # torchvision Resize(bilinear) on a tensor: antialiased bilinear interpolation
            # (a device op; the [-1,1] -> ImageNet normalisation commutes with it)
            x = F.interpolate(x, size=self.resize, mode="bilinear", align_corners=False,
                              antialias=True)
        grids, final = self.model.forward_grids(x)
        return grids + [final]
