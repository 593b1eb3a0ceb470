"""ViT encoder: DINO / DINOv2 blocks on gfx950 MFMA.

timm is absent here and unpinned by the reference, so parity is pinned to
oracle/vit_oracle.py (PyTorch fp32 restatement of timm's VisionTransformer as the
reference runs it) on random weights -- "parity unpinned" against reference fixtures.

Tolerances (written here):
  * sd_gemm (bf16 operands, fp32 accumulate): vs fp32 matmul of the same bf16 operands,
    max |d| <= 1e-3 * sqrt(K) * max|ref| scale for f32 epilogues; bf16 outputs add one bf16
    rounding (rel 2^-8).
  * sd_attention: vs fp32 softmax attention of the same bf16 q, k, v: max |d| <= 2e-2.
  * sd_layernorm: vs F.layer_norm, bf16 output: max |d| <= 2e-2 (|y| ~ 1).
  * full encoder (12 blocks, bf16 activations, fp32 residual stream): per output grid
    rel-L2 <= 3e-2 against the fp32 oracle.
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import vit_oracle as VO


def init_vit(vit, seed=0):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in vit.named_parameters():
            if name.endswith("gamma"):
                p.copy_(0.5 + 0.2 * torch.rand(p.shape, generator=g))
            elif "norm" in name and name.endswith("weight"):
                p.copy_(1 + 0.1 * torch.randn(p.shape, generator=g))
            elif name.endswith("bias"):
                p.copy_(0.02 * torch.randn(p.shape, generator=g))
            elif name in ("cls_token", "pos_embed"):
                p.copy_(0.3 * torch.randn(p.shape, generator=g))
            else:
                fan_in = p[0].numel()
                p.copy_(torch.randn(p.shape, generator=g) / math.sqrt(fan_in))
    return vit


def test_state_dict_keys_follow_timm_names():
    from scenedino_amd.models.backbones.dino.vit import DINOv2Encoder
    enc = DINOv2Encoder("vit-s", (192, 640), [3, 6, 9], False, "v2")
    keys = set(enc.state_dict())
    for k in ("model.vit.cls_token", "model.vit.pos_embed", "model.vit.patch_embed.proj.weight",
              "model.vit.blocks.0.norm1.weight", "model.vit.blocks.0.attn.qkv.weight",
              "model.vit.blocks.0.attn.qkv.bias", "model.vit.blocks.0.attn.proj.bias",
              "model.vit.blocks.0.ls1.gamma", "model.vit.blocks.11.mlp.fc1.weight",
              "model.vit.blocks.11.mlp.fc2.bias", "model.vit.blocks.11.ls2.gamma",
              "model.vit.norm.weight"):
        assert k in keys, k
    assert enc.model.vit.pos_embed.shape == (1, 12 * 40 + 1, 384)  # 168x560 / 14
    e1 = DINOv2Encoder("vit-b", (192, 640), [3, 6, 9], False, "v1")
    assert e1.model.vit.pos_embed.shape == (1, 24 * 80 + 1, 768)
    assert "model.vit.blocks.0.ls1.gamma" not in set(e1.state_dict())


def test_oracle_shapes_and_normalisation():
    from scenedino_amd.models.backbones.dino.vit import VisionTransformer
    vit = init_vit(VisionTransformer((32, 64), 16, 384, 2, 6))
    out = VO.encoder_forward(vit, torch.rand(2, 3, 32, 64) * 2 - 1, [0])
    assert [tuple(o.shape) for o in out] == [(2, 384, 2, 4), (2, 384, 2, 4)]
    assert torch.allclose(out[-1].norm(dim=1), torch.ones(2, 2, 4), atol=1e-5)


# ------------------------------------------------------------------------ GPU
@pytest.fixture(scope="module")
def gpu():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    from scenedino_amd import _lib
    _lib.load()
    return "cuda"


def _bf(t):
    return t.to(torch.bfloat16)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(481, 1152, 384), (77, 96, 64), (1921, 768, 3072),
                                   (4096, 1024, 256)])
def test_gemm_epilogues(gpu, M, N, K):
    from scenedino_amd import _lib
    g = torch.Generator().manual_seed(M + N)
    a = _bf(torch.randn(M, K, generator=g)).to(gpu)
    w = _bf(torch.randn(N, K, generator=g) / math.sqrt(K)).to(gpu)
    bias = (0.1 * torch.randn(N, generator=g)).to(gpu)
    ref = a.float() @ w.float().t() + bias
    scale = ref.abs().max().item()
    out = torch.empty(M, N, device=gpu)
    _lib.gemm(a, w, bias, _lib.SD_EPI_F32, out=out)
    assert (out - ref).abs().max().item() <= 1e-4 * scale + 1e-5
    ob = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    _lib.gemm(a, w, bias, _lib.SD_EPI_BF16, out=ob)
    assert (ob.float() - ref).abs().max().item() <= 8e-3 * scale
    _lib.gemm(a, w, bias, _lib.SD_EPI_GELU, out=ob)
    assert (ob.float() - F.gelu(ref)).abs().max().item() <= 8e-3 * scale
    res = torch.randn(M, N, generator=g).to(gpu)
    gam = torch.rand(N, generator=g).to(gpu)
    x = res.clone()
    _lib.gemm(a, w, bias, _lib.SD_EPI_RESID, out=x, gamma=gam)
    assert (x - (res + gam * ref)).abs().max().item() <= 1e-4 * scale + 1e-5
    x = res.clone()
    _lib.gemm(a, w, None, _lib.SD_EPI_RESID, out=x)
    assert (x - (res + ref - bias)).abs().max().item() <= 1e-4 * scale + 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("B,gh,gw,C", [(1, 12, 40, 384), (2, 3, 5, 768), (1, 1, 3, 1024)])
@pytest.mark.parametrize("l2", [True, False])
def test_layernorm_nhwc_equals_two_launches(gpu, B, gh, gw, C, l2):
    """sd_layernorm_nhwc (the encoder's final norm straight into the DPT's last token grid)
    is bit-equal to sd_layernorm (f32 rows) followed by sd_tokens_to_nhwc."""
    from scenedino_amd import _lib
    g = torch.Generator().manual_seed(C + gw)
    T = gh * gw + 1
    x = (2 * torch.randn(B * T, C, generator=g) + 0.3).to(gpu)
    w = (1 + 0.1 * torch.randn(C, generator=g)).to(gpu)
    b = (0.1 * torch.randn(C, generator=g)).to(gpu)
    xf = torch.empty(B * T, C, device=gpu)
    _lib.layernorm(x, w, b, 1e-6, xf)
    ref = _lib.tokens_to_nhwc(xf, B, T, C, 1, gh, gw, l2)
    got = _lib.layernorm_nhwc(x, w, b, 1e-6, B, T, C, 1, gh, gw, l2)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("B,gh,gw,C,Kh", [(1, 12, 40, 384, 1536), (2, 3, 5, 768, 3072)])
def test_resid_epilogue_writes_the_token_grid(gpu, B, gh, gw, C, Kh):
    """fc2's residual epilogue with grid_out also writes the intermediate-layer NHWC bf16
    grid (the class token dropped): bit-equal to sd_tokens_to_nhwc of the updated rows,
    which the ViT no longer launches for the DPT's intermediate layers."""
    from scenedino_amd import _lib
    g = torch.Generator().manual_seed(B * gh + C)
    T = gh * gw + 1
    M = B * T
    hid = _bf(torch.randn(M, Kh, generator=g)).to(gpu)
    w = _bf(torch.randn(C, Kh, generator=g) / math.sqrt(Kh)).to(gpu)
    b = (0.1 * torch.randn(C, generator=g)).to(gpu)
    gam = torch.rand(C, generator=g).to(gpu)
    x0 = torch.randn(M, C, generator=g).to(gpu)
    x1, x2 = x0.clone(), x0.clone()
    grid = torch.empty(B, gh, gw, C, device=gpu, dtype=torch.bfloat16)
    _lib.gemm(hid, w, b, _lib.SD_EPI_RESID, out=x1, gamma=gam, tokens=T, grid_out=grid)
    _lib.gemm(hid, w, b, _lib.SD_EPI_RESID, out=x2, gamma=gam)
    assert torch.equal(x1, x2)
    ref = _lib.tokens_to_nhwc(x2, B, T, C, 1, gh, gw, False)
    torch.cuda.synchronize()
    assert torch.equal(grid, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(481, 384, 384), (481, 384, 1536), (481, 768, 768),
                                   (481, 768, 3072), (1921, 768, 3072), (97, 384, 1536),
                                   (8192, 1024, 256), (50, 256, 512)])
def test_resid_gemm_layernorm_tail_equals_two_launches(gpu, M, N, K):
    """sd_gemm_resid_ln: the residual GEMM whose row bands' last workgroups also write the
    next block norm's bf16 rows -- the residual stream bit-equal to sd_gemm and the
    normalised rows bit-equal to sd_layernorm on it, on each tiling the shapes pick (32 x 32
    split-K tiles with 128- / 256-deep steps, 64 x 64, 128 x 128; ragged last bands), over
    repeated launches (self-resetting tickets)."""
    from scenedino_amd import _lib
    g = torch.Generator().manual_seed(M + N + K)
    a = _bf(torch.randn(M, K, generator=g)).to(gpu)
    w = _bf(torch.randn(N, K, generator=g) / math.sqrt(K)).to(gpu)
    b = (0.1 * torch.randn(N, generator=g)).to(gpu)
    gam = torch.rand(N, generator=g).to(gpu)
    lw = (1 + 0.1 * torch.randn(N, generator=g)).to(gpu)
    lb = (0.1 * torch.randn(N, generator=g)).to(gpu)
    x0 = (torch.randn(M, N, generator=g) + 0.5).to(gpu)
    ws = torch.zeros((M + 31) // 32, device=gpu, dtype=torch.int32)
    x2 = x0.clone()
    _lib.gemm(a, w, b, _lib.SD_EPI_RESID, out=x2, gamma=gam)
    ref = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    _lib.layernorm(x2, lw, lb, 1e-6, ref)
    for _ in range(3):
        x1 = x0.clone()
        xn = torch.full((M, N), float("nan"), device=gpu, dtype=torch.bfloat16)
        _lib.gemm(a, w, b, _lib.SD_EPI_RESID, out=x1, gamma=gam, ln=(lw, lb, 1e-6, xn, ws))
        torch.cuda.synchronize()
        assert torch.equal(x1, x2)
        assert torch.equal(xn, ref)
        assert int(ws.abs().sum()) == 0  # tickets reset
    ln_ref = torch.nn.functional.layer_norm(x2, (N,), lw, lb, 1e-6)
    assert (xn.float() - ln_ref).abs().max().item() < 0.05


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(481, 384, 1536), (481, 384, 1024), (97, 64, 2048)])
def test_gemm_cross_workgroup_split_k(gpu, M, N, K, monkeypatch):
    """32 x 32 tiles whose K range is split over workgroups (SD_SPLITK_WG=512 forces it on the ViT-S/16 fc2 at 481 tokens: two
    slices; the last arriver sums the slices' f32 partials in slice order): every epilogue
    equals the f32 product within the single-workgroup tolerance, the result is
    bit-identical across launches (deterministic combine, self-resetting tickets), and
    SD_SPLITK_WG=0 (no split) agrees."""
    from scenedino_amd import _lib
    g = torch.Generator().manual_seed(M + K)
    a = _bf(torch.randn(M, K, generator=g)).to(gpu)
    w = _bf(torch.randn(N, K, generator=g) / math.sqrt(K)).to(gpu)
    bias = (0.1 * torch.randn(N, generator=g)).to(gpu)
    ref = a.float() @ w.float().t() + bias
    scale = ref.abs().max().item()
    res = torch.randn(M, N, generator=g).to(gpu)
    gam = torch.rand(N, generator=g).to(gpu)

    def run():
        out = torch.empty(M, N, device=gpu)
        _lib.gemm(a, w, bias, _lib.SD_EPI_F32, out=out)
        x = res.clone()
        _lib.gemm(a, w, bias, _lib.SD_EPI_RESID, out=x, gamma=gam)
        ob = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
        _lib.gemm(a, w, bias, _lib.SD_EPI_GELU, out=ob)
        torch.cuda.synchronize()
        return out, x, ob

    monkeypatch.setenv("SD_SPLITK_WG", "512")  # split these shapes (the default cap is 1 tile per CU)
    runs = [run() for _ in range(3)]
    out, x, ob = runs[0]
    assert (out - ref).abs().max().item() <= 1e-4 * scale + 1e-5
    assert (x - (res + gam * ref)).abs().max().item() <= 1e-4 * scale + 1e-5
    assert (ob.float() - F.gelu(ref)).abs().max().item() <= 8e-3 * scale
    for r in runs[1:]:
        for t0, t1 in zip(runs[0], r):
            assert torch.equal(t0, t1)
    monkeypatch.setenv("SD_SPLITK_WG", "0")
    o1, x1, _ = run()
    assert (o1 - out).abs().max().item() <= 1e-4 * scale + 1e-5
    assert (x1 - x).abs().max().item() <= 1e-4 * scale + 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,T", [(1, 6, 481), (2, 12, 77), (1, 12, 1921), (1, 1, 1),
                                   (4, 12, 1921)])
@pytest.mark.parametrize("mode", ["auto", "lds", "dir", "2split"])
def test_qkv_scatter_and_attention(gpu, B, H, T, mode, monkeypatch):
    """k_attn_lds<1> (128 queries sharing LDS K / V^T), k_attn_lds<2> (64 queries per key
    half, halves merged through LDS) and k_attn_dir (32 queries x 4 key quarters, fragments
    from L2): the launcher picks by occupancy, SD_ATTN forces one."""
    if mode != "auto":
        monkeypatch.setenv("SD_ATTN", mode)
    from scenedino_amd import _lib
    g = torch.Generator().manual_seed(T)
    C = 64 * H
    xn = _bf(torch.randn(B * T, C, generator=g)).to(gpu)
    w = _bf(torch.randn(3 * C, C, generator=g) / math.sqrt(C)).to(gpu)
    b = (0.1 * torch.randn(3 * C, generator=g)).to(gpu)
    Tp = (T + 63) // 64 * 64
    q = torch.empty(B, H, T, 64, device=gpu, dtype=torch.bfloat16)
    k = torch.zeros(B, H, Tp, 64, device=gpu, dtype=torch.bfloat16)
    vt = torch.zeros(B, H, 64, Tp, device=gpu, dtype=torch.bfloat16)
    _lib.gemm(xn, w, b, _lib.SD_EPI_QKV, qkv=(q, k, vt), tokens=T, heads=H)
    qkv = torch.empty(B * T, 3 * C, device=gpu, dtype=torch.bfloat16)
    _lib.gemm(xn, w, b, _lib.SD_EPI_BF16, out=qkv)
    r = qkv.view(B, T, 3, H, 64).permute(2, 0, 3, 1, 4)
    assert torch.equal(q, r[0])
    assert torch.equal(k[:, :, :T], r[1])
    assert torch.equal(vt[..., :T], r[2].transpose(-1, -2))
    assert not k[:, :, T:].any() and not vt[..., T:].any()
    out = torch.empty(B * T, C, device=gpu, dtype=torch.bfloat16)
    _lib.attention(q, k, vt, 64 ** -0.5, out)
    att = ((r[0].float() * 64 ** -0.5) @ r[1].float().transpose(-1, -2)).softmax(-1)
    ref = (att @ r[2].float()).transpose(1, 2).reshape(B * T, C)
    assert (out.float() - ref).abs().max().item() <= 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize("C", [384, 768, 1024, 68])
def test_layernorm(gpu, C):
    from scenedino_amd import _lib
    g = torch.Generator().manual_seed(C)
    x = (3 * torch.randn(333, C, generator=g) + 1).to(gpu)
    w = (1 + 0.1 * torch.randn(C, generator=g)).to(gpu)
    b = (0.1 * torch.randn(C, generator=g)).to(gpu)
    ref = F.layer_norm(x, (C,), w, b, 1e-6)
    ob = torch.empty(333, C, device=gpu, dtype=torch.bfloat16)
    _lib.layernorm(x, w, b, 1e-6, ob)
    assert (ob.float() - ref).abs().max().item() <= 2e-2
    of = torch.empty(333, C, device=gpu)
    _lib.layernorm(x, w, b, 1e-6, of)
    assert (of - ref).abs().max().item() <= 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("C,H,T,B", [(384, 6, 481, 1), (768, 12, 481, 1), (768, 12, 77, 2)])
def test_ln_gemm_equals_layernorm_then_gemm(gpu, C, H, T, B):
    """sd_ln_gemm (norm fused into the qkv / fc1 GEMM prologue): its normalised rows are
    sd_layernorm's bf16 rows, so the products equal the two-launch path up to the GEMM's
    accumulation order -- checked against the f32 product of sd_layernorm's rows
    (|d| <= 8e-3 of the output scale, bf16 output rounding) and the qkv scatter layout."""
    from scenedino_amd import _lib
    g = torch.Generator().manual_seed(C + T)
    M = B * T
    x = (2 * torch.randn(M, C, generator=g) + 0.5).to(gpu)
    lw = (1 + 0.1 * torch.randn(C, generator=g)).to(gpu)
    lb = (0.1 * torch.randn(C, generator=g)).to(gpu)
    xn = torch.empty(M, C, device=gpu, dtype=torch.bfloat16)
    _lib.layernorm(x, lw, lb, 1e-6, xn)
    # qkv
    w = _bf(torch.randn(3 * C, C, generator=g) / math.sqrt(C)).to(gpu)
    b = (0.1 * torch.randn(3 * C, generator=g)).to(gpu)
    ref = xn.float() @ w.float().t() + b
    scale = ref.abs().max().item()
    Tp = (T + 63) // 64 * 64
    q = torch.empty(B, H, T, 64, device=gpu, dtype=torch.bfloat16)
    k = torch.zeros(B, H, Tp, 64, device=gpu, dtype=torch.bfloat16)
    vt = torch.zeros(B, H, 64, Tp, device=gpu, dtype=torch.bfloat16)
    _lib.ln_gemm(x, lw, lb, 1e-6, w, b, _lib.SD_EPI_QKV, qkv=(q, k, vt), tokens=T, heads=H)
    r = ref.view(B, T, 3, H, 64).permute(2, 0, 3, 1, 4)
    assert (q.float() - r[0]).abs().max().item() <= 8e-3 * scale
    assert (k[:, :, :T].float() - r[1]).abs().max().item() <= 8e-3 * scale
    assert (vt[..., :T].float() - r[2].transpose(-1, -2)).abs().max().item() <= 8e-3 * scale
    assert not k[:, :, T:].any() and not vt[..., T:].any()
    # fc1 + GELU
    w1 = _bf(torch.randn(4 * C, C, generator=g) / math.sqrt(C)).to(gpu)
    b1 = (0.1 * torch.randn(4 * C, generator=g)).to(gpu)
    ref1 = F.gelu(xn.float() @ w1.float().t() + b1)
    hid = torch.empty(M, 4 * C, device=gpu, dtype=torch.bfloat16)
    _lib.ln_gemm(x, lw, lb, 1e-6, w1, b1, _lib.SD_EPI_GELU, out=hid)
    assert (hid.float() - ref1).abs().max().item() <= 8e-3 * ref1.abs().max().item()


@pytest.mark.gpu
@pytest.mark.parametrize("M,hidden,ls", [(481, 1536, True), (481, 1536, False), (77, 512, True),
                                         (33, 256, False)])
def test_vit_mlp_equals_ln_gemm_then_gemm(gpu, M, hidden, ls):
    """sd_vit_mlp (norm2 + fc1 + GELU + fc2 + residual in one launch, the hidden chunks'
    partials added into x by f32 atomics) vs the two-launch path it replaces (sd_ln_gemm
    GELU, then sd_gemm SD_EPI_RESID): the same bf16 LayerNorm rows and bf16 hidden rows, so
    they differ only by f32 summation order (|d| <= 1e-4 of the update's scale); and the
    SD_EPI_RESID f32 copy (args->k) equals the updated rows."""
    from scenedino_amd import _lib
    C = 384
    g = torch.Generator().manual_seed(M + hidden)
    x0 = (2 * torch.randn(M, C, generator=g) + 0.5).to(gpu)
    lw = (1 + 0.1 * torch.randn(C, generator=g)).to(gpu)
    lb = (0.1 * torch.randn(C, generator=g)).to(gpu)
    w1 = _bf(torch.randn(hidden, C, generator=g) / math.sqrt(C)).to(gpu)
    b1 = (0.1 * torch.randn(hidden, generator=g)).to(gpu)
    w2 = _bf(torch.randn(C, hidden, generator=g) / math.sqrt(hidden)).to(gpu)
    b2 = (0.1 * torch.randn(C, generator=g)).to(gpu)
    gam = (0.5 + torch.rand(C, generator=g)).to(gpu) if ls else None
    hid = torch.empty(M, hidden, device=gpu, dtype=torch.bfloat16)
    _lib.ln_gemm(x0, lw, lb, 1e-6, w1, b1, _lib.SD_EPI_GELU, out=hid)
    ref = x0.clone()
    _lib.gemm(hid, w2, b2, _lib.SD_EPI_RESID, out=ref, gamma=gam)
    # the residual GEMM's f32 copy
    a = _bf(torch.randn(M, C, generator=g)).to(gpu)
    wa = _bf(torch.randn(C, C, generator=g) / math.sqrt(C)).to(gpu)
    xr, xc = x0.clone(), torch.full_like(x0, float("nan"))
    _lib.gemm(a, wa, b2, _lib.SD_EPI_RESID, out=xr, gamma=gam, copy_out=xc)
    assert torch.equal(xr, xc)
    x = x0.clone()
    _lib.vit_mlp(x0.clone(), x, lw, lb, 1e-6, w1, b1, w2, b2, gamma=gam)
    scale = (ref - x0).abs().max().item()
    assert (x - ref).abs().max().item() <= 1e-4 * scale + 1e-5


def _encoder_check(enc, images, tol=3e-2):
    dev = images.device
    with torch.no_grad():
        got = enc(images)
    vit = enc.model.vit.cpu()
    x = images.cpu()
    if getattr(enc, "resize", None) is not None:
        x = F.interpolate(x, size=enc.resize, mode="bilinear", align_corners=False, antialias=True)
    ref = VO.encoder_forward(vit, x, enc.model.intermediate)
    enc.to(dev)
    assert len(got) == len(ref)
    for i, (a, r) in enumerate(zip(got, ref)):
        assert a.shape == r.shape, (i, a.shape, r.shape)
        rel = ((a.double().cpu() - r.double()).norm() / r.double().norm()).item()
        assert rel <= tol, f"output {i}: rel-L2 {rel:.3g}"


@pytest.mark.gpu
def test_encoder_vit_s16_192x640_vs_oracle(gpu):
    from scenedino_amd.models.backbones.dino.vit import DINOv2Encoder
    enc = DINOv2Encoder("vit-s", (192, 640), [3, 6, 9], False, "v1_16")
    init_vit(enc.model.vit, 1)
    enc = enc.to(gpu).eval()
    img = (torch.rand(1, 3, 192, 640, generator=torch.Generator().manual_seed(2)) * 2 - 1).to(gpu)
    _encoder_check(enc, img)


@pytest.mark.gpu
def test_encoder_dinov2_b14_layerscale_resize_vs_oracle(gpu):
    from scenedino_amd.models.backbones.dino.vit import DINOv2Encoder
    enc = DINOv2Encoder("vit-b", (64, 224), [3, 6, 9], False, "v2")
    init_vit(enc.model.vit, 3)
    enc = enc.to(gpu).eval()
    img = (torch.rand(2, 3, 64, 224, generator=torch.Generator().manual_seed(4)) * 2 - 1).to(gpu)
    _encoder_check(enc, img)


@pytest.mark.gpu
def test_encoder_vit_b8_1921_tokens_two_blocks(gpu):
    from scenedino_amd.models.backbones.dino.vit import VisionTransformer, _ViT
    vit = init_vit(VisionTransformer((192, 640), 8, 768, 2, 12), 5)
    m = _ViT(vit, 8, intermediate_features=[0]).to(gpu).eval()
    img = (torch.rand(1, 3, 192, 640, generator=torch.Generator().manual_seed(6)) * 2 - 1).to(gpu)
    with torch.no_grad():
        grids, final = m.forward_grids(img)
    ref = VO.encoder_forward(vit.cpu(), img.cpu(), [0])
    for a, r in zip(grids + [final], ref):
        rel = ((a.double().cpu() - r.double()).norm() / r.double().norm()).item()
        assert rel <= 3e-2, rel


@pytest.mark.gpu
def test_encoder_layernorm_tails_bit_equal(gpu, monkeypatch):
    """DINOv2-B/14 (C = 768: separate LayerNorm launches) with the block norms written by the
    residual GEMMs' tails (SCENEDINO_AMD_LN_TAIL=1, off by default: slower) gives the same
    grids bit for bit."""
    from scenedino_amd.models.backbones.dino import vit as vm
    enc = vm.DINOv2Encoder("vit-b", (64, 224), [3, 6, 9], False, "v2")
    init_vit(enc.model.vit, 9)
    enc = enc.to(gpu).eval()
    enc.model.use_graph = False
    img = (torch.rand(2, 3, 64, 224, generator=torch.Generator().manual_seed(10)) * 2 - 1).to(gpu)
    with torch.no_grad():
        monkeypatch.setattr(vm, "LN_TAIL", False)
        ref = enc(img)
        monkeypatch.setattr(vm, "LN_TAIL", True)
        out = enc(img)
    for a, b in zip(ref, out):
        assert torch.equal(a, b)


@pytest.mark.gpu
def test_graph_replay_matches_eager(gpu):
    from scenedino_amd.models.backbones.dino.vit import DINOv2Encoder
    enc = DINOv2Encoder("vit-s", (64, 160), [3, 6, 9], False, "v1_16")
    init_vit(enc.model.vit, 7)
    enc = enc.to(gpu).eval()
    g = torch.Generator().manual_seed(8)
    imgs = [(torch.rand(1, 3, 64, 160, generator=g) * 2 - 1).to(gpu) for _ in range(3)]
    with torch.no_grad():
        enc.model.use_graph = False
        eager = [enc(x) for x in imgs]
        enc.model.use_graph = True
        graph = [enc(x) for x in imgs]  # capture on the first, replay on the others
    for e, gr in zip(eager, graph):
        for a, b in zip(e, gr):
            assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("B,gh,gw,C,l2", [(1, 24, 80, 768, False), (2, 13, 45, 96, True),
                                          (1, 3, 5, 70, True)])
def test_tokens_to_grid(gpu, B, gh, gw, C, l2):
    """sd_tokens_to_grid (class token dropped, (B, T, C) -> (B, C, gh, gw), optional double
    F.normalize as vit.py:188 + dinov2_module.py:282) against the torch view."""
    from scenedino_amd import _lib
    g = torch.Generator().manual_seed(gh * gw + C)
    T = 1 + gh * gw
    x = (3 * torch.randn(B * T, C, generator=g)).to(gpu)
    out = _lib.tokens_to_grid(x, B, T, C, 1, gh, gw, l2)
    ref = x.view(B, T, C)[:, 1:].reshape(B, gh, gw, C).permute(0, 3, 1, 2)
    if l2:
        ref = F.normalize(F.normalize(ref, dim=1), dim=1)
    assert tuple(out.shape) == (B, C, gh, gw)
    assert (out - ref).abs().max().item() <= 1e-6 * (1 if l2 else ref.abs().max().item())
