"""DPT decoder: NHWC bf16 implicit-GEMM convolutions on gfx950.

CPU: the fp32 oracle (oracle/dpt_oracle.py) against the reference's own DPTHead output
(tests/golden/dpt_head.npz); the mirror module's checkpoint names.
GPU (through the C ABI): conv3x3 (stride 1 / 2, pre-ReLU, residuals), ConvTranspose
(k = stride) shuffle, bilinear x2 against torch fp32 ops on the same bf16 operands, and the
whole head against the reference fixture.  Tolerances (written here): single layers max
|d| <= 2e-2 * max|ref| (bf16 output rounding); whole head (about 20 bf16 layers) rel-L2
<= 3e-2.
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from _helpers import load
from oracle import dpt_oracle as DO


def det_fill(module, seed):
    """Same deterministic fill as tests/golden/make_golden.py:det_fill."""
    g = torch.Generator().manual_seed(seed)
    sd = module.state_dict()
    with torch.no_grad():
        for name in sorted(sd):
            t = sd[name]
            if t.dim() > 1:
                t.copy_(torch.randn(t.shape, generator=g) / float(t[0].numel()) ** 0.5)
            else:
                t.copy_(0.05 * torch.randn(t.shape, generator=g))


def make_head():
    from scenedino_amd.models.backbones.dino.dpt_head import DPTHead
    head = DPTHead(embed_dims=384, post_process_channels=[64, 64, 128, 256], d_out=256).eval()
    det_fill(head, 70)
    return head


def test_state_dict_names():
    keys = set(make_head().state_dict())
    for k in ("reassemble_blocks.projects.0.weight", "reassemble_blocks.resize_layers.0.weight",
              "reassemble_blocks.resize_layers.3.bias", "convs.2.weight",
              "fusion_blocks.1.res_conv_unit1.conv1.weight",
              "fusion_blocks.0.res_conv_unit2.conv2.bias", "fusion_blocks.3.project.weight",
              "project.bias", "output_head.head_modules.1.weight"):
        assert k in keys, k
    assert not any(k.startswith("fusion_blocks.0.res_conv_unit1") for k in keys)


def test_oracle_matches_reference():
    d = load("dpt_head.npz")
    head = make_head()
    out = DO.dpt_forward(head, [torch.as_tensor(d[f"in{i}"]) for i in range(4)])
    ref = torch.as_tensor(d["out"].astype(np.float32))
    rel = ((out - ref).norm() / ref.norm()).item()
    assert rel < 2e-3, rel  # fixture stored in fp16


# ------------------------------------------------------------------------ GPU
@pytest.fixture(scope="module")
def gpu():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    from scenedino_amd import _lib
    _lib.load()
    return "cuda"


def _q(t):
    return t.to(torch.bfloat16).float()


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,W,Cin,Cout,stride", [(1, 12, 40, 256, 256, 1), (2, 7, 9, 64, 128, 1),
                                                    (1, 12, 40, 256, 256, 2), (1, 5, 3, 128, 64, 2)])
def test_conv3x3(gpu, B, H, W, Cin, Cout, stride):
    from scenedino_amd import _lib
    g = torch.Generator().manual_seed(H * W + Cin)
    x = torch.randn(B, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / math.sqrt(9 * Cin)
    b = 0.1 * torch.randn(Cout, generator=g)
    xq, wq = _q(x), _q(w)
    xn = x.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous().to(gpu)
    wp = w.permute(0, 2, 3, 1).reshape(Cout, -1).to(torch.bfloat16).contiguous().to(gpu)
    for relu in (False, True):
        ref = F.conv2d(F.relu(xq) if relu else xq, wq, b, stride=stride, padding=1)
        out = _lib.conv3x3(xn, wp, b.to(gpu), stride=stride, relu_in=relu)
        got = out.float().permute(0, 3, 1, 2).cpu()
        assert got.shape == ref.shape
        assert (got - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()
    if stride == 1 and Cin == Cout:
        r1 = torch.randn(B, H, W, Cout, generator=g).to(torch.bfloat16)
        r2 = torch.randn(B, H, W, Cout, generator=g).to(torch.bfloat16)
        ref = (F.conv2d(xq, wq, b, padding=1) + r1.float().permute(0, 3, 1, 2)
               + r2.float().permute(0, 3, 1, 2))
        out = _lib.conv3x3(xn, wp, b.to(gpu), res=r1.to(gpu), res2=r2.to(gpu))
        got = out.float().permute(0, 3, 1, 2).cpu()
        assert (got - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()
    ref = F.conv2d(xq, wq, b, stride=stride, padding=1)
    out = _lib.conv3x3(xn, wp, b.to(gpu), stride=stride, epi=_lib.SD_EPI_NCHW)
    assert (out.cpu() - ref).abs().max().item() <= 1e-3 * ref.abs().max().item()
    # deterministic across launches
    out2 = _lib.conv3x3(xn, wp, b.to(gpu), stride=stride, epi=_lib.SD_EPI_NCHW)
    assert torch.equal(out, out2)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [2, 4])
def test_conv_transpose_shuffle(gpu, k):
    from scenedino_amd import _lib
    from scenedino_amd.models.backbones.dino.dpt_head import _pack_convT
    g = torch.Generator().manual_seed(k)
    conv = torch.nn.ConvTranspose2d(64, 96, kernel_size=k, stride=k)
    x = torch.randn(2, 64, 5, 7, generator=g)
    ref = conv(_q(x)).detach()
    wp, bp, kk = _pack_convT(conv)
    xn = x.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous().to(gpu)
    out = _lib.linear_nhwc(xn, wp.to(gpu), bp.to(gpu), shuf=kk)
    got = out.float().permute(0, 3, 1, 2).cpu()
    ref = F.conv_transpose2d(_q(x), _q(conv.weight.detach()), conv.bias.detach(), stride=k)
    assert got.shape == ref.shape
    assert (got - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()


@pytest.mark.gpu
def test_upsample2x(gpu):
    from scenedino_amd import _lib
    x = torch.randn(2, 6, 20, 64).to(torch.bfloat16)
    out = _lib.upsample2x(x.to(gpu)).float().cpu()
    ref = F.interpolate(x.float().permute(0, 3, 1, 2), scale_factor=2, mode="bilinear",
                        align_corners=True).permute(0, 2, 3, 1)
    assert (out - ref).abs().max().item() <= 2e-2


@pytest.mark.gpu
def test_dpt_head_vs_reference(gpu):
    d = load("dpt_head.npz")
    head = make_head().to(gpu)
    with torch.no_grad():
        out = head([torch.as_tensor(d[f"in{i}"]).to(gpu) for i in range(4)])[0]
    ref = torch.as_tensor(d["out"].astype(np.float32))
    assert out.shape == ref.shape
    rel = ((out.cpu() - ref).norm() / ref.norm()).item()
    assert rel <= 3e-2, f"DPT rel-L2 {rel:.3g}"


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,W,Cin,Cout,f32", [(1, 96, 320, 256, 256, False), (1, 192, 640, 256, 256, True),
                                                (1, 192, 640, 256, 256, False), (2, 61, 250, 128, 384, True),
                                                (1, 197, 650, 256, 256, True)])
def test_conv3x3_big_tiles(gpu, B, H, W, Cin, Cout, f32, monkeypatch):
    """sdhip_conv.hip's tiles for the DPT head's 96x320 / 192x640 convolutions -- the 8 x 32
    halo tiles (default: 128 output channels per tile at 96x320, all 256 at 192x640) and the
    256-row im2col tiles (SD_CONV_BIG=b); 2 x 61 x 250 with Cout 384: ragged edge tiles,
    128-column tiles, two images' padding; 197 x 650: ragged 256-column halo tiles -- against
    torch fp32 on the same bf16 operands and against sd_gemm's k_gemm path (SD_CONV_BIG=0)."""
    from scenedino_amd import _lib
    g = torch.Generator().manual_seed(H + W + Cout)
    x = torch.randn(B, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / math.sqrt(9 * Cin)
    b = 0.1 * torch.randn(Cout, generator=g)
    xq, wq = _q(x).to(gpu), _q(w).to(gpu)
    xn = x.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous().to(gpu)
    wp = w.permute(0, 2, 3, 1).reshape(Cout, -1).to(torch.bfloat16).contiguous().to(gpu)
    epi = _lib.SD_EPI_F32 if f32 else _lib.SD_EPI_BF16
    ref = F.conv2d(xq, wq, b.to(gpu), padding=1).permute(0, 2, 3, 1)
    got = _lib.conv3x3(xn, wp, b.to(gpu), epi=epi).float()  # halo tiles where they fit
    monkeypatch.setenv("SD_CONV_BIG", "b")
    im2col = _lib.conv3x3(xn, wp, b.to(gpu), epi=epi).float()  # 256-row im2col tiles
    monkeypatch.setenv("SD_CONV_BIG", "0")
    old = _lib.conv3x3(xn, wp, b.to(gpu), epi=epi).float()
    torch.cuda.synchronize()
    scale = ref.abs().max().item()
    tol = (1e-3 if f32 else 2e-2) * scale  # f32 out: fp32 accumulation order only
    for t in (got, im2col):
        assert (t - ref).abs().max().item() <= tol
        assert (t - old).abs().max().item() <= tol
        assert torch.isfinite(t).all()


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,W,Cin,Cout,k", [(1, 96, 320, 256, 256, 2), (1, 96, 320, 256, 256, None),
                                              (2, 37, 211, 128, 128, 2)])
def test_linear_big_tiles(gpu, B, H, W, Cin, Cout, k, monkeypatch):
    """Dense-A forms of sdhip_conv.hip's 256-row tiles: the output head's ConvTranspose2d(2, 2)
    at 96x320 (sub-pixel scatter epilogue), a 1x1 convolution, and a ragged two-image
    transposed convolution, against torch fp32 and sd_gemm's k_gemm path (SD_CONV_BIG=0)."""
    from scenedino_amd import _lib
    from scenedino_amd.models.backbones.dino.dpt_head import _pack_conv1, _pack_convT
    g = torch.Generator().manual_seed(H * W + Cout)
    x = torch.randn(B, Cin, H, W, generator=g)
    if k:
        conv = torch.nn.ConvTranspose2d(Cin, Cout, kernel_size=k, stride=k)
        wp, bp, kk = _pack_convT(conv)
        ref = F.conv_transpose2d(_q(x).to(gpu), _q(conv.weight.detach()).to(gpu),
                                 conv.bias.detach().to(gpu), stride=k)
    else:
        conv = torch.nn.Conv2d(Cin, Cout, kernel_size=1)
        (wp, bp), kk = _pack_conv1(conv), None
        ref = F.conv2d(_q(x).to(gpu), _q(conv.weight.detach()).to(gpu), conv.bias.detach().to(gpu))
    xn = x.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous().to(gpu)
    got = _lib.linear_nhwc(xn, wp.to(gpu), bp.to(gpu), shuf=kk).float().permute(0, 3, 1, 2)
    monkeypatch.setenv("SD_CONV_BIG", "0")
    old = _lib.linear_nhwc(xn, wp.to(gpu), bp.to(gpu), shuf=kk).float().permute(0, 3, 1, 2)
    torch.cuda.synchronize()
    assert got.shape == ref.shape
    tol = 2e-2 * ref.abs().max().item()
    assert (got - ref).abs().max().item() <= tol
    assert (got - old).abs().max().item() <= tol


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,W,C", [(1, 48, 160, 256), (2, 61, 130, 128)])
def test_conv3x3_big_tiles_residual_unit(gpu, B, H, W, C, monkeypatch):
    """The residual conv units' convolutions on sdhip_conv.hip's 128-row im2col tiles
    (48x160: 240 tiles of 128 x 64; the default and SD_CONV_BIG=b agree here): pre-activation
    ReLU, the two bf16 residuals added
    before the output rounding (dpt_head.py PreActResidualConvUnit / FeatureFusionBlock),
    against torch fp32 and the k_gemm path (SD_CONV_BIG=0)."""
    from scenedino_amd import _lib
    g = torch.Generator().manual_seed(H * W + C)
    x = torch.randn(B, C, H, W, generator=g)
    w = torch.randn(C, C, 3, 3, generator=g) / math.sqrt(9 * C)
    b = 0.1 * torch.randn(C, generator=g)
    r1 = torch.randn(B, H, W, C, generator=g).to(torch.bfloat16)
    r2 = torch.randn(B, H, W, C, generator=g).to(torch.bfloat16)
    xq, wq = _q(x).to(gpu), _q(w).to(gpu)
    xn = x.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous().to(gpu)
    wp = w.permute(0, 2, 3, 1).reshape(C, -1).to(torch.bfloat16).contiguous().to(gpu)
    r1g, r2g = r1.to(gpu), r2.to(gpu)
    for relu, res in ((True, False), (True, True), (False, True)):
        ref = F.conv2d(F.relu(xq) if relu else xq, wq, b.to(gpu), padding=1).permute(0, 2, 3, 1)
        if res:
            ref = ref + r1g.float() + r2g.float()
        kw = dict(relu_in=relu, res=r1g if res else None, res2=r2g if res else None)
        monkeypatch.delenv("SD_CONV_BIG", raising=False)
        got = _lib.conv3x3(xn, wp, b.to(gpu), **kw).float()  # halo tiles
        monkeypatch.setenv("SD_CONV_BIG", "b")
        im2col = _lib.conv3x3(xn, wp, b.to(gpu), **kw).float()  # 128-row im2col tiles
        monkeypatch.setenv("SD_CONV_BIG", "0")
        old = _lib.conv3x3(xn, wp, b.to(gpu), **kw).float()
        torch.cuda.synchronize()
        tol = 2e-2 * ref.abs().max().item()
        for t in (got, im2col):
            assert (t - ref).abs().max().item() <= tol, (relu, res)
            assert (t - old).abs().max().item() <= tol, (relu, res)
