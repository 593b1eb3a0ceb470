"""PatchSalienceDownsampler (downsampler.py:31-98) on the
sd_salience_fwd / sd_salience_bwd kernels vs the reference module's own forward and autograd
(tests/golden/salience_downsampler.npz, make_golden.py fx_salience_downsampler).
Tolerance (fp32, different summation order): |d| <= 1e-6 + 1e-5 |ref| for the outputs and
maps, rel-L2 <= 1e-5 for the gradients (the conv bias gradient, a cancelling sum: 1e-5 of the
summed |patch-bias gradient| terms)."""
import numpy as np
import pytest
import torch

from _helpers import load, rel_l2
from scenedino_amd.models.backbones.dino.downsampler import PatchSalienceDownsampler

CASES = {"p8c64": (8, 64), "p14c768": (14, 768)}


def _module(d, name, dev):
    ps, c = CASES[name]
    m = PatchSalienceDownsampler(c, ps, True)
    with torch.no_grad():
        m.conv.weight.copy_(torch.from_numpy(d[f"{name}_conv_w"]))
        m.conv.bias.copy_(torch.from_numpy(d[f"{name}_conv_b"]))
        m.patch_weight.copy_(torch.from_numpy(d[f"{name}_pw"]))
        m.patch_bias.copy_(torch.from_numpy(d[f"{name}_pb"]))
    return m.to(dev)


def test_parameters_match_reference_layout():
    d = load("salience_downsampler.npz")
    for name, (ps, c) in CASES.items():
        m = PatchSalienceDownsampler(c, ps, True)
        assert [k for k in m.state_dict()] == ["patch_weight", "patch_bias", "conv.weight", "conv.bias"]
        for k, fx in (("conv.weight", "conv_w"), ("conv.bias", "conv_b"), ("patch_weight", "pw"),
                      ("patch_bias", "pb")):
            assert tuple(m.state_dict()[k].shape) == d[f"{name}_{fx}"].shape


def _close(a, ref, what):
    a = a.detach().double().cpu()
    ref = torch.as_tensor(np.asarray(ref)).double().reshape(a.shape)
    err = (a - ref).abs()
    assert bool((err <= 1e-6 + 1e-5 * ref.abs()).all()), f"{what}: max err {float(err.max()):.3g}"


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_forward_backward_vs_reference(name):
    d = load("salience_downsampler.npz")
    m = _module(d, name, "cuda")
    x = torch.from_numpy(d[f"{name}_x"]).cuda().requires_grad_(True)
    res, sal, wmap, pwb = m(x, "patch")
    _close(res, d[f"{name}_out"], "features")
    _close(sal, d[f"{name}_sal"], "salience")
    _close(wmap, d[f"{name}_wmap"], "weights")
    assert pwb.shape == (CASES[name][0], 2 * CASES[name][0])
    (res * torch.from_numpy(d[f"{name}_gout"]).cuda()).sum().backward()
    assert rel_l2(x.grad, d[f"{name}_gx"]) <= 1e-5
    assert rel_l2(m.conv.weight.grad, d[f"{name}_gconv_w"]) <= 1e-5
    # the bias gradient is a sum of softmax-gradient terms that cancel (sum_i g_l_i = 0 per
    # patch, patch_weight ~ 1): held to 1e-5 of the magnitude of those terms, not of itself
    scale = float(np.abs(d[f"{name}_gpb"]).sum())
    assert abs(float(m.conv.bias.grad) - float(d[f"{name}_gconv_b"][0])) <= 1e-5 * scale
    assert rel_l2(m.patch_weight.grad, d[f"{name}_gpw"]) <= 1e-5
    assert rel_l2(m.patch_bias.grad, d[f"{name}_gpb"]) <= 1e-5


@pytest.mark.gpu
def test_map_gradients_and_image_mode():
    """Gradients through the salience / weight maps (visualisation outputs) against torch
    autograd of the same formula, and mode="image" (:62-79) against patch mode on the
    re-tiled input."""
    torch.manual_seed(3)
    m = PatchSalienceDownsampler(32, 4, True).cuda()
    x = torch.randn(1, 2, 8, 12, 1, 32, device="cuda", requires_grad=True)
    res, sal, wmap, _ = m(x, "image")
    g1, g2, g3 = (torch.randn_like(t) for t in (res, sal, wmap))
    ((res * g1).sum() + (sal * g2).sum() + (wmap * g3).sum()).backward()
    xr = x.detach().clone().requires_grad_(True)
    w, b = m.conv.weight.detach().view(-1), m.conv.bias.detach()
    pw, pb = m.patch_weight.detach(), m.patch_bias.detach()
    p = xr.reshape(1, 2, 2, 4, 3, 4, 1, 32).swapaxes(3, 4).flatten(1, 3)  # (1, 12, 4, 4, 1, 32)
    s = (p[..., 0, :] @ w) + b
    a = torch.softmax((s * pw + pb).reshape(-1, 16), 1).reshape(1, 12, 4, 4, 1, 1)
    y = (a * p).sum((2, 3))
    y = y / torch.linalg.norm(y, dim=-1, keepdim=True)
    sal_r = s.reshape(1, 2, 2, 3, 4, 4).swapaxes(3, 4).reshape(1, 2, 8, 12, 1, 1)
    a_r = a.reshape(1, 2, 2, 3, 4, 4).swapaxes(3, 4).reshape(1, 2, 8, 12, 1, 1)
    assert rel_l2(res, y.reshape(res.shape)) < 1e-5
    assert rel_l2(sal, sal_r) < 1e-5 and rel_l2(wmap, a_r) < 1e-5
    ((y.reshape(res.shape) * g1).sum() + (sal_r * g2).sum() + (a_r * g3).sum()).backward()
    assert rel_l2(x.grad, xr.grad) < 1e-5
