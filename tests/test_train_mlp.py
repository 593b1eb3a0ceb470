"""Fused training MLP (csrc/sdhip_mlp.hip; resnetfc.py:135-203 under autocast, SURVEY
§8(f) rank 1): fragment maps on CPU (unpacked back to the weights), then the kernels vs the
reference op sequence (nn.Linear pair under torch.autocast, softplus) on the GPU.
Tolerances: outputs rel-L2 <= 1e-2, gradients rel-L2 <= 2e-2 (16-bit operands, as the
autocast reference)."""
import pytest
import torch
import torch.nn.functional as F

from _helpers import rel_l2
from scenedino_amd import _lib
from scenedino_amd.mlp_pack import PackedTrainMLP


def _weights(seed, d_in=295, D=64):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(128, d_in, generator=g) * 0.08, torch.randn(128, generator=g) * 0.1,
            torch.randn(1 + D, 128, generator=g) * 0.1, torch.randn(1 + D, generator=g) * 0.1)


def _kap(s, h, j):
    return 16 * s + 8 * (j >> 2) + 4 * h + (j & 3)


def test_fragment_maps_unpack_to_the_weights():
    W_in, b_in, W_out, b_out = _weights(1)
    p = PackedTrainMLP(W_in, b_in, W_out, b_out, _lib.SD_F16, 256)
    W1 = torch.cat((W_in, b_in[:, None]), 1)
    Wo = torch.cat((W_out[1:], W_out[:1]), 0)  # dino rows, then out_0
    got1 = torch.zeros(128, 19 * 16)
    got2 = torch.zeros(96, 128)
    gott = torch.zeros(128, 80)
    gotx = torch.zeros(256, 128)
    for l in range(64):
        r, h = l & 31, l >> 5
        for j in range(8):
            for t in range(4):
                for s in range(19):
                    got1[32 * t + r, 16 * s + 8 * h + j] = p.w1f[t, s, l, j].float()
                for s in range(5):
                    gott[32 * t + r, 16 * s + 8 * h + j] = p.wtf[t, s, l, j].float()
            for s in range(8):
                for u in range(3):
                    got2[32 * u + r, _kap(s, h, j)] = p.w2f[u, s, l, j].float()
                for u in range(8):
                    gotx[32 * u + r, _kap(s, h, j)] = p.wxf[u, s, l, j].float()
    f16 = lambda t: t.half().float()
    assert torch.equal(got1[:, :296], f16(W1)) and not got1[:, 296:].any()
    assert torch.equal(got2[:65], f16(Wo)) and not got2[65:].any()
    assert torch.equal(gott[:, :65], f16(Wo.t())) and not gott[:, 65:].any()
    assert torch.equal(gotx, f16(W_in[:, :256].t()))


@pytest.mark.gpu
@pytest.mark.parametrize("N", [262144, 1000, 37])
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
def test_fused_mlp_vs_autocast_linear(N, dt):
    from scenedino_amd.autograd import FieldMLPFused
    dev = "cuda"
    W_in, b_in, W_out, b_out = (t.to(dev) for t in _weights(2))
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(N, 296, device=dev, generator=g)
    x[:, 295] = 1.0
    x = x.to(dt)
    ps = [t.clone().requires_grad_(True) for t in (W_in, b_in, W_out, b_out)]
    xr = x.clone().requires_grad_(True)
    sig, dino = FieldMLPFused.apply(xr, *ps, 256)
    gs = torch.randn(N, device=dev, generator=g)
    gd = torch.randn(N, 64, device=dev, generator=g)
    ((sig * gs).sum() + (dino * gd).sum()).backward()
    # reference: the nn.Linear pair under autocast (bts.py:502-541)
    qs = [t.clone().requires_grad_(True) for t in (W_in, b_in, W_out, b_out)]
    xq = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=dt):
        out = F.linear(torch.relu(F.linear(xq[:, :295], qs[0], qs[1])), qs[2], qs[3])
    sr, dr = F.softplus(out[:, 0].float()), out[:, 1:].float()
    ((sr * gs).sum() + (dr * gd).sum()).backward()
    assert rel_l2(sig, sr) <= 1e-2 and rel_l2(dino, dr) <= 1e-2
    assert rel_l2(xr.grad[:, :256].float(), xq.grad[:, :256].float()) <= 2e-2
    assert not xr.grad[:, 256:].any()
    for a, b, name in zip(ps, qs, ("W_in", "b_in", "W_out", "b_out")):
        assert rel_l2(a.grad, b.grad) <= 2e-2, name


@pytest.mark.gpu
@pytest.mark.parametrize("N,Ma,Nb,lda,ldb", [(262144, 128, 296, 128, 296), (262144, 72, 136, 72, 136),
                                            (1000, 128, 296, 136, 304), (37, 72, 136, 72, 136)])
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
def test_wgrad_kernel_vs_matmul(N, Ma, Nb, lda, ldb, dt):
    """sd_wgrad (the training MLP's weight gradients, A^T B over the points) vs an f64
    matmul of the same 16-bit operands: rel-L2 <= 1e-5 (f32 accumulation order only)."""
    g = torch.Generator(device="cuda").manual_seed(N + Ma)
    a = torch.randn(N, lda, device="cuda", generator=g).to(dt)
    b = torch.randn(N, ldb, device="cuda", generator=g).to(dt)
    got = _lib.wgrad(a, b, Ma, Nb)
    ref = a[:, :Ma].double().t() @ b[:, :Nb].double()
    assert rel_l2(got, ref) <= 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("N,ldx,kx,nparts", [(262144, 296, 296, None), (1000, 304, 296, None),
                                             (37, 296, 296, None), (4133, 320, 320, 7),
                                             (64, 128, 104, 256), (0, 296, 296, None)])
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
def test_mlp_wgrad_fused_vs_matmul(N, ldx, kx, nparts, dt):
    """sd_mlp_train_wgrad (dW1 = dH^T X and dW_o = dY^T [H | 1] in one LDS-DMA pass, the
    parameter layout out) vs f64 matmuls of the same 16-bit rows: rel-L2 <= 1e-5 (f32
    accumulation order only).  Partial last chunk (N % 32), more workgroups than chunks,
    padded rows (ldx > kx), N = 0.  NaN rows past the used columns / past N must not leak."""
    D = 64
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(N + kx)
    # one allocation with NaN after the N rows: DMA reads past N would poison the sums
    buf = lambda n, w: torch.full((n + 64, w), float("nan"), device=dev, dtype=dt)
    x, dh, dy, h = buf(N, ldx), buf(N, 128), buf(N, 72), buf(N, 136)
    x[:N] = torch.randn(N, ldx, device=dev, generator=g).to(dt)
    dh[:N] = torch.randn(N, 128, device=dev, generator=g).to(dt)
    dy[:N] = 0
    dy[:N, :D + 1] = torch.randn(N, D + 1, device=dev, generator=g).to(dt)
    h[:N] = 0
    h[:N, :128] = torch.randn(N, 128, device=dev, generator=g).to(dt)
    h[:N, 128] = 1
    dw_in, db_in, dw_out, db_out = _lib.mlp_train_wgrad(x[:N], dh[:N], dy[:N], h[:N], kx, D,
                                                        nparts=nparts)
    if N == 0:
        assert not dw_in.any() and not db_in.any() and not dw_out.any() and not db_out.any()
        return
    X, dH, dY, H = (t[:N].double() for t in (x, dh, dy, h))
    dW1 = dH.t() @ X[:, :kx]
    dWo = dY[:, :D + 1].t() @ H[:, :129]
    order = [D] + list(range(D))  # lin_out rows: out_0, then dino
    assert rel_l2(dw_in, dW1[:, :kx - 1]) <= 1e-5 and rel_l2(db_in, dW1[:, kx - 1]) <= 1e-5
    assert rel_l2(dw_out, dWo[order, :128]) <= 1e-5 and rel_l2(db_out, dWo[order, 128]) <= 1e-5
