"""CPU checks of the projected-grid head packing (scenedino_amd/mlp_pack.py, 16x16x32
fragments) against dense ResnetFC math, emulating the lane-level semantics of
v_mfma_f32_16x16x32_{f16,bf16} exactly as sdhip_proj.hip feeds them:
A[i = l & 15][k = 8 (l >> 4) + e], B[k = 8 (l >> 4) + e][j = l & 15],
accumulator row 4 (l >> 4) + r, column l & 15.  No GPU needed."""
import numpy as np
import pytest
import torch

from scenedino_amd import _lib
from scenedino_amd.mlp_pack import PackedMLP, proj_pe_col

LANES = np.arange(64)
LI, GG = LANES & 15, LANES >> 4


def mfma_16x16x32(a_frag, b_frag, acc):
    """a_frag, b_frag: (64, 8); acc: (64, 4)."""
    A = np.zeros((16, 32)); Bm = np.zeros((32, 16))
    for l in range(64):
        for e in range(8):
            A[LI[l], 8 * GG[l] + e] = a_frag[l, e]
            Bm[8 * GG[l] + e, LI[l]] = b_frag[l, e]
    Dm = A @ Bm
    out = acc.copy()
    for l in range(64):
        for r in range(4):
            out[l, r] += Dm[4 * GG[l] + r, LI[l]]
    return out


def mfma_16x16x16(a_frag, b_frag, acc):
    """a_frag, b_frag: (64, 4) -- A[i = l & 15][k = 4 (l >> 4) + e]; acc: (64, 4)."""
    A = np.zeros((16, 16)); Bm = np.zeros((16, 16))
    for l in range(64):
        for e in range(4):
            A[LI[l], 4 * GG[l] + e] = a_frag[l, e]
            Bm[4 * GG[l] + e, LI[l]] = b_frag[l, e]
    Dm = A @ Bm
    out = acc.copy()
    for l in range(64):
        for r in range(4):
            out[l, r] += Dm[4 * GG[l] + r, LI[l]]
    return out


def identity_frag(which):
    f = np.zeros((64, 8))
    for l in range(64):
        for e in range(8):
            f[l, e] = 1.0 if 8 * GG[l] + e == LI[l] + 16 * which else 0.0
    return f


def code_frag(v, pc, g):
    """sd_code_frags of sdhip_render.h for one sample (v = [x, y, z~]), exact math:
    chunk 0 has 8 slots, chunk 1 (the 16x16x16 operand) 4."""
    out = np.zeros(8 if pc == 0 else 4)
    if g == 3:
        if pc == 0:
            out[:3] = v
        return out
    for e in range(len(out)):
        f, ph = 4 * pc + (e >> 1), e & 1
        out[e] = np.sin(v[g] * 1.5 * 2.0 ** f + ph * np.pi / 2)
    return out


def ref_code(v):
    freqs = 1.5 * 2.0 ** np.arange(6)
    c = [v[0], v[1], v[2]]
    for i in range(6):
        for ph in range(2):
            for d in range(3):
                c.append(np.sin(ph * np.pi / 2 + v[d] * freqs[i]))
    return np.array(c)


def test_code_slots_cover_the_reference_code_once():
    v = np.array([0.3, -0.7, 0.45])
    rc = ref_code(v)
    seen = []
    for pc in range(2):
        for g in range(4):
            vals = code_frag(v, pc, g)
            for e in range(len(vals)):
                c = proj_pe_col(pc, g, e)
                if c < 0:
                    assert vals[e] == 0
                else:
                    assert abs(vals[e] - rc[c]) < 1e-9
                    seen.append(c)
    assert sorted(seen) == list(range(39))


@pytest.mark.parametrize("D", [32, 64])
def test_projected_head_reproduces_dense_mlp(D):
    g = torch.Generator().manual_seed(7)
    C = 64
    W_in = torch.randn(128, C + 39, generator=g) * 0.1
    b_in = torch.randn(128, generator=g) * 0.1
    W_out = torch.randn(1 + D, 128, generator=g) * 0.1
    b_out = torch.randn(1 + D, generator=g) * 0.1
    X = torch.randn(16, C, generator=g).double().numpy()   # 16 samples' blended grid features
    V = (torch.rand(16, 3, generator=g) * 2 - 1).double().numpy()
    pk = PackedMLP(W_in, b_in, W_out, b_out, _lib.SD_BF16)
    f = lambda t: t.float().double().numpy()
    Wd, Wo = W_in.double().numpy(), W_out.double().numpy()
    # projected grid rows: P = W_feat X + b_in (what sd_project_grid stores per pixel)
    Pm = X @ Wd[:, :C].T + b_in.double().numpy()          # (16, 128)
    acc = [np.zeros((64, 4)) for _ in range(8)]
    I0, I1 = identity_frag(0), identity_frag(1)
    for q in range(4):                                     # 4 chunks of 32 P channels
        b = np.zeros((64, 8))
        for l in range(64):
            b[l] = Pm[LI[l], 32 * q + 8 * GG[l]: 32 * q + 8 * GG[l] + 8]
        acc[2 * q] = mfma_16x16x32(I0, b, acc[2 * q])
        acc[2 * q + 1] = mfma_16x16x32(I1, b, acc[2 * q + 1])
    wpe = f(pk.w_pe16)
    wpe0 = wpe[:8 * 64 * 8].reshape(8, 64, 8)
    wpe1 = wpe[8 * 64 * 8:].reshape(8, 64, 4)
    b0 = np.array([code_frag(V[LI[l]], 0, GG[l]) for l in range(64)])
    b1 = np.array([code_frag(V[LI[l]], 1, GG[l]) for l in range(64)])
    for t in range(8):
        acc[t] = mfma_16x16x32(wpe0[t], b0, acc[t])
        acc[t] = mfma_16x16x16(wpe1[t], b1, acc[t])
    # dense reference with the same rounded code weights (bf16 mode: f16 up to sigma, the
    # DINO head bf16 -- _lib.FIELD_DTYPE)
    assert pk.w_pe16.dtype == torch.float16 and pk.w_sig16.dtype == torch.float16
    assert pk.w_out16.dtype == torch.bfloat16
    Wpe_bf = W_in[:, C:].to(torch.float16).double().numpy()
    codes = np.array([ref_code(V[i]) for i in range(16)])
    hdense = Pm + codes @ Wpe_bf.T                         # (16, 128)
    for t in range(8):
        for l in range(64):
            for r in range(4):
                assert abs(acc[t][l, r] - hdense[LI[l], 16 * t + 4 * GG[l] + r]) < 1e-6
    # ReLU -> operand fragments, sigma and dino
    Hh = np.maximum(hdense, 0)
    Xf = np.zeros((4, 64, 8))
    for s in range(4):
        for l in range(64):
            for e in range(4):
                Xf[s, l, e] = max(acc[2 * s][l, e], 0)
                Xf[s, l, 4 + e] = max(acc[2 * s + 1][l, e], 0)
    sg = np.zeros((64, 4))
    wsig = f(pk.w_sig16)
    for s in range(4):
        sg = mfma_16x16x32(wsig[s], Xf[s], sg)
    sig_ref = Hh @ W_out[0].to(torch.float16).double().numpy()
    for l in range(64):
        for r in range(4):
            assert abs(sg[l, r] - sig_ref[LI[l]]) < 1e-6
    wo = f(pk.w_out16)
    Wo_bf = W_out[1:].to(torch.bfloat16).double().numpy()
    dino_ref = Hh @ Wo_bf.T                                # (16, D)
    for dt in range(D // 16):
        o = np.zeros((64, 4))
        for s in range(4):
            o = mfma_16x16x32(wo[dt, s], Xf[s], o)
        for l in range(64):
            for r in range(4):
                assert abs(o[l, r] - dino_ref[LI[l], 16 * dt + 4 * GG[l] + r]) < 1e-6
