"""Pack ResnetFC(n_blocks=0) parameters into the MFMA fragment order the gfx950
kernels read (see scenedino_amd/csrc/sdhip_field.hip).

ResnetFC (scenedino/models/prediction_heads/resnetfc.py:135-203) with
n_blocks=0 computes  out = lin_out(relu(lin_in(x)))  for x = [grid features (C),
positional code (39)] (bts.py:321-328).  out[0] -> sigma (softplus), out[1:] -> DINO.

Fragment maps (32x32 MFMA, lane l, half h = l >> 5; accumulator row of register r
is (r & 3) + 8 (r >> 2) + 4 h, column l & 31):
  layer 1 A   : wpk[q][ht][l][j] = W_in'[32 ht + (l & 31)][16 q + 8 h + j]
                where W_in' holds the C grid columns, then the 39 code columns
                permuted into the kernel's slot order (3 chunks of 16, padded).
  bias/sigma  : [t][h][r] = vec[32 t + (r & 3) + 8 (r >> 2) + 4 h]
  layer 2 A   : bf16 [dt][t][s][l][j] = W_out[1 + 32 dt + (l & 31)][32 t + 16 s + 8 (j >> 2) + 4 h + (j & 3)]
                f32  [dt][t][l][r]    = W_out[1 + 32 dt + (l & 31)][32 t + (r & 3) + 8 (r >> 2) + 4 h]

Projected-grid head (16x16x32 MFMA, sdhip_proj.hip; lane l, sample/row i = l & 15,
group g = l >> 4; hidden index of operand element e in k-step s:
hid(s, g, e) = 32 s + 16 (e >> 2) + 4 g + (e & 3)):
  code A      : w_pe = [chunk 0: t][l][e < 8] ++ [chunk 1: t][l][e < 4],
                w_pe[pc][t][l][e] = W_in[16 t + (l & 15)][C + proj_pe_col(pc, g, e)]
                (chunk 1 is the 16x16x16 operand: lane l holds k = 4 g + e)
  sigma A     : w_sig[s][l][e]     = W_out[0][hid(s, g, e)]
  dino A      : w_out16[dt][s][l][e] = W_out[1 + 16 dt + (l & 15)][hid(s, g, e)]
"""
from __future__ import annotations

import functools

import numpy as np
import torch

from . import _lib

N_PE = 39
PE_CHUNKS = 3
D_HIDDEN = 128


def pe_slot_to_ref_col(pc: int, h: int, j: int) -> int:
    """Column (within the 39 code columns) feeding fragment element j of PE chunk pc,
    lane half h; -1 = zero padding.  Reference code order (positional_encoding.py:75-79):
    [x, y, z~] then for j' = 2 i + phase (i = freq, phase 0 sin / 1 cos), dims 0..2."""
    s = 8 * pc + j
    if s < 18:
        i, d = divmod(s, 3)
        return 3 + 3 * (2 * i + h) + d
    if s < 21 and h == 0:
        return s - 18
    return -1


def proj_pe_col(pc: int, g: int, e: int) -> int:
    """Code column (0..38) feeding element e of code chunk pc (0: 16x16x32 operand, 8
    slots; 1: 16x16x16 operand, 4 slots) for lane group g in the projected-grid kernels
    (sd_code_frags, sdhip_render.h); -1 = zero.  Group c < 3 carries coordinate c's
    sinusoids (slot 2 f' + ph, f = f' + 4 pc), group 3 the raw inputs.  Reference order
    (positional_encoding.py:75-79): [x, y, z~] then sin / cos at frequency f for dims 0..2."""
    if g == 3:
        return e if (pc == 0 and e < 3) else -1
    f, ph = 4 * pc + (e >> 1), e & 1
    return 3 + 6 * f + 3 * ph + g


@functools.lru_cache(maxsize=8)
def _proj_tables(C: int, D: int):
    lanes = np.arange(64)
    li, gg = lanes & 15, lanes >> 4
    e = np.arange(8)
    # chunk 0: [8 tiles][64 lanes][8 slots]; chunk 1: [8 tiles][64 lanes][4 slots], flattened
    pe_rows, pe_cols = [], []
    for pc, ne in ((0, 8), (1, 4)):
        for t in range(8):
            for l in range(64):
                for k in range(ne):
                    c = proj_pe_col(pc, l >> 4, k)
                    pe_rows.append(16 * t + (l & 15))
                    pe_cols.append(C + c if c >= 0 else -1)
    pe_rows, pe_cols = np.array(pe_rows, np.int64), np.array(pe_cols, np.int64)
    s = np.arange(4)[:, None, None]
    hid = 32 * s + 16 * (e[None, None, :] >> 2) + 4 * gg[None, :, None] + (e[None, None, :] & 3)
    hid = np.broadcast_to(hid, (4, 64, 8))
    nd = D // 16
    out_rows = np.broadcast_to(1 + 16 * np.arange(nd)[:, None, None, None] + li[None, None, :, None],
                               (nd, 4, 64, 8))
    out_cols = np.broadcast_to(hid[None], (nd, 4, 64, 8))
    to_t = lambda a: torch.from_numpy(np.array(a, copy=True))
    return {"pe_rows": to_t(pe_rows), "pe_cols": to_t(pe_cols), "sig_cols": to_t(hid),
            "out_rows": to_t(out_rows), "out_cols": to_t(out_cols)}


@functools.lru_cache(maxsize=8)
def _index_tables(C: int, D: int):
    nq = C // 16 + PE_CHUNKS
    lanes = np.arange(64)
    lo, hh = lanes & 31, lanes >> 5
    # layer-1 columns of W_in' -> original W_in column (or -1)
    kk_src = np.full(C + 16 * PE_CHUNKS, -1, dtype=np.int64)
    kk_src[:C] = np.arange(C)
    for pc in range(PE_CHUNKS):
        for h in range(2):
            for j in range(8):
                c = pe_slot_to_ref_col(pc, h, j)
                if c >= 0:
                    kk_src[C + 16 * pc + 8 * h + j] = C + c
    q = np.arange(nq)[:, None, None, None]
    ht = np.arange(4)[None, :, None, None]
    l_lo = lo[None, None, :, None]
    l_h = hh[None, None, :, None]
    j = np.arange(8)[None, None, None, :]
    rows1 = np.broadcast_to(32 * ht + l_lo, (nq, 4, 64, 8))
    cols1 = kk_src[16 * q + 8 * l_h + j]
    cols1 = np.broadcast_to(cols1, (nq, 4, 64, 8))
    # accumulator-row order for bias / sigma rows
    t = np.arange(4)[:, None, None]
    h2 = np.arange(2)[None, :, None]
    r = np.arange(16)[None, None, :]
    accrow = 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h2  # (4,2,16)
    ndt = max(D // 32, 1)
    dt = np.arange(ndt)[:, None, None, None, None]
    tt = np.arange(4)[None, :, None, None, None]
    s = np.arange(2)[None, None, :, None, None]
    l5_lo = lo[None, None, None, :, None]
    l5_h = hh[None, None, None, :, None]
    j5 = np.arange(8)[None, None, None, None, :]
    rows2b = np.broadcast_to(1 + 32 * dt + l5_lo, (ndt, 4, 2, 64, 8))
    cols2b = np.broadcast_to(32 * tt + 16 * s + 8 * (j5 >> 2) + 4 * l5_h + (j5 & 3),
                             (ndt, 4, 2, 64, 8))
    dt4 = np.arange(ndt)[:, None, None, None]
    t4 = np.arange(4)[None, :, None, None]
    l4_lo = lo[None, None, :, None]
    l4_h = hh[None, None, :, None]
    r4 = np.arange(16)[None, None, None, :]
    rows2f = np.broadcast_to(1 + 32 * dt4 + l4_lo, (ndt, 4, 64, 16))
    cols2f = np.broadcast_to(32 * t4 + (r4 & 3) + 8 * (r4 >> 2) + 4 * l4_h, (ndt, 4, 64, 16))
    to_t = lambda a: torch.from_numpy(np.array(a, copy=True))
    return {
        "rows1": to_t(rows1), "cols1": to_t(cols1), "accrow": to_t(accrow),
        "rows2b": to_t(rows2b), "cols2b": to_t(cols2b),
        "rows2f": to_t(rows2f), "cols2f": to_t(cols2f),
    }


class PackedMLP:
    """Device buffers + the ctypes ``sd_mlp`` record.  Keep the object alive while
    kernels that use it may run."""

    def __init__(self, W_in, b_in, W_out, b_out, dtype: int, empty_feature=None):
        W_in = W_in.detach().float()
        b_in = b_in.detach().float()
        W_out = W_out.detach().float()
        b_out = b_out.detach().float()
        dh, din = W_in.shape
        C = din - N_PE
        D = W_out.shape[0] - 1
        if dh != D_HIDDEN or C <= 0 or C % 64 or D % 16 or W_out.shape[1] != dh:
            raise NotImplementedError(
                f"field kernels need d_hidden=128, C%64==0, D%16==0 (got W_in {tuple(W_in.shape)}, "
                f"W_out {tuple(W_out.shape)})")
        dev = W_in.device
        ix = {k: v.to(dev) for k, v in _index_tables(C, D).items()}
        Wz = torch.cat((W_in, torch.zeros(dh, 1, device=dev)), 1)  # column din = zero pad
        cols1 = torch.where(ix["cols1"] < 0, torch.full_like(ix["cols1"], din), ix["cols1"])
        w1 = Wz[ix["rows1"], cols1]
        # operands upstream of sigma in the field dtype (f16 for both 16-bit modes), the DINO
        # output layer in the mode's dtype (RMode, csrc/sdhip_render.h)
        tdt = _lib.TORCH_DTYPE[dtype]
        fdt = _lib.TORCH_DTYPE[_lib.FIELD_DTYPE[dtype]]
        self.w_in = w1.to(fdt).contiguous()
        self.b_in_h = b_in[ix["accrow"]].contiguous()
        self.w_sig_h = W_out[0][ix["accrow"]].contiguous()
        self.b_empty_h = None
        if empty_feature is not None:  # learn_empty (bts.py:311-319): b_in + W_in[:, :C] e
            e = empty_feature.detach().to(device=dev, dtype=torch.float64)
            be = b_in.double() + W_in[:, :C].double() @ e
            self.b_empty_h = be.float()[ix["accrow"]].contiguous()
        if D % 32:  # the 32x32 grid / field kernels need D % 32 == 0 (they reject NULL)
            self.w_out = None
        elif dtype != _lib.SD_F32:
            self.w_out = W_out[ix["rows2b"], ix["cols2b"]].to(tdt).contiguous()
        else:
            self.w_out = W_out[ix["rows2f"], ix["cols2f"]].contiguous()
        self.b_dino = b_out[1:].contiguous()
        self.b_sigma = float(b_out[0].item())
        self.C, self.D, self.dtype = C, D, dtype
        self.head_rec = None
        if dtype != _lib.SD_F32 and D % 16 == 0 and D <= 512:
            px = {k: v.to(dev) for k, v in _proj_tables(C, D).items()}
            pe_cols = torch.where(px["pe_cols"] < 0, torch.full_like(px["pe_cols"], din), px["pe_cols"])
            self.w_pe16 = Wz[px["pe_rows"], pe_cols].to(fdt).contiguous()
            self.w_sig16 = W_out[0][px["sig_cols"]].to(fdt).contiguous()
            self.w_out16 = W_out[px["out_rows"], px["out_cols"]].to(tdt).contiguous()
            self.head_rec = _lib.SdHead(
                w_pe=self.w_pe16.data_ptr(), w_sig=self.w_sig16.data_ptr(),
                w_out=self.w_out16.data_ptr(), b_dino=self.b_dino.data_ptr(),
                b_sigma=self.b_sigma, D=D, dtype=dtype)
        self.rec = _lib.SdMlp(
            w_in=self.w_in.data_ptr(), b_in_h=self.b_in_h.data_ptr(),
            w_sig_h=self.w_sig_h.data_ptr(), b_sigma=self.b_sigma,
            w_out=self.w_out.data_ptr() if self.w_out is not None else None,
            b_dino=self.b_dino.data_ptr(), C=C, D=D, dtype=dtype, d_hidden=dh,
            b_empty_h=self.b_empty_h.data_ptr() if self.b_empty_h is not None else None)


def param_key(*ts):
    return tuple((t.data_ptr(), t._version, tuple(t.shape), str(t.device)) for t in ts)


# ---------------------------------------------------------------------------
# training-path MLP (csrc/sdhip_mlp.hip): 32x32x16 MFMA fragments, lane l = 32 h + r holds
# 8 consecutive k elements 8 h .. 8 h + 7 of its row (A) / column (B) r.  Operands fed from
# an accumulator tile use the permuted k order kappa(s, h, j) = 16 s + 8 (j >> 2) + 4 h + (j & 3).
# ---------------------------------------------------------------------------
_TRAIN_IDX = {}


def _train_index(d_in: int, D: int, C: int, dev):
    """Flat gather index of all four training fragment arrays into the source vector
    src = [W1 (128 x kx, row-major) | Wo (D+1 x 128: dino rows, then out_0) | 0]:
    w1f [4][KS][64][8], w2f [U][8][64][8], wtf [4][KO][64][8], wxf [C/32][8][64][8].
    Built once per shape (the optimizer changes the weights every step, not the maps)."""
    key = (d_in, D, C, str(dev))
    if key in _TRAIN_IDX:
        return _TRAIN_IDX[key]
    kx = d_in + 1
    KS, U, KO = (kx + 15) // 16, (D + 1 + 31) // 32, (D + 1 + 15) // 16
    n_w1 = D_HIDDEN * kx
    zero = n_w1 + (D + 1) * D_HIDDEN
    l = torch.arange(64).view(1, 64, 1)
    r, h = l & 31, l >> 5
    j = torch.arange(8).view(1, 1, 8)

    def lin(n):  # k = 16 s + 8 h + j
        return 16 * torch.arange(n).view(-1, 1, 1) + 8 * h + j

    def kap(n):  # permuted k of an accumulator-fed operand
        return 16 * torch.arange(n).view(-1, 1, 1) + 8 * (j >> 2) + 4 * h + (j & 3)

    parts = []
    for t in range(4):  # W1 rows (hidden), k = x column
        row, k = 32 * t + r, lin(KS)
        parts.append(torch.where(k < kx, row * kx + k, zero))
    for u in range(U):  # Wo rows (outputs), k = hidden (permuted)
        row, k = 32 * u + r, kap(8)
        parts.append(torch.where(row < D + 1, n_w1 + row * D_HIDDEN + k, zero).expand(8, 64, 8))
    for t in range(4):  # Wo^T rows (hidden), k = output
        hid, k = 32 * t + r, lin(KO)
        parts.append(torch.where(k < D + 1, n_w1 + k * D_HIDDEN + hid, zero))
    for u in range(C // 32):  # W_in^T rows (input column c), k = hidden (permuted)
        c, k = 32 * u + r, kap(8)
        parts.append((k * kx + c).expand(8, 64, 8))
    idx = torch.cat([p.reshape(-1) for p in parts]).to(dev)
    sizes = (4 * KS * 512, U * 8 * 512, 4 * KO * 512, (C // 32) * 8 * 512)
    _TRAIN_IDX[key] = (idx, sizes, (KS, U, KO))
    return _TRAIN_IDX[key]


class PackedTrainMLP:
    """Fragments of the fused training MLP (sd_mlp_train_fwd / _bwd) for ResnetFC weights
    W_in (128, d_in), b_in, W_out (1 + D, 128), b_out; dtype SD_F16 / SD_BF16.  One gather
    of the flattened weights through a cached index (_train_index) per weight version."""

    def __init__(self, W_in, b_in, W_out, b_out, dtype: int, C: int):
        dev = W_in.device
        dh, d_in = W_in.shape
        D = W_out.shape[0] - 1
        if dh != D_HIDDEN or D > 64 or C % 32:
            raise NotImplementedError("fused training MLP: d_hidden 128, D <= 64, C % 32 == 0")
        idx, sizes, (KS, U, KO) = _train_index(d_in, D, C, dev)
        with torch.no_grad():
            src = torch.cat((torch.cat((W_in, b_in[:, None]), 1).reshape(-1),
                             W_out[1:].reshape(-1), W_out[:1].reshape(-1),
                             torch.zeros(1, device=dev, dtype=W_in.dtype)))
            frags = src.float()[idx].to(_lib.TORCH_DTYPE[dtype])
        a, b, c, d = torch.split(frags, sizes)
        self.w1f = a.view(4, KS, 64, 8)
        self.w2f = b.view(U, 8, 64, 8)
        self.wtf = c.view(4, KO, 64, 8)
        self.wxf = d.view(C // 32, 8, 64, 8)
        self.b_out = b_out.detach().float().contiguous()
        self.D, self.C, self.kx, self.dtype = D, C, d_in + 1, dtype
