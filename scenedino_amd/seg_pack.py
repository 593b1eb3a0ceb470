"""Pack MlpDimReduction + SemanticHead("stego_kmeans") parameters into the folded,
MFMA-fragment-ordered record ``sd_seg_head`` that k_seg_head (csrc/sdhip_seg.hip) reads.

Reference modules: MlpDimReduction (scenedino/models/backbones/dino/dim_reduction.py:15-25),
StegoClusterHead (scenedino/downstream_head/semantic_head.py:285-305), KMeansParamHead
(semantic_head.py:308-373).

Folding (exact algebra, done once here in fp64):
    L  = Wl  @ W2   (d_code x d_latent)      bl_f = Wl  @ b2
    M  = Wn1 @ W2   (d_full x d_latent)      bm   = Wn1 @ b2
    bo = bl + bn2
    G  = W2^T W2    (d_latent x d_latent)    g2 = 2 W2^T b2,  b2sq = |b2|^2
(|W2 h + b2|^2 = h^T G h + g2.h + b2sq: the norm without the d_full x d_latent product;
G rides as bf16 hi + lo fragments so the quadratic form does not lose the cancellation
between W2 h and b2 to G's rounding)
where W2, b2 = linear_out; Wl, bl = linear_path[0]; Wn1, bn1 = nonlinear_path[0];
Wn2, bn2 = nonlinear_path[2] (1x1 convolutions viewed as matrices).

Fragment maps (v_mfma_f32_32x32x16_bf16; lane l, r = l & 31, h = l >> 5, element j;
accumulator register i of lane half h holds row (i & 3) + 8 (i >> 2) + 4 h):
  natural k   : A[t][s][l][j]  = W[32 t + r][16 s + 8 h + j]                 (W1: input = x)
  permuted k  : A[t][q][l][j]  = W[32 t + r][perm(q, h, j)],
                perm(q, h, j)  = 32 (q >> 1) + 16 (q & 1) + 8 (j >> 2) + 4 h + (j & 3)
                (inputs that are accumulator tiles converted in place: W2, L, M, Wn2)
  row vectors : v[t][h][i]     = vec[32 t + (i & 3) + 8 (i >> 2) + 4 h]
  centres     : c[k][rt][h][i] = C_norm[k][32 rt + (i & 3) + 8 (i >> 2) + 4 h]  (f32, emulation)
  wc (record) : the centres as permuted-k A fragments, hi and lo bf16 halves per 32-row tile
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _lib


def _accrow(n_tiles: int, device):
    t = torch.arange(n_tiles, device=device).view(-1, 1, 1)
    h = torch.arange(2, device=device).view(1, -1, 1)
    i = torch.arange(16, device=device).view(1, 1, -1)
    return 32 * t + (i & 3) + 8 * (i >> 2) + 4 * h  # (n_tiles, 2, 16)


def _frag_natural(W: torch.Tensor):
    """(rows, cols) -> [rows/32][cols/16][64][8]"""
    R, Ccols = W.shape
    dev = W.device
    t = torch.arange(R // 32, device=dev).view(-1, 1, 1, 1)
    s = torch.arange(Ccols // 16, device=dev).view(1, -1, 1, 1)
    l = torch.arange(64, device=dev).view(1, 1, -1, 1)
    j = torch.arange(8, device=dev).view(1, 1, 1, -1)
    rows = 32 * t + (l & 31)
    cols = 16 * s + 8 * (l >> 5) + j
    rows, cols = torch.broadcast_tensors(rows, cols)
    return W[rows, cols]


def _frag_permuted(W: torch.Tensor):
    """(rows, cols) -> [rows/32][cols/16][64][8] with the accumulator-as-operand k order."""
    R, Ccols = W.shape
    dev = W.device
    t = torch.arange(R // 32, device=dev).view(-1, 1, 1, 1)
    q = torch.arange(Ccols // 16, device=dev).view(1, -1, 1, 1)
    l = torch.arange(64, device=dev).view(1, 1, -1, 1)
    j = torch.arange(8, device=dev).view(1, 1, 1, -1)
    rows = 32 * t + (l & 31)
    cols = 32 * (q >> 1) + 16 * (q & 1) + 8 * (j >> 2) + 4 * (l >> 5) + (j & 3)
    rows, cols = torch.broadcast_tensors(rows, cols)
    return W[rows, cols]


def _accrow16(n_tiles: int, device):
    """Row vectors of the 16x16x32 layout: register i of lane group g holds row 4 g + i."""
    t = torch.arange(n_tiles, device=device).view(-1, 1, 1)
    g = torch.arange(4, device=device).view(1, -1, 1)
    i = torch.arange(4, device=device).view(1, 1, -1)
    return 16 * t + 4 * g + i  # (n_tiles, 4, 4)


def _frag16(W: torch.Tensor, permuted: bool):
    """(rows, cols) -> [rows/16][cols/32][64][8]: A operands of v_mfma_f32_16x16x32_bf16
    (lane l holds A[l & 15][8 (l >> 4) + j]).  permuted: k-step q, element j of lane group
    g = l >> 4 <- column 32 q + 16 (j >> 2) + 4 g + (j & 3), the rows an accumulator pair
    (row tiles 2 q, 2 q + 1) holds in the registers the kernel turns into the B operand."""
    R, Ccols = W.shape
    dev = W.device
    t = torch.arange(R // 16, device=dev).view(-1, 1, 1, 1)
    q = torch.arange(Ccols // 32, device=dev).view(1, -1, 1, 1)
    l = torch.arange(64, device=dev).view(1, 1, -1, 1)
    j = torch.arange(8, device=dev).view(1, 1, 1, -1)
    rows = 16 * t + (l & 15)
    if permuted:
        cols = 32 * q + 16 * (j >> 2) + 4 * (l >> 4) + (j & 3)
    else:
        cols = 32 * q + 8 * (l >> 4) + j
    rows, cols = torch.broadcast_tensors(rows, cols)
    return W[rows, cols]


def _frag_f8(W: torch.Tensor):
    """(rows, 128) -> [rows/32][2][64][32]: A operands of v_mfma_scale_f32_32x32x64_f8f6f4
    (lane l holds A[l & 31][32 (l >> 5) + j], byte j) in the fp8 accumulator-as-operand k
    order of k_seg_head: k-step s, byte j of lane half h <- hidden
    32 (2 s + (j >> 4)) + (jj & 3) + 8 (jj >> 2) + 4 h, jj = j & 15."""
    R, Ccols = W.shape
    dev = W.device
    t = torch.arange(R // 32, device=dev).view(-1, 1, 1, 1)
    s = torch.arange(Ccols // 64, device=dev).view(1, -1, 1, 1)
    l = torch.arange(64, device=dev).view(1, 1, -1, 1)
    j = torch.arange(32, device=dev).view(1, 1, 1, -1)
    jj = j & 15
    rows = 32 * t + (l & 31)
    cols = 32 * (2 * s + (j >> 4)) + (jj & 3) + 8 * (jj >> 2) + 4 * (l >> 5)
    rows, cols = torch.broadcast_tensors(rows, cols)
    return W[rows, cols]


def quant_e4m3(W: torch.Tensor):
    """Per-tensor power-of-two scaled OCP e4m3: (codes uint8, scale) with
    W ~= e4m3(codes) * scale and max |W| / scale in [128, 256)."""
    import math
    mx = float(W.abs().max())
    e = (math.floor(math.log2(mx)) - 7) if mx > 0 else 0
    scale = 2.0 ** e
    q = (W / scale).float().to(torch.float8_e4m3fn)
    return q.view(torch.uint8), scale


def _mat(w: torch.Tensor) -> torch.Tensor:
    """nn.Linear weight or 1x1 Conv2d weight -> (out, in) float64."""
    return w.detach().reshape(w.shape[0], -1).double()


class PackedSegHead:
    """Device buffers + the ctypes ``sd_seg_head`` record.  Keep the object alive while
    kernels that use it may run.

    dim_reduction: module with ``linear_in`` / ``linear_out`` (MlpDimReduction).
    stego_head / cluster_head: StegoClusterHead / KMeansParamHead, or None for an
    expand-only record (transform_expand)."""

    def __init__(self, dim_reduction, stego_head=None, cluster_head=None, device=None,
                 frag_dtype=torch.bfloat16, fp8: bool = False, mfma: int | None = None):
        W1 = _mat(dim_reduction.linear_in.weight)
        b1 = dim_reduction.linear_in.bias.detach().double()
        W2 = _mat(dim_reduction.linear_out.weight)
        b2 = dim_reduction.linear_out.bias.detach().double()
        dev = device if device is not None else W1.device
        W1, b1, W2, b2 = (x.to(dev) for x in (W1, b1, W2, b2))
        d_latent, d_in = W1.shape
        d_full = W2.shape[0]
        if d_in != 64 or d_latent != 128 or d_full % 32 or W2.shape[1] != d_latent:
            raise NotImplementedError(
                f"sd_seg_query needs MlpDimReduction(64 -> 128 -> d_full % 32 == 0); got "
                f"linear_in {tuple(W1.shape)}, linear_out {tuple(W2.shape)}")
        bf = frag_dtype  # bf16 for the kernel; float64 lets tests emulate the MFMA chain
        fdt = torch.float64 if frag_dtype == torch.float64 else torch.float32
        # fragment layout: 16x16x32 by default (faster); the fp8 norm's kernel
        # reads the 32x32x16 maps
        # (SCENEDINO_AMD_SEG_MFMA=32 selects the 32x32x16 record for A/B runs)
        if mfma is None:
            mfma = 32 if fp8 else int(os.environ.get("SCENEDINO_AMD_SEG_MFMA", "16"))
        self.mfma = mfma
        if self.mfma not in (16, 32) or (fp8 and self.mfma != 32):
            raise ValueError("mfma must be 16 or 32 (fp8 needs 32)")
        m16 = self.mfma == 16
        perm = (lambda W: _frag16(W, True)) if m16 else _frag_permuted
        nat = (lambda W: _frag16(W, False)) if m16 else _frag_natural
        rowv = (lambda v, n: v[_accrow16(n // 16, dev)]) if m16 else (lambda v, n: v[_accrow(n // 32, dev)])
        self.w1 = nat(W1).to(bf).contiguous()
        self.b1 = rowv(b1, d_latent).to(fdt).contiguous()
        self.w2 = perm(W2).to(bf).contiguous()
        self.b2 = rowv(b2, d_full).to(fdt).contiguous()
        self.d_in, self.d_latent, self.d_full = d_in, d_latent, d_full
        G = W2.t() @ W2
        Ghi = G.to(bf).double()
        if m16:  # tile t = row tiles 2 t, 2 t + 1: [t][(row tile) (hi, lo) (k-step)]
            gh = torch.stack([perm(Ghi), perm(G - Ghi)], 1)  # (8, 2, 4, 64, 8)
            self.wg = gh.reshape(d_latent // 32, 16, 64, 8).to(bf).contiguous()
        else:
            self.wg = torch.cat([_frag_permuted(Ghi), _frag_permuted(G - Ghi)], 1).to(bf).contiguous()
        self.g2 = rowv(2 * (W2.t() @ b2), d_latent).to(fdt).contiguous()
        self.b2sq = float(b2 @ b2)
        self.seg = stego_head is not None and cluster_head is not None
        null = None
        fields = dict(w1=self.w1.data_ptr(), b1=self.b1.data_ptr(), w2=self.w2.data_ptr(),
                      b2=self.b2.data_ptr(), wl=null, bl=null, bo=null, wm=null, bm=null,
                      bn1=null, wn2=null, centres=null, assign=null, n_clusters=0,
                      d_in=d_in, d_latent=d_latent, d_full=d_full, d_code=0,
                      wg=self.wg.data_ptr(), g2=self.g2.data_ptr(), b2sq=self.b2sq,
                      frag_layout=_lib.SD_SEG_FRAG16 if m16 else _lib.SD_SEG_FRAG32)
        if self.seg:
            lin = stego_head.linear_path[0]
            nl0, nl2 = stego_head.nonlinear_path[0], stego_head.nonlinear_path[2]
            Wl, bl = _mat(lin.weight).to(dev), lin.bias.detach().double().to(dev)
            Wn1, bn1 = _mat(nl0.weight).to(dev), nl0.bias.detach().double().to(dev)
            Wn2, bn2 = _mat(nl2.weight).to(dev), nl2.bias.detach().double().to(dev)
            d_code, d_mid = Wn2.shape
            if (Wl.shape != (d_code, d_full) or Wn1.shape != (d_mid, d_full) or d_mid != d_full
                    or d_code != 64):
                raise NotImplementedError(
                    "sd_seg_query needs StegoClusterHead(d_full -> 64, mid = d_full)")
            L = Wl @ W2
            M = Wn1 @ W2
            self.wl = perm(L).to(bf).contiguous()
            self.bl = rowv(Wl @ b2, d_code).to(fdt).contiguous()
            self.bo = rowv(bl + bn2, d_code).to(fdt).contiguous()
            self.wm = perm(M).to(bf).contiguous()
            self.bm = rowv(Wn1 @ b2, d_full).to(fdt).contiguous()
            self.bn1 = rowv(bn1, d_full).to(fdt).contiguous()
            self.wn2 = perm(Wn2).to(bf).contiguous()
            # KMeansParamHead._kmeans_cosine: F.normalize(cluster_centers, dim=1) (fp32)
            cn = F.normalize(cluster_head.cluster_centers.detach().to(fdt), dim=1).to(dev)
            n_cl = cn.shape[0]
            if cn.shape[1] != d_code or not 1 <= n_cl <= 256:
                raise NotImplementedError("cluster centres must be (1..256, 64)")
            self.centres = cn[:, _accrow(d_code // 32, dev)].contiguous()  # (k, rt, h, 16)
            # the kernel's copy: hi + lo bf16 A fragments, rows = clusters (zero-padded to
            # 32 (16) per tile), [tile][hi, lo][k-step][64][8] in the permuted k order
            ct_rows = 16 if m16 else 32
            nct = (n_cl + ct_rows - 1) // ct_rows
            cpad = torch.zeros(ct_rows * nct, d_code, dtype=torch.float64, device=dev)
            cpad[:n_cl] = cn.double()
            chi = cpad.to(bf).double()
            self.wc = torch.stack([perm(chi), perm(cpad - chi)], 1).to(bf).contiguous()
            self.assign = cluster_head.pseudo_assignment.detach().to(dev, torch.int32).contiguous()
            if self.assign.numel() != n_cl:
                raise ValueError("pseudo_assignment must have one entry per cluster")
            fields.update(wl=self.wl.data_ptr(), bl=self.bl.data_ptr(), bo=self.bo.data_ptr(),
                          wm=self.wm.data_ptr(), bm=self.bm.data_ptr(), bn1=self.bn1.data_ptr(),
                          wn2=self.wn2.data_ptr(), centres=self.wc.data_ptr(),
                          assign=self.assign.data_ptr(), n_clusters=n_cl, d_code=d_code)
            self.n_clusters, self.d_code = n_cl, d_code
        self.fp8 = bool(fp8)
        if self.fp8:
            # BASELINE configs[4] fp8 MFMA: the norm product |W2 h + b2| (the only product
            # whose fp8 rounding keeps >= 99 % label agreement on the reference fixture;
            # the M / Wn2 chain stays bf16 -- see DESIGN.md)
            codes, self.w2_f8_scale = quant_e4m3(W2)
            self.w2_f8 = _frag_f8(codes).contiguous()
            fields.update(w2_f8=self.w2_f8.data_ptr(), w2_f8_scale=self.w2_f8_scale)
        self.rec = _lib.SdSegHead(**fields)


def seg_key(*modules):
    """Cache key over every parameter / buffer of the given modules."""
    key = []
    for m in modules:
        if m is None:
            continue
        for t in list(m.parameters()) + list(m.buffers()):
            key.append((t.data_ptr(), t._version, tuple(t.shape), str(t.device)))
    return tuple(key)
