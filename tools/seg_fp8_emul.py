"""Diagnostic: label agreement of the folded SSCBench head (k_seg_head's algebra)
with the M = Wn1 W2 and Wn2 products on e4m3 operands under block-scaled quantisation --
the scales v_mfma_scale_f32_32x32x64_f8f6f4 applies in hardware (E8M0 = power of two, one
per 32-element K block of each A row and each B column) -- against the reference's labels
(tests/golden/seg_head.npz).  Everything else as the bf16 kernel (h, L, Gram norm in bf16 /
hi + lo, f32 accumulate)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
d = np.load(os.path.join(ROOT, "tests", "golden", "seg_head.npz"))


def e4m3(v):
    return v.float().to(torch.float8_e4m3fn).double()


def bq(X, block=32, mode="block"):
    """Quantise X (rows, K) to e4m3 with power-of-two scales: 'tensor' (one), 'row' (one
    per row), 'block' (one per row and 32-wide K block).  Largest |value| -> [256, 448]."""
    X = X.double()
    if mode == "none":
        return X
    if mode == "tensor":
        m = X.abs().max().clamp_min(1e-30)
        s = 2.0 ** torch.floor(torch.log2(448.0 / m))
        return e4m3(X * s) / s
    R, K = X.shape
    Xb = X.view(R, K // block, block) if mode == "block" else X.view(R, 1, K)
    m = Xb.abs().amax(-1, keepdim=True).clamp_min(1e-30)
    s = 2.0 ** torch.floor(torch.log2(448.0 / m))
    return (e4m3(Xb * s) / s).view(R, K)


def run(t, mM="none", mWn2="none", mh="none", mu="none", bf=True):
    g = lambda k: torch.as_tensor(d[k + t]).double()
    W1, b1, W2, b2 = g("W1"), g("b1"), g("W2"), g("b2")
    Wl, bl, Wn1, bn1 = g("Wl").reshape(64, -1), g("bl"), g("Wn1").reshape(W2.shape[0], -1), g("bn1")
    Wn2, bn2, C = g("Wn2").reshape(64, -1), g("bn2"), g("centres")
    assign = torch.as_tensor(d["assign" + t]).long()
    x = g("x")
    BF = (lambda v: v.float().to(torch.bfloat16).double()) if bf else (lambda v: v)
    h = BF(torch.relu(x @ BF(W1).t() + b1))                      # (P, 128) bf16 operand
    e = h @ W2.t() + b2
    n = e.norm(dim=1, keepdim=True).clamp_min(1e-12)
    M, L = Wn1 @ W2, Wl @ W2
    Mq = bq(M, mode=mM) if mM != "none" else BF(M)
    hq = bq(h, mode=mh) if mh != "none" else h
    u = torch.relu(hq @ Mq.t() + (Wn1 @ b2) + n * bn1)
    Wn2q = bq(Wn2, mode=mWn2) if mWn2 != "none" else BF(Wn2)
    uq = bq(u, mode=mu) if mu != "none" else BF(u)
    s = h @ BF(L).t() + Wl @ b2 + n * (bl + bn2) + uq @ Wn2q.t()
    cn = C / C.norm(dim=1, keepdim=True)
    scores = s @ cn.t()
    lab = assign[scores.argmax(1)]
    ref = torch.as_tensor(d["labels" + t]).long()
    rs = torch.as_tensor(d["scores" + t]).double() if ("scores" + t) in d else None
    agree = float((lab == ref).double().mean())
    if rs is not None:
        top2 = rs.topk(2, dim=1).values
        marg = (top2[:, 0] - top2[:, 1]) > 2e-2
        amarg = float((lab[marg] == ref[marg]).double().mean())
    else:
        amarg = float("nan")
    return agree, amarg


if __name__ == "__main__":
    print("keys:", [k for k in d.files if k.endswith("_768")][:20])
    schemes = [
        ("bf16 (the kernel)", {}),
        ("M e4m3 per tensor, h per tensor", dict(mM="tensor", mh="tensor")),
        ("M e4m3 per row, h per point", dict(mM="row", mh="row")),
        ("M e4m3 32-blocks, h 32-blocks", dict(mM="block", mh="block")),
        ("Wn2 e4m3 per tensor, u per tensor", dict(mWn2="tensor", mu="tensor")),
        ("Wn2 e4m3 32-blocks, u 32-blocks", dict(mWn2="block", mu="block")),
        ("M + Wn2 e4m3 32-blocks (h, u blocks)", dict(mM="block", mh="block", mWn2="block", mu="block")),
        ("M + Wn2 e4m3 per row (h, u per point)", dict(mM="row", mh="row", mWn2="row", mu="row")),
    ]
    for t in ("_768", "_384"):
        for name, kw in schemes:
            a, am = run(t, **kw)
            print(f"d_full {t[1:]:>4s}  {name:42s} labels {100 * a:6.2f} %   margin>2e-2 {100 * am:6.2f} %")
