"""Test infrastructure (oracle): CPU restatement of the alpha-compositing backward that
sdhip_train.hip's k_composite_bwd implements -- the gradient of nerf.py:376-405
(alphas = 1 - exp(-|delta| relu(sigma)); hard_alpha_cap; T = cumprod(1 - alpha + 1e-10);
weights = alpha T; depth / dino / rgb = sum_k weights * (z, dino, rgb)) -- written as the
division-free reverse recurrence

    dL/dalpha_k = T_k (g_k - U_k) + dL/dalphas_k,  U_{K-1} = 0,
    U_{k-1} = g_k alpha_k + (1 - alpha_k + 1e-10) U_k,
    g_k = dL/dweights_k + z_k dL/ddepth + <dL/ddino, dino_k> + <dL/drgb, rgb_k>.

tests/test_train.py pins it against torch autograd of oracle/render_oracle.composite (the
reference's own op sequence) in float64.  Only tests import this module.
"""
from __future__ import annotations

import numpy as np


def composite_bwd(z, sigma, feat, rgb, hard_alpha_cap, g_depth=None, g_feat=None, g_rgb=None,
                  g_weights=None, g_alphas=None):
    z = np.asarray(z, np.float64)
    sigma = np.asarray(sigma, np.float64)
    R, K = z.shape
    delta = np.concatenate([z[:, 1:] - z[:, :-1], np.full((R, 1), 1e10)], 1)
    e = np.exp(-np.abs(delta) * np.maximum(sigma, 0.0))
    a = 1.0 - e
    if hard_alpha_cap:
        a[:, -1] = 1.0
    g = np.zeros((R, K))
    if g_weights is not None:
        g += g_weights
    if g_depth is not None:
        g += g_depth[:, None] * z
    if g_feat is not None:
        g += np.einsum("rkf,rf->rk", feat, g_feat)
    if g_rgb is not None:
        g += np.einsum("rkc,rc->rk", rgb, g_rgb)
    T = np.ones((R, K))
    for k in range(1, K):
        T[:, k] = T[:, k - 1] * (1.0 - a[:, k - 1] + 1e-10)
    U = np.zeros(R)
    da = np.zeros((R, K))
    for k in range(K - 1, -1, -1):
        da[:, k] = T[:, k] * (g[:, k] - U)
        U = g[:, k] * a[:, k] + (1.0 - a[:, k] + 1e-10) * U
    if g_alphas is not None:
        da += g_alphas
    if hard_alpha_cap:
        da[:, -1] = 0.0
    d_sigma = np.where(sigma > 0, da * e * np.abs(delta), 0.0)
    w = a * T
    d_feat = w[..., None] * g_feat[:, None, :] if g_feat is not None else None
    d_rgb = w[..., None] * g_rgb[:, None, :] if g_rgb is not None else None
    return d_sigma, d_feat, d_rgb
