"""seg_oracle -- TEST INFRASTRUCTURE ONLY (the checker, never shipped).

Pure-PyTorch CPU fp32 restatement of the SSCBench voxel-query head, written from the
reference's behaviour (citations are /root/reference file:line).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import it.  Pinned by
tests/golden/seg_head.npz (the reference's own MlpDimReduction / SemanticHead run on
CPU, tests/golden/make_golden.py) and tests/golden/voxel_points.json.

Unlike the gfx950 kernel it does NOT fold the products: it evaluates the reference's
op sequence (768 x 768 stego layer included).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def transform_expand(x, W1, b1, W2, b2):
    """MlpDimReduction.transform_expand (dim_reduction.py:22-25)."""
    return F.normalize(F.linear(torch.relu(F.linear(x, W1, b1)), W2, b2), dim=-1)


def stego(f, Wl, bl, Wn1, bn1, Wn2, bn2):
    """StegoClusterHead.forward (semantic_head.py:302-305) on (..., d) features: the 1x1
    convolutions are linear maps over the channel dim; dropout is the identity in eval."""
    lin = F.linear(f, Wl, bl)
    nl = F.linear(torch.relu(F.linear(f, Wn1, bn1)), Wn2, bn2)
    return F.normalize(lin + nl, dim=-1, eps=1e-10)


def kmeans_scores(s, centres):
    """KMeansParamHead._kmeans_cosine inner products (semantic_head.py:361-366)."""
    return F.normalize(s, dim=1) @ F.normalize(centres, dim=1).t()


def seg_head(x, p):
    """x (P, 64) DINO codes; p: dict of float32 parameters (W1, b1, W2, b2, Wl, bl, Wn1,
    bn1, Wn2, bn2, centres, assign).  Returns dino_full (P, d_full), scores (P, n_cl),
    labels (P,) int64 = pseudo_assignment[argmax] (semantic_head.py:107-111,349-359)."""
    full = transform_expand(x, p["W1"], p["b1"], p["W2"], p["b2"])
    f = F.normalize(full, dim=-1, eps=1e-10)  # SemanticHead.forward's _norm
    s = stego(f, p["Wl"], p["bl"], p["Wn1"], p["bn1"], p["Wn2"], p["bn2"])
    scores = kmeans_scores(s, p["centres"])
    labels = p["assign"].long()[scores.argmax(dim=1)]
    return full, scores, labels


def alpha_seg(sigma, labels, voxel_size=0.2):
    """evaluate_model_sscbench.py:727-742 at factor 1: argmax over classes of
    alpha * one_hot(label), alpha = 1 - exp(-VOXEL_SIZE * sigma)."""
    alphas = 1 - torch.exp(-voxel_size * sigma)
    onehot = F.one_hot(labels.long(), 19).float()
    return (alphas.unsqueeze(-1) * onehot).argmax(dim=-1)
