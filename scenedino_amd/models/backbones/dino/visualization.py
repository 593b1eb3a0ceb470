"""PCA / k-means colouring of feature maps (the encoder's visualization API).

Restatement of scenedino/models/backbones/dino/visualization.py:9-153, which
``DINOv2Module`` owns as ``self.visualization`` (dinov2_module.py:156) and exposes as
``fit_visualization`` / ``transform_visualization`` / ``fit_transform_kmeans_visualization``
(dinov2_module.py:194-201).  Callers: demo_script.py:43-78, demo_gradio.py:98-133 and
the ``visualization`` validation tags of trainer_downstream.py:56-65,189-196.

This is visualisation, not the render hot path: plain device tensor ops on whatever
device the features live on.  The reference's cosine k-means runs through pykeops
``LazyTensor`` (absent here); ``x_i | c_j`` followed by ``argmax(dim=1)`` is the dense
(N, K) dot-product matrix and its row argmax, computed here in row blocks so that a
192x640 frame never materialises more than ``_KM_BLOCK`` rows of scores.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np
import torch
from torch import Tensor, nn

# matplotlib's "tab10" ListedColormap (the reference's cmap_kmeans, visualization.py:19)
_TAB10 = np.array([
    (0x1f, 0x77, 0xb4), (0xff, 0x7f, 0x0e), (0x2c, 0xa0, 0x2c), (0xd6, 0x27, 0x28),
    (0x94, 0x67, 0xbd), (0x8c, 0x56, 0x4b), (0xe3, 0x77, 0xc2), (0x7f, 0x7f, 0x7f),
    (0xbc, 0xbd, 0x22), (0x17, 0xbe, 0xcf)], dtype=np.float64) / 255.0

_KM_BLOCK = 1 << 18


def tab10(values: np.ndarray) -> np.ndarray:
    """``plt.get_cmap("tab10")(values)[..., :3]`` for float inputs in [0, 1]
    (ListedColormap.__call__: x * N, x == N -> N - 1, clip, truncate to int)."""
    n = len(_TAB10)
    xa = np.array(values, copy=True)
    if not np.issubdtype(xa.dtype, np.floating):
        xa = xa.astype(np.float64)
    with np.errstate(invalid="ignore"):
        xa *= n
        xa[xa == n] = n - 1
        np.clip(xa, -1, n, out=xa)
    idx = xa.astype(int)
    idx = np.clip(idx, 0, n - 1)  # under / over colours of tab10 equal its end colours
    return _TAB10[idx]


class VisualizationModule(nn.Module):
    """visualization.py:9-19: state is plain tensors (no buffers, so no checkpoint keys)."""

    def __init__(self, in_channels: int, reduce_images: int = 3):
        super().__init__()
        self.batch_rgb_mean = torch.zeros(in_channels)
        self.batch_rgb_comp = torch.eye(in_channels, 3)
        self.reduce_images = reduce_images
        self.fitted_pca = False
        self.n_kmeans_clusters = 8
        self.kmeans_cluster_centers = torch.zeros(self.n_kmeans_clusters, in_channels)

    # -- PCA (visualization.py:21-88) -------------------------------------------
    def fit_pca(self, batch_features: Tensor, refit: bool) -> None:
        if batch_features.dim() > 2:
            raise ValueError(f"Wrong dims for PCA: {batch_features.shape}")
        if not self.fitted_pca or refit:
            keep = ~torch.isnan(batch_features).any(dim=1)
            self._pca_fast(batch_features[keep], num_components=3 * self.reduce_images)
            self.fitted_pca = True

    def transform_pca(self, features: Tensor, norm: bool, from_dim: int) -> Tensor:
        features = features - self.batch_rgb_mean
        if norm:
            features = features / torch.linalg.norm(features, dim=-1, keepdim=True)
        return features @ self.batch_rgb_comp[..., from_dim:from_dim + 3]

    def _pca_fast(self, data: Tensor, num_components: int = 3) -> None:
        """visualization.py:36-62: standardise, ``torch.pca_lowrank(q=max(n, 6), niter=2,
        center=True)``, SVD sign flip, keep the first ``num_components`` right vectors."""
        mean = data.mean(dim=-2, keepdim=True)
        normalized = (data - mean) / (data.std(dim=-2, keepdim=True) + 1e-08)
        u, _, v = torch.pca_lowrank(normalized, q=max(num_components, 6), niter=2, center=True)
        v = v.transpose(-1, -2)
        u, v = self._svd_flip(u, v)
        comps = v[:num_components] if normalized.ndim == 2 else v[:, :num_components]
        self.batch_rgb_mean = mean
        self.batch_rgb_comp = comps.transpose(-1, -2)

    @staticmethod
    def _svd_flip(u: Tensor, v: Tensor) -> Tuple[Tensor, Tensor]:
        """visualization.py:64-88: sign of each column's largest-|u| entry."""
        max_abs = torch.abs(u).argmax(dim=-2)
        cols = torch.arange(u.shape[-1], device=u.device)
        if u.ndim == 2:
            signs = torch.sign(u[max_abs, cols])
            return u * signs, v * signs.unsqueeze(-1)
        rows = torch.arange(u.shape[0], device=u.device).unsqueeze(-1)
        signs = torch.sign(u[rows, max_abs, cols])
        return u * signs.unsqueeze(1), v * signs.unsqueeze(-1)

    # -- cosine k-means (visualization.py:111-153) ------------------------------
    def fit_transform_kmeans_batch(self, batch_features: Tensor) -> Tensor:
        flat = batch_features.flatten(0, -2)
        with torch.no_grad():
            cl, c = self._kmeans_cosine(flat.float(), K=self.n_kmeans_clusters)
        self.kmeans_cluster_centers = c
        labels = cl.reshape(batch_features.shape[:-1]).float().cpu().numpy()
        label_map = tab10(labels / (self.n_kmeans_clusters - 1))
        return torch.Tensor(label_map).squeeze(-2)

    @staticmethod
    def _assign(x: Tensor, c: Tensor) -> Tensor:
        out = torch.empty(x.shape[0], dtype=torch.long, device=x.device)
        for s in range(0, x.shape[0], _KM_BLOCK):
            out[s:s + _KM_BLOCK] = (x[s:s + _KM_BLOCK] @ c.t()).argmax(dim=1)
        return out

    def _kmeans_cosine(self, x: Tensor, K: int = 19, Niter: int = 100):
        """Lloyd's algorithm for cosine similarity (visualization.py:125-153): centres
        initialised from the first K points, normalised; E step = argmax of dot products;
        M step = scatter-add of the points, normalised."""
        N, D = x.shape
        c = torch.nn.functional.normalize(x[:K].clone(), dim=1, p=2)
        cl = torch.zeros(N, dtype=torch.long, device=x.device)
        for _ in range(Niter):
            cl = self._assign(x, c)
            c = torch.zeros_like(c).scatter_add_(0, cl[:, None].expand(N, D), x)
            c = torch.nn.functional.normalize(c, dim=1, p=2)
        return cl, c
