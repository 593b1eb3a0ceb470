"""Unsupervised SSC head, MI355X build (inference subset).

Mirror of scenedino/downstream_head/semantic_head.py (SemanticHead :41-120,
StegoClusterHead :285-305, KMeansParamHead :308-373, LinearHead :460-477, MLPHead
:480-501): same class names, constructor arguments, sub-module / parameter / buffer names
(``stego_head.linear_path.0``, ``stego_head.nonlinear_path.{0,2}``,
``{direct,stego}_cluster_head.cluster_centers``, ``.pseudo_assignment``,
``{direct,stego}_linear_head.linear``), so reference checkpoints load unchanged.

The hot use of this head -- BTSNet.forward(..., predict_segmentation=True) and the
SSCBench voxel query -- never calls ``forward`` here: BTSNet hands the 64-d DINO codes
straight to the folded gfx950 kernel ``sd_seg_query`` (transform_expand + stego +
cosine k-means in registers, csrc/sdhip_seg.hip), which reads these modules'
parameters.  ``forward`` on already-expanded 768-d features (a standalone call outside
the hot path) evaluates the same math with device tensor ops.  Training-only state
(kNN buffers, CRF, losses) is out of scope.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from .. import _lib


def _norm(x):
    # semantic_head.py:37-38
    return F.normalize(x, dim=-1, eps=1e-10)


class StegoClusterHead(nn.Module):
    def __init__(self, in_channels, out_channels, mid_channels=None):
        super().__init__()
        mid = in_channels if mid_channels is None else mid_channels
        self.linear_path = nn.Sequential(nn.Conv2d(in_channels, out_channels, (1, 1)),
                                         nn.Dropout2d(p=0.1))
        self.nonlinear_path = nn.Sequential(nn.Conv2d(in_channels, mid, (1, 1)), nn.ReLU(),
                                            nn.Conv2d(mid, out_channels, (1, 1)),
                                            nn.Dropout2d(p=0.1))

    @staticmethod
    def _lin(conv, x):
        return F.linear(x, conv.weight.reshape(conv.weight.shape[0], -1), conv.bias)

    def forward(self, x):
        """1x1 convolutions over the channel (last) dim, as linear maps; L2-normalised."""
        lin = self._lin(self.linear_path[0], x)
        mid = torch.relu(self._lin(self.nonlinear_path[0], x))
        out = lin + self._lin(self.nonlinear_path[2], mid)
        return _norm(out).to(x.dtype)


class KMeansParamHead(nn.Module):
    def __init__(self, n_classes: int, gt_classes: int, dim: int):
        super().__init__()
        self.n_classes = n_classes
        self.dim = dim
        self.cluster_centers = nn.Parameter(torch.randn(n_classes, dim))
        self.register_buffer("pseudo_assignment", torch.arange(0, n_classes).remainder(gt_classes))

    def forward(self, features, weight=None):
        flat = features.flatten(0, -2)
        centres = F.normalize(self.cluster_centers, dim=1)
        scores = F.normalize(flat, dim=1) @ centres.t()
        labels = scores.argmax(dim=1).view(*features.shape[:-1])
        return {"pseudo_segs_pred": labels,
                "segs_pred": self.pseudo_assignment[labels].long()}


class LinearHead(nn.Module):
    def __init__(self, dim: int, gt_classes: int):
        super().__init__()
        self.linear = nn.Linear(dim, gt_classes)

    def forward(self, features, target=None):
        return {"segs_pred": self.linear(features).float().argmax(-1)}


class MLPHead(nn.Module):
    def __init__(self, dim: int, gt_classes: int):
        super().__init__()
        self.linear1 = nn.Linear(dim, 2 * dim)
        self.linear2 = nn.Linear(2 * dim, gt_classes)
        self.activation = nn.ReLU()

    def forward(self, features, target=None):
        return {"segs_pred": self.linear2(self.activation(self.linear1(features))).float().argmax(-1)}


class SemanticHead(nn.Module):
    def __init__(self, n_classes, gt_classes, input_dim, code_dim, buffer_size=0,
                 patch_sample_size=0, knn_neighbors=0, mode="2d", mlp_head=False,
                 apply_crf=False):
        super().__init__()
        self.n_classes = n_classes
        self.gt_classes = gt_classes
        self.input_dim = input_dim
        self.code_dim = code_dim
        self.knn_neighbors = knn_neighbors
        self.mode = mode
        self.apply_crf = apply_crf
        self.direct_cluster_head = KMeansParamHead(n_classes, gt_classes, input_dim)
        self.stego_head = StegoClusterHead(input_dim, code_dim)
        self.stego_cluster_head = KMeansParamHead(n_classes, gt_classes, code_dim)
        head = MLPHead if mlp_head else LinearHead
        self.direct_linear_head = head(input_dim, gt_classes)
        self.stego_linear_head = head(code_dim, gt_classes)

    @classmethod
    def from_conf(cls, config):
        g = config.get
        return cls(n_classes=g("n_classes"), gt_classes=g("gt_classes"),
                   input_dim=g("input_dim"), code_dim=g("code_dim"),
                   buffer_size=g("buffer_size", 0), patch_sample_size=g("patch_sample_size", 0),
                   knn_neighbors=g("knn_neighbors", 0), mode=g("mode", "2d"),
                   mlp_head=g("mlp_head", False), apply_crf=g("apply_crf", False))

    def _folded_labels(self, features):
        """segs_pred of mode stego_kmeans for features that MlpDimReduction.transform_expand
        produced (and nobody modified since): the folded kernel sd_seg_query on the 64-d codes
        (transform_expand + stego + k-means in registers), or None."""
        prov = getattr(features, "_sd_expand", None)
        if prov is None or features.requires_grad or torch.is_grad_enabled() and self.training:
            return None
        codes, dr, key, version = prov
        from ..seg_pack import PackedSegHead, seg_key
        if features._version != version or seg_key(dr) != key:
            return None
        hkey = seg_key(dr, self.stego_head, self.stego_cluster_head)
        cache = getattr(self, "_fold_cache", None)
        if cache is None or cache[0] != hkey or cache[1] is not dr:
            cache = self._fold_cache = (hkey, dr, PackedSegHead(
                dr, self.stego_head, self.stego_cluster_head, device=codes.device))
        labels, _, _ = _lib.seg_query(codes, cache[2].rec, want_labels=True)
        return labels.view(features.shape[:-1]).long()

    def forward(self, features, mode="stego_kmeans"):
        """semantic_head.py:107-120 (segs_pred for the given mode).  stego_kmeans on
        features straight from MlpDimReduction.transform_expand (the 2-D demo's
        expand_dim -> downstream_head) runs as the folded sd_seg_query kernel on their
        64-d codes; any other input or mode evaluates the chain with device tensor ops."""
        if mode == "stego_kmeans":
            labels = self._folded_labels(features)
            if labels is not None:
                return labels
        features = _norm(features)
        if mode == "stego_kmeans":
            return self.stego_cluster_head(self.stego_head(features))["segs_pred"]
        if mode == "stego_linear":
            return self.stego_linear_head(self.stego_head(features))["segs_pred"]
        if mode == "direct_kmeans":
            return self.direct_cluster_head(features)["segs_pred"]
        if mode == "direct_linear":
            return self.direct_linear_head(features)["segs_pred"]
        raise NotImplementedError(f"Mode '{mode}' is not known!")

    def update_model_eval(self, metrics):
        self.direct_cluster_head.pseudo_assignment[:] = metrics["direct_cluster_assignment"]
        self.stego_cluster_head.pseudo_assignment[:] = metrics["stego_cluster_assignment"]
