"""Unsupervised SSC head (mirror of scenedino/downstream_head/, inference subset)."""
from .semantic_head import KMeansParamHead, LinearHead, MLPHead, SemanticHead, StegoClusterHead


def make_downstream_head(config):
    """scenedino/downstream_head/__init__.py: type 'segmentation' -> SemanticHead."""
    kind = config.get("type", "segmentation")
    if kind != "segmentation":
        raise NotImplementedError(f"downstream head type {kind!r}")
    return SemanticHead.from_conf(config)


__all__ = ["SemanticHead", "StegoClusterHead", "KMeansParamHead", "LinearHead", "MLPHead",
           "make_downstream_head"]
