"""DINO encoder pieces (mirror of scenedino/models/backbones/dino/)."""
from .dim_reduction import MlpDimReduction, NoDimReduction

__all__ = ["MlpDimReduction", "NoDimReduction"]
