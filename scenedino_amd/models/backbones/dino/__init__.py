"""DINO encoder pieces (mirror of scenedino/models/backbones/dino/)."""
from .dim_reduction import MlpDimReduction, NoDimReduction
from .dinov2_module import DINOv2Module, OrthogonalLinearDimReduction
from .dpt_head import DPTHead
from .vit import DINOv2Encoder

__all__ = ["MlpDimReduction", "NoDimReduction", "OrthogonalLinearDimReduction", "DPTHead",
           "DINOv2Encoder", "DINOv2Module"]
