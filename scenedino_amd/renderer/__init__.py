from .nerf import NeRFRenderer

__all__ = ["NeRFRenderer"]
