"""scenedino_amd -- MI355X-native (gfx950) SceneDINO volumetric feature-field render path.

Mirrors the reference's plugin API for the hot path (scenedino.renderer.NeRFRenderer,
scenedino.models.make_model / BTSNet, scenedino.common.ray_sampler.ImageRaySampler)
on top of the C-ABI library libsdhip.so (include/sdhip.h).
"""
from . import _lib  # noqa: F401

__version__ = "0.1.0"
