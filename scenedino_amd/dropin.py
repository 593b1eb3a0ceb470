"""Drop the MI355X render path into an unmodified reference checkout.

The reference's callers (train.py, eval.py, demo_script.py, sscbench/
evaluate_model_sscbench.py) import the hot path as

    from scenedino.renderer import NeRFRenderer            # renderer/__init__.py:1
    from scenedino.models import make_model                # models/__init__.py:9
    from scenedino.common.ray_sampler import ImageRaySampler

``install()`` registers this package's mirrors under those module names before the
reference is imported, so those imports resolve here while every other reference
module (encoders, data sets, trainer, losses, visualisation) stays the reference's.
``make_model`` keeps the reference's signature (scenedino/models/__init__.py:9-63): the
image encoder is this package's ``DINOv2Module`` (ViT + DPT on gfx950, one HIP graph per
pass) for every configuration it covers, else the reference's own ``make_backbone``
(models/backbones/backbone_util.py) with its ViT and DPTHead aliased to the gfx950
mirrors; the downstream head comes from ``scenedino.downstream_head.make_downstream_head``.
Both go to this package's BTSNet, whose parameter names equal the reference's, so
``checkpoint.pt`` state dicts load unchanged (demo_utils/utils.py:52-55).
"""
from __future__ import annotations

import importlib
import sys
import types


_NATIVE_ENCODER = True


def _ref_make_model(config, downstream_config=None):
    from . import models as amd_models
    from .models.backbones import make_backbone as amd_make_backbone
    try:
        # the native DINOv2Module (ViT + DPT as one HIP graph; same parameter names)
        if not _NATIVE_ENCODER:
            raise NotImplementedError("native encoder disabled (install(native_encoder=False))")
        encoder = amd_make_backbone(config["encoder"])
    except NotImplementedError:
        # encoder variants this build does not cover (non-DPT decoders, register / FiT3D
        # ViTs, separate gt versions, upsample-gt mode): the reference's own module, whose
        # ViT and DPTHead still resolve to the gfx950 mirrors aliased by install()
        backbones = importlib.import_module("scenedino.models.backbones")
        encoder = backbones.make_backbone(config["encoder"])
    downstream_head = None
    if downstream_config is not None:
        heads = importlib.import_module("scenedino.downstream_head")
        downstream_head = heads.make_downstream_head(downstream_config)
    return amd_models.make_model(config, downstream_config, encoder=encoder,
                                 downstream_head=downstream_head)


def install(native_encoder: bool = True):
    """Alias scenedino.renderer / scenedino.models.make_model / ImageRaySampler to the
    MI355X build.  Call before the first ``import scenedino...``.

    native_encoder=False keeps the image encoder entirely the reference's (its timm ViT and
    DPTHead with autograd): use it for train.py when the encoder or the DPT decoder is
    trained -- the native ViT / DPT kernels are forward-only and DINOv2Module refuses a
    training forward with trainable parameters rather than drop their gradients.  The
    field / render path (BTSNet, NeRFRenderer, ImageRaySampler) is the build's either way."""
    global _NATIVE_ENCODER
    _NATIVE_ENCODER = bool(native_encoder)
    from . import renderer as amd_renderer
    from .common import ray_sampler as amd_rs
    from .models import bts as amd_bts

    ren = types.ModuleType("scenedino.renderer")
    ren.NeRFRenderer = amd_renderer.NeRFRenderer
    ren.__path__ = []  # package: scenedino.renderer.nerf resolves below
    sys.modules["scenedino.renderer"] = ren
    sys.modules["scenedino.renderer.nerf"] = importlib.import_module(
        "scenedino_amd.renderer.nerf")

    models = importlib.import_module("scenedino.models")
    models.make_model = _ref_make_model
    models.BTSNet = amd_bts.BTSNet
    sys.modules["scenedino.models.bts"] = amd_bts

    rs = importlib.import_module("scenedino.common.ray_sampler")
    rs.ImageRaySampler = amd_rs.ImageRaySampler

    # The DINO / DINOv2 ViT of the encoder (dinov2_module.py:19-28 build_encoder looks
    # DINOv2Encoder up at call time): same parameter names (model.vit.*), gfx950 kernels,
    # no hub download -- the weights come from checkpoint.pt.  The DPT decoder, the
    # downsampler and the dimension reduction stay the reference's modules (BTSNet reads
    # dim_reduction's parameters for the fused sd_seg_query head).
    try:
        dm = importlib.import_module("scenedino.models.backbones.dino.dinov2_module") \
            if native_encoder else None
    except ImportError:  # the reference's encoder dependencies (timm, torchvision) absent
        dm = None
    if dm is not None:
        from .models.backbones.dino import vit as amd_vit
        from .models.backbones.dino import dpt_head as amd_dpt
        dm.DINOv2Encoder = amd_vit.DINOv2Encoder
        # build_decoder (dinov2_module.py:31-56) looks DPTHead up at call time too
        dm.DPTHead = amd_dpt.DPTHead
