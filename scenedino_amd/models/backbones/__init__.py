"""Encoder-side pieces of the MI355X build (mirror of scenedino/models/backbones/)."""


def make_backbone(conf, **kwargs):
    """backbone_util.py:7-19.  Only the ``dinov2`` encoder type is shipped by SceneDINO's
    configs (configs/model/*.yaml); the monodepth2 / spatial / global ResNet encoders of
    the BTS lineage are not part of this build."""
    enc_type = conf.get("type", "monodepth2")
    if enc_type == "dinov2":
        from .dino.dinov2_module import DINOv2Module
        return DINOv2Module.from_conf(conf, **kwargs)
    raise NotImplementedError(f"Unsupported encoder type: {enc_type}")


__all__ = ["make_backbone"]
