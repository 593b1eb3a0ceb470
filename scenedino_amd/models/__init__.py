"""Model factory (mirror of scenedino/models/__init__.py:9-63)."""
from ..common.positional_encoding import PositionalEncoding
from .bts import BTSNet
from .prediction_heads import make_head


def make_model(config, downstream_config=None, encoder=None, downstream_head=None):
    """Build BTSNet from the reference's model config.

    As the reference, the encoder is built from ``config['encoder']``
    (backbones.make_backbone -> DINOv2Module: ViT + DPT on the gfx950 kernels) and the
    downstream head from ``downstream_config``; ``encoder`` / ``downstream_head`` may be
    passed in instead (any module exposing ``latent_size``, ``extra_outs``,
    ``forward(x, ground_truth=False) -> [grid]`` and ``expand_dim``).
    """
    arch = config.get("arch", "BTSNet")
    if arch != "BTSNet":
        raise NotImplementedError("Model architecture was not implemented yet")
    sample_color = config.get("sample_color", True)
    predict_dino = config.get("predict_dino", False)
    dino_dims = config.get("dino_dims", 16)
    if sample_color and predict_dino:
        d_out = 1 + dino_dims
    elif sample_color:
        d_out = 1
    else:
        d_out = 4
    if encoder is None:
        from .backbones import make_backbone
        encoder = make_backbone(config["encoder"])
    if downstream_head is None and downstream_config is not None:
        from ..downstream_head import make_downstream_head
        downstream_head = make_downstream_head(downstream_config)
    code_xyz = PositionalEncoding.from_conf(config["code"], d_in=3)
    d_in = encoder.latent_size + code_xyz.d_out
    if config.get("split_dino_heads", False):
        raise NotImplementedError("split_dino_heads is not used by any shipped config")
    heads = {hc["name"]: make_head(hc, d_in, d_out) for hc in config["decoder_heads"]}
    return BTSNet(config, encoder, code_xyz, heads, config.get("final_pred_head", None),
                  downstream_head=downstream_head)


__all__ = ["BTSNet", "make_model", "make_head"]
