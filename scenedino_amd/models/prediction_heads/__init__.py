"""Prediction heads (mirror of scenedino/models/prediction_heads/__init__.py:14-47).
Only the ResNet head used by every shipped config is provided."""
from .resnetfc import ResnetFC


def make_head(conf, d_in: int, d_out: int):
    head_type = conf.get("type", "resnet")
    if head_type != "resnet":
        raise NotImplementedError(f"head type {head_type!r}: only 'resnet' (ResnetFC) is on the "
                                  "MI355X hot path")
    head = ResnetFC.from_conf(conf["args"], d_in, d_out)
    if conf.get("freeze", False):
        for p in head.parameters():
            p.requires_grad = False
    return head
