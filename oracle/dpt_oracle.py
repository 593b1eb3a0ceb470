"""dpt_oracle -- TEST INFRASTRUCTURE ONLY (the checker, never shipped).

PyTorch CPU fp32 restatement of the DPT decoder forward
(scenedino/models/backbones/dino/dpt_head.py:10-236) over the parameters of a
scenedino_amd DPTHead (same names as the reference).  Pinned by tests/golden/dpt_head.npz,
written by running the reference's own DPTHead (tests/golden/make_golden.py).
"""
from __future__ import annotations

import torch.nn.functional as F


def _conv(m, x, stride=1, padding=0):
    return F.conv2d(x, m.weight, m.bias, stride=stride, padding=padding)


def _rcu(u, x):
    """PreActResidualConvUnit (dpt_head.py:73-118, bn=False)."""
    y = _conv(u.conv1, F.relu(x), padding=1)
    y = _conv(u.conv2, F.relu(y), padding=1)
    return y + x


def _fusion(fb, x, res=None):
    """FeatureFusionBlock (dpt_head.py:121-158)."""
    if res is not None:
        if x.shape != res.shape:
            res = F.interpolate(res, size=x.shape[2:], mode="bilinear", align_corners=False)
        x = x + _rcu(fb.res_conv_unit1, res)
    x = _rcu(fb.res_conv_unit2, x)
    x = F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=fb.align_corners)
    return _conv(fb.project, x)


def dpt_forward(head, inputs):
    """inputs: 4 NCHW grids -> NCHW output grid (DPTHead.forward, dpt_head.py:226-236)."""
    rb = head.reassemble_blocks
    r = []
    for i, x in enumerate(inputs):
        x = _conv(rb.projects[i], x)
        if i < 2:
            t = rb.resize_layers[i]
            x = F.conv_transpose2d(x, t.weight, t.bias, stride=t.stride)
        elif i == 3:
            x = _conv(rb.resize_layers[3], x, stride=2, padding=1)
        r.append(x)
    f = [_conv(c, x, padding=1) for c, x in zip(head.convs, r)]
    out = _fusion(head.fusion_blocks[0], f[-1])
    for i in range(1, len(head.fusion_blocks)):
        out = _fusion(head.fusion_blocks[i], out, f[-(i + 1)])
    out = _conv(head.project, out, padding=1)
    hm = head.output_head.head_modules
    out = _conv(hm[0], out, padding=1)
    out = F.conv_transpose2d(out, hm[1].weight, hm[1].bias, stride=hm[1].stride)
    return _conv(hm[2], out, padding=1)
