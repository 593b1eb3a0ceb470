"""SceneDINO checkpoint loading.

The reference loads ``checkpoint.pt`` -- the state_dict of the trainer's ``BTSWrapper``
-- with ``model.load_state_dict(cp, strict=False)`` (demo_utils/utils.py:52-55): keys
``renderer.net.*`` are BTSNet's (``renderer.net.encoder.encoder.model.vit.*``,
``renderer.net.encoder.decoder.*``, ``renderer.net.heads.normal_head.*``,
``renderer.net.encoder.dim_reduction.*``, ``renderer.net.downstream_head.*``, ...),
``renderer.renderer.{iter_idx,last_sched}`` the renderer's buffers.  The MI355X build keeps
every hot-path parameter under the same name and shape, so the mapping is the identity
after the prefix; this loader

  * reads the file with ``torch.load(weights_only=True)`` (no unpickling of code),
  * accepts the older ``{"model": state_dict}`` layout (utils.py:54 comment),
  * loads into a BTSNet or a ``bind_parallel`` wrapper (``net`` + ``renderer``),
  * ignores (and reports) the training-only modules this build does not construct
    (``encoder.visualization.*``, ``encoder.gt_wrapper.*``), as strict=False
    does in the reference,
  * but fails loudly when a parameter the kernels read is missing or mis-shaped (the
    reference would silently keep random weights there).

The kernels' packed operands (bf16 / NHWC weight images) are keyed on each parameter's
storage version, so they are rebuilt on the next forward after a load.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, List, Mapping, Union

import torch

PREFIX_NET = "renderer.net."
PREFIX_RENDERER = "renderer.renderer."
# modules of the reference DINOv2Module that this build does not construct (training loss /
# TensorBoard colouring): their keys are reported, not loaded
IGNORED_SUBTREES = ("encoder.visualization.", "encoder.gt_wrapper.")


@dataclass
class LoadReport:
    loaded: List[str] = field(default_factory=list)
    ignored: List[str] = field(default_factory=list)      # training-only reference modules
    unexpected: List[str] = field(default_factory=list)   # other keys with no target
    missing: List[str] = field(default_factory=list)      # target keys absent from the file


def read_state_dict(src: Union[str, os.PathLike, Mapping[str, torch.Tensor]]) -> Dict[str, torch.Tensor]:
    if isinstance(src, Mapping):
        sd = dict(src)
    else:
        sd = torch.load(src, map_location="cpu", weights_only=True)
    if "model" in sd and isinstance(sd["model"], Mapping):
        sd = dict(sd["model"])
    return sd


def load_checkpoint(target: torch.nn.Module, src, strict: bool = True) -> LoadReport:
    """Load a reference SceneDINO checkpoint into ``target`` (BTSNet or its render
    wrapper).  ``strict``: raise when a key the build reads is missing or a shape differs."""
    sd = read_state_dict(src)
    net = getattr(target, "net", target)
    renderer = getattr(target, "renderer", None) if net is not target else None
    rep = LoadReport()
    net_sd, ren_sd = {}, {}
    for k, v in sd.items():
        if k.startswith(PREFIX_NET):
            net_sd[k[len(PREFIX_NET):]] = v
        elif k.startswith(PREFIX_RENDERER):
            ren_sd[k[len(PREFIX_RENDERER):]] = v
        elif not any(k.startswith(p) for p in (PREFIX_NET, PREFIX_RENDERER, "renderer.")):
            net_sd.setdefault(k, v)  # bare BTSNet state_dict
        else:
            rep.unexpected.append(k)
    own = net.state_dict()
    load = {}
    for k, v in net_sd.items():
        if any(k.startswith(p) for p in IGNORED_SUBTREES):
            rep.ignored.append(k)
        elif k not in own:
            rep.unexpected.append(k)
        elif tuple(own[k].shape) != tuple(v.shape):
            raise ValueError(f"checkpoint key {k}: shape {tuple(v.shape)}, model expects "
                             f"{tuple(own[k].shape)}")
        else:
            load[k] = v
    rep.missing = sorted(k for k in own if k not in load)
    if strict and rep.missing:
        raise KeyError(f"checkpoint lacks {len(rep.missing)} parameter(s) the model reads, "
                       f"e.g. {rep.missing[:5]}")
    net.load_state_dict(load, strict=False)
    rep.loaded = sorted(load)
    if renderer is not None and ren_sd:
        own_r = renderer.state_dict()
        rl = {k: v for k, v in ren_sd.items() if k in own_r}
        rep.unexpected += [PREFIX_RENDERER + k for k in ren_sd if k not in own_r]
        renderer.load_state_dict(rl, strict=False)
        rep.loaded += [PREFIX_RENDERER + k for k in sorted(rl)]
    return rep
