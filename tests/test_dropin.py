"""CPU: scenedino_amd.dropin.install() aliases the reference's hot-path imports
(scenedino.renderer.NeRFRenderer, scenedino.models.make_model / BTSNet / models.bts,
scenedino.common.ray_sampler.ImageRaySampler) to this build, leaving every other module of
the checkout alone.  A minimal stand-in `scenedino` package plays the reference checkout
(the test must not depend on /root/reference, which does not travel)."""
import importlib
import os
import sys
import textwrap

import pytest


@pytest.fixture
def fake_reference(tmp_path, monkeypatch):
    root = tmp_path / "ref"
    files = {
        "scenedino/__init__.py": "",
        "scenedino/renderer/__init__.py": "from .nerf import NeRFRenderer\n",
        "scenedino/renderer/nerf.py": "class NeRFRenderer:\n    origin = 'reference'\n",
        "scenedino/models/__init__.py": textwrap.dedent("""
            def make_model(config, downstream_config=None):
                return 'reference make_model'
            class BTSNet:
                origin = 'reference'
            """),
        "scenedino/models/bts.py": "class BTSNet:\n    origin = 'reference'\n",
        "scenedino/common/__init__.py": "",
        "scenedino/common/ray_sampler.py": textwrap.dedent("""
            class ImageRaySampler:
                origin = 'reference'
            class PatchRaySampler:
                origin = 'reference'
            """),
        "scenedino/losses/__init__.py": "MARK = 'reference losses'\n",
    }
    for rel, txt in files.items():
        f = root / rel
        f.parent.mkdir(parents=True, exist_ok=True)
        f.write_text(txt)
    saved = {k: v for k, v in sys.modules.items() if k == "scenedino" or k.startswith("scenedino.")}
    for k in saved:
        del sys.modules[k]
    monkeypatch.syspath_prepend(str(root))
    yield root
    for k in [k for k in sys.modules if k == "scenedino" or k.startswith("scenedino.")]:
        del sys.modules[k]
    sys.modules.update(saved)


def test_install_aliases_hot_path_only(fake_reference):
    from scenedino_amd import dropin
    from scenedino_amd.renderer import NeRFRenderer
    from scenedino_amd.models.bts import BTSNet
    from scenedino_amd.common.ray_sampler import ImageRaySampler
    dropin.install()
    from scenedino.renderer import NeRFRenderer as R1
    from scenedino.renderer.nerf import NeRFRenderer as R2
    from scenedino.models import make_model, BTSNet as B1
    from scenedino.models.bts import BTSNet as B2
    from scenedino.common.ray_sampler import ImageRaySampler as S1, PatchRaySampler
    assert R1 is NeRFRenderer and R2 is NeRFRenderer
    assert B1 is BTSNet and B2 is BTSNet
    assert S1 is ImageRaySampler
    assert make_model is dropin._ref_make_model
    # everything else stays the checkout's
    assert PatchRaySampler.origin == "reference"
    assert importlib.import_module("scenedino.losses").MARK == "reference losses"


def test_install_native_encoder_switch(fake_reference):
    from scenedino_amd import dropin
    dropin.install(native_encoder=False)
    assert dropin._NATIVE_ENCODER is False
    dropin.install()
    assert dropin._NATIVE_ENCODER is True


def test_native_encoder_refuses_training_forward():
    """DINOv2Module: a training forward with trainable decoder parameters raises instead
    of silently leaving them without gradients (dinov2_module.py:176-183)."""
    import torch
    from scenedino_amd.models.backbones import make_backbone
    conf = dict(type="dinov2", mode="downsample-prediction", decoder_arch="dpt",
                downsampler_arch="featup", encoder_arch="vit-s", version="v1_16",
                separate_gt_version=None, encoder_freeze=True, flip_avg_gt=False,
                dim_reduction_arch="mlp", num_ch_enc=[64, 64, 128, 256],
                intermediate_features=[3, 6, 9], decoder_out_dim=256, dino_pca_dim=64,
                image_size=[32, 64], key_features=False)
    m = make_backbone(conf).train()
    x = torch.zeros(1, 3, 32, 64)
    with pytest.raises(NotImplementedError, match="forward-only"):
        m(x)
    for p in m.decoder.parameters():
        p.requires_grad_(False)
    for p in m.encoder.parameters():
        p.requires_grad_(False)
    m.train()
    # all frozen: the guard lets the forward through to the kernels (which need the GPU)
    with pytest.raises(RuntimeError) as e:
        m(x)
    assert not isinstance(e.value, NotImplementedError)
