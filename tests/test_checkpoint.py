"""Reference checkpoint loading (demo_utils/utils.py:52-55), on CPU.

No released checkpoint travels here (remote download), so the file is synthesised in the
reference's layout: the BTSWrapper state_dict keys (``renderer.net.*``,
``renderer.renderer.*``) of a model built from the shipped model config (the featup
downsampler of the loss included), plus keys of the visualisation module the build does
not construct.  Loading must reproduce every parameter bit-for-bit in a freshly initialised model.
"""
import pytest
import torch

from test_encoder import MODEL_CONF

DOWNSTREAM = {"type": "segmentation", "n_classes": 19, "gt_classes": 19, "input_dim": 384,
              "code_dim": 64, "knn_neighbors": 4, "buffer_size": 256, "patch_sample_size": 576,
              "mode": "3d", "apply_crf": False}


def build(seed):
    from scenedino_amd.models import make_model
    from scenedino_amd.renderer import NeRFRenderer
    torch.manual_seed(seed)
    net = make_model(MODEL_CONF, DOWNSTREAM)
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for p in net.parameters():
            p.copy_(torch.randn(p.shape, generator=g))
    return NeRFRenderer(n_coarse=32, lindisp=True).bind_parallel(net, gpus=None)


def reference_layout(wrapper):
    sd = {"renderer." + k: v.clone() for k, v in wrapper.state_dict().items()}
    sd["renderer.net.encoder.visualization.pca.weight"] = torch.randn(3, 64)
    sd["renderer.renderer.iter_idx"] = torch.tensor(1234)
    return sd


def test_roundtrip_through_file(tmp_path):
    from scenedino_amd.checkpoint import load_checkpoint
    src = build(1)
    sd = reference_layout(src)
    assert any(k.startswith("renderer.net.encoder.encoder.model.vit.blocks.") for k in sd)
    assert any(k.startswith("renderer.net.downstream_head.") for k in sd)
    path = tmp_path / "checkpoint.pt"
    torch.save(sd, path)
    dst = build(2)
    rep = load_checkpoint(dst, str(path))
    assert not rep.missing and not rep.unexpected
    assert sorted(rep.ignored) == ["encoder.visualization.pca.weight"]
    assert "encoder.downsampler.conv.weight" in src.net.state_dict()
    a, b = src.net.state_dict(), dst.net.state_dict()
    assert a.keys() == b.keys()
    for k in a:
        assert torch.equal(a[k], b[k]), k
    assert int(dst.renderer.iter_idx) == 1234
    # the older {"model": ...} layout and a bare BTSNet target load the same way
    dst2 = build(3)
    rep2 = load_checkpoint(dst2.net, {"model": sd})
    assert not rep2.missing
    assert torch.equal(dst2.net.heads["normal_head"].lin_in.weight,
                       src.net.heads["normal_head"].lin_in.weight)


def test_missing_or_misshaped_hot_path_keys_fail_loudly():
    from scenedino_amd.checkpoint import load_checkpoint
    src = build(4)
    sd = reference_layout(src)
    del sd["renderer.net.heads.normal_head.lin_in.weight"]
    with pytest.raises(KeyError):
        load_checkpoint(build(5), sd)
    rep = load_checkpoint(build(5), sd, strict=False)
    assert rep.missing == ["heads.normal_head.lin_in.weight"]
    sd = reference_layout(src)
    sd["renderer.net.encoder.decoder.project.weight"] = torch.zeros(3, 3)
    with pytest.raises(ValueError):
        load_checkpoint(build(6), sd)


def test_state_dict_layout_matches_reference_manifest():
    """Every module whose parameters come from a reference checkpoint has the reference's
    exact key -> shape layout (tests/golden/state_dict_manifest.json, written by
    make_golden.fx_state_dict_manifest from the reference modules themselves)."""
    import json
    import os
    from conftest import GOLDEN
    from scenedino_amd.models import BTSNet
    from scenedino_amd.models.prediction_heads import ResnetFC
    from scenedino_amd.common.positional_encoding import PositionalEncoding
    from scenedino_amd.renderer import NeRFRenderer
    from scenedino_amd.models.backbones.dino.dpt_head import DPTHead
    from scenedino_amd.models.backbones.dino import MlpDimReduction
    from scenedino_amd.downstream_head import SemanticHead
    man = json.load(open(os.path.join(GOLDEN, "state_dict_manifest.json")))

    class FixedGrid(torch.nn.Module):
        latent_size, extra_outs = 256, 0

        def forward(self, x, ground_truth=False):
            return [torch.zeros(1, 256, 4, 8)]

    shapes = lambda m, drop=(): {k: list(v.shape) for k, v in m.state_dict().items()
                                 if not k.startswith(drop)}
    head = ResnetFC(d_in=295, d_out=65, n_blocks=0, d_hidden=128)
    conf = {"predict_dino": True, "dino_dims": 64, "learn_empty": False, "code_mode": "z",
            "inv_z": True, "z_near": 3, "z_far": 80, "sample_color": True}
    net = BTSNet(conf, FixedGrid(), PositionalEncoding(6, 3, 1.5, True), {"normal_head": head},
                 final_pred_head="normal_head")
    ours = {
        "resnetfc": shapes(head),
        "btsnet": shapes(net, drop=("encoder.",)),
        "nerf_renderer": shapes(NeRFRenderer(n_coarse=32, lindisp=True)),
        "dpt_head_vits": shapes(DPTHead(embed_dims=384, post_process_channels=[64, 64, 128, 256],
                                        readout_type="ignore", patch_size=16, d_out=256)),
        "dpt_head_vitb": shapes(DPTHead(embed_dims=768, post_process_channels=[64, 64, 128, 256],
                                        readout_type="ignore", patch_size=16, d_out=256)),
        "mlp_dim_reduction": shapes(MlpDimReduction(768, 64, 128)),
        "semantic_head": shapes(SemanticHead(19, 19, 768, 64, mlp_head=False)),
        "semantic_head_mlp": shapes(SemanticHead(19, 19, 768, 64, mlp_head=True)),
    }
    assert sorted(ours) == sorted(man)
    for name in man:
        assert ours[name] == man[name], name

