"""SceneDINO encoder module (ViT -> DPT, dinov2_module.py:91-222) on gfx950.

CPU: the mirror's constructor / ``from_conf`` / ``make_backbone`` contract and checkpoint
key names.  GPU: the whole prediction pass (one HIP graph: ViT kernels, NHWC token grids,
DPT kernels) against the fp32 oracles chained (oracle/vit_oracle.py ->
oracle/dpt_oracle.py) on the same random weights: rel-L2 <= 5e-2 (12 bf16 ViT blocks then
~20 bf16 convolution layers, tolerance written here); graph replay bit-identical to eager;
the ground-truth path returns the gt encoder's normalised final grid.
"""
import pytest
import torch

from oracle import dpt_oracle as DO
from oracle import vit_oracle as VO
from test_dpt import det_fill
from test_vit import init_vit

CONF = dict(type="dinov2", mode="downsample-prediction", decoder_arch="dpt",
            downsampler_arch="featup", encoder_arch="vit-s", version="v1_16",
            separate_gt_version="v1_16", encoder_freeze=False, flip_avg_gt=False,
            dim_reduction_arch="mlp", num_ch_enc=[64, 64, 128, 256],
            intermediate_features=[3, 6, 9], decoder_out_dim=256, dino_pca_dim=64,
            image_size=[64, 160], key_features=False)


def make(conf=CONF, seed=0):
    from scenedino_amd.models.backbones import make_backbone
    m = make_backbone(conf).eval()
    init_vit(m.encoder.model.vit, seed)
    init_vit(m.gt_encoder.model.vit, seed + 1)
    det_fill(m.decoder, seed + 2)
    return m


def test_from_conf_and_checkpoint_keys():
    m = make()
    keys = set(m.state_dict())
    for k in ("encoder.model.vit.blocks.0.attn.qkv.weight", "gt_encoder.model.vit.norm.bias",
              "decoder.reassemble_blocks.projects.0.weight", "decoder.output_head.head_modules.2.bias",
              "dim_reduction.linear_in.weight", "dim_reduction.linear_out.bias"):
        assert k in keys, k
    assert m.latent_size == 256 and m.extra_outs == 0
    assert m.encoder.patch_size == 16 and m.encoder.latent_size == 384
    with pytest.raises(NotImplementedError):
        m.downsample(torch.zeros(1))  # featup downsampler: training loss, out of scope
    shared = make(dict(CONF, separate_gt_version=None))
    assert shared.gt_encoder is shared.encoder and shared.encoder_frozen


def test_unsupported_modes_fail_loudly():
    from scenedino_amd.models.backbones import make_backbone
    with pytest.raises(NotImplementedError):
        make_backbone(dict(CONF, mode="upsample-gt", downsampler_arch=None,
                           upsampler_arch="multiscale-crop"))
    with pytest.raises(NotImplementedError):
        make_backbone(dict(CONF, type="monodepth2"))


# ------------------------------------------------------------------------ GPU
@pytest.fixture(scope="module")
def gpu():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    from scenedino_amd import _lib
    _lib.load()
    return "cuda"


def _rel(a, r):
    return ((a.double().cpu() - r.double()).norm() / r.double().norm()).item()


@pytest.mark.gpu
@pytest.mark.parametrize("conf", [CONF, dict(CONF, encoder_arch="vit-b", version="v2",
                                              separate_gt_version=None, image_size=[64, 192])])
def test_encoder_module_vs_oracles(gpu, conf):
    m = make(conf, seed=11)
    H, W = conf["image_size"]
    g = torch.Generator().manual_seed(12)
    x = torch.rand(2, 3, H, W, generator=g) * 2 - 1
    m_cpu_vit = m.encoder.model.vit
    m = m.to(gpu)
    with torch.no_grad():
        out = m(x.to(gpu))
        gt = m(x.to(gpu), ground_truth=True)
    assert len(out) == 1 and out[0].shape == (2, 256, H, W)
    xr = x
    if m.encoder.resize is not None:
        xr = torch.nn.functional.interpolate(x, size=m.encoder.resize, mode="bilinear",
                                             align_corners=False, antialias=True)
    vit = m_cpu_vit.cpu()
    feats = VO.encoder_forward(vit, xr, m.encoder.model.intermediate)
    ref = DO.dpt_forward(m.decoder.cpu(), feats)
    assert _rel(out[0], ref) <= 5e-2
    gvit = m.gt_encoder.model.vit.cpu()
    gref = VO.encoder_forward(gvit, xr, m.gt_encoder.model.intermediate)[-1]
    assert len(gt) == 1 and _rel(gt[0], gref) <= 3e-2


@pytest.mark.gpu
def test_encoder_graph_replay_matches_eager(gpu):
    m = make(seed=21).to(gpu)
    g = torch.Generator().manual_seed(22)
    xs = [(torch.rand(1, 3, 64, 160, generator=g) * 2 - 1).to(gpu) for _ in range(3)]
    with torch.no_grad():
        m.use_graph = False
        eager = [m(x)[0] for x in xs]
        m.use_graph = True
        graph = [m(x)[0] for x in xs]
    for a, b in zip(eager, graph):
        assert torch.equal(a, b)
