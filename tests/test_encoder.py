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
    from scenedino_amd.models.backbones.dino.downsampler import PatchSalienceDownsampler
    assert isinstance(m.downsampler, PatchSalienceDownsampler)  # featup (the loss)
    assert "downsampler.conv.weight" in keys and "downsampler.patch_weight" in keys
    assert tuple(m.downsampler.conv.weight.shape) == (1, 384, 1, 1)
    shared = make(dict(CONF, separate_gt_version=None))
    assert shared.gt_encoder is shared.encoder and shared.encoder_frozen


def test_encode_defers_the_ground_truth_pass():
    """bts.py:207 runs the gt encoder inside encode(); the build runs it on the first read
    of grid_l_loss_features (same value), so render-only callers skip it."""
    import _helpers
    calls = []

    class Enc(_helpers.FixedGridEncoder):
        def forward(self, x, ground_truth=False):
            calls.append((ground_truth, tuple(x.shape)))
            g = self.grid.expand(x.shape[0], -1, -1, -1)
            return [g * (2.0 if ground_truth else 1.0)]

    grid = torch.randn(1, 8, 6, 10)
    net = _helpers.build_net(torch.zeros(1, 8, 6, 10), torch.zeros(128, 47), torch.zeros(128),
                             torch.zeros(5, 128), torch.zeros(5), device="cpu")
    net.encoder = Enc(grid)
    imgs = torch.rand(1, 2, 3, 12, 20) * 2 - 1
    Ks = torch.eye(3).expand(1, 2, 3, 3).contiguous()
    poses = torch.eye(4).expand(1, 2, 4, 4).contiguous()
    net.encode(imgs, Ks, poses, ids_encoder=[0], ids_render=[0, 1])
    assert calls == [(False, (1, 3, 12, 20))]
    loss = net.grid_l_loss_features
    assert calls[1] == (True, (2, 3, 12, 20)) and len(calls) == 2
    assert len(loss) == 1 and loss[0].shape == (1, 2, 8, 6, 10)
    assert torch.equal(loss[0][0, 1], 2 * grid[0])
    assert net.grid_l_loss_features is loss and len(calls) == 2  # computed once


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
    from scenedino_amd import _lib
    if conf.get("decoder_arch") == "dpt":  # the DPT writes the grid channels-last
        assert _lib.channels_last(out[0])
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


@pytest.mark.gpu
def test_dpt_level_fronts_on_side_streams_match_one_stream(gpu):
    """DINOv2Module can run the DPT's per-level fronts on side streams beside the later ViT
    blocks (overlap_levels; off by default, slower): the same kernels on the same operands,
    so the grid equals the one-stream order bit for bit, eager and graph-replayed."""
    m = make(seed=23).to(gpu)
    g = torch.Generator().manual_seed(24)
    xs = [(torch.rand(1, 3, 64, 160, generator=g) * 2 - 1).to(gpu) for _ in range(3)]
    outs = {}
    with torch.no_grad():
        for ov in (False, True):
            m.overlap_levels = ov
            for ug in (False, True):
                m.use_graph = ug
                m._graph = None
                outs[(ov, ug)] = [m(x)[0].clone() for x in xs]
    torch.cuda.synchronize()
    ref = outs[(False, False)]
    for key, o in outs.items():
        for a, b in zip(ref, o):
            assert torch.equal(a, b), key


@pytest.mark.gpu
def test_dpt_level_fronts_cold_pack_with_overlap(gpu):
    """The overlapped level fronts starting from a cold weight pack (the first forward of a
    fresh module with overlap on) equal the one-stream order: the pack is made on the main
    stream before any side stream starts."""
    xs = [(torch.rand(1, 3, 64, 160, generator=torch.Generator().manual_seed(25 + i)) * 2 - 1).to(gpu)
          for i in range(2)]
    with torch.no_grad():
        m1 = make(seed=26).to(gpu)
        m1.overlap_levels, m1.use_graph = True, False
        a = [m1(x)[0].clone() for x in xs]
        m2 = make(seed=26).to(gpu)
        m2.overlap_levels, m2.use_graph = False, False
        b = [m2(x)[0].clone() for x in xs]
    torch.cuda.synchronize()
    for u, v in zip(a, b):
        assert torch.equal(u, v)


MODEL_CONF = {"arch": "BTSNet", "predict_dino": True, "dino_dims": 64, "learn_empty": False,
              "code_mode": "z", "inv_z": True, "z_near": 3, "z_far": 80, "sample_color": True,
              "encoder": CONF, "code": {"num_freqs": 6, "freq_factor": 1.5, "include_input": True},
              "decoder_heads": [{"type": "resnet", "name": "normal_head", "freeze": False,
                                 "args": {"n_blocks": 0, "d_hidden": 128}}],
              "final_prediction_head": "normal_head", "precision": "bf16"}


@pytest.mark.gpu
def test_make_model_encode_render_end_to_end(gpu):
    """make_model builds the native encoder; encode() -> render reads the DPT grid exactly
    as a fixed-grid net holding the same grid does."""
    import _helpers
    from scenedino_amd.models import make_model
    from scenedino_amd.renderer import NeRFRenderer
    from scenedino_amd.common.ray_sampler import ImageRaySampler
    torch.manual_seed(31)
    net = make_model(MODEL_CONF)
    init_vit(net.encoder.encoder.model.vit, 32)
    det_fill(net.encoder.decoder, 33)
    net = net.to(gpu).eval()
    g = torch.Generator().manual_seed(34)
    imgs = (torch.rand(1, 1, 3, 64, 160, generator=g) * 2 - 1).to(gpu)
    Ks = torch.tensor([[0.7849, 0, -0.0312], [0, 2.9391, 0.2701], [0, 0, 1]], device=gpu).view(1, 1, 3, 3)
    poses = torch.eye(4, device=gpu).view(1, 1, 4, 4)
    with torch.no_grad():
        net.encode(imgs, Ks, poses, ids_encoder=[0], ids_render=[0])
        grid = net.grid_f_features[0][:, 0]
        assert grid.shape == (1, 256, 64, 160) and torch.isfinite(grid).all()
        assert torch.equal(grid, net.encoder(imgs[:, 0])[0])
        ref = _helpers.build_net(grid.cpu(), *(t.detach().cpu() for t in (
            net.heads["normal_head"].lin_in.weight, net.heads["normal_head"].lin_in.bias,
            net.heads["normal_head"].lin_out.weight, net.heads["normal_head"].lin_out.bias)),
            precision="bf16", device=gpu)
        ref.encode(imgs, Ks, poses, ids_encoder=[0], ids_render=[0])
        rays, _ = ImageRaySampler(3, 80, 64, 160).sample(None, poses, Ks)
        outs = []
        for n in (net, ref):
            r = NeRFRenderer(n_coarse=32, lindisp=True, hard_alpha_cap=False)
            torch.manual_seed(35)
            outs.append(r.bind_parallel(n, gpus=None).eval()(rays, want_weights=True)["coarse"])
    for k in ("depth", "dino_features", "weights"):
        assert torch.isfinite(outs[0][k]).all()
        assert torch.equal(outs[0][k], outs[1][k]), k


def test_default_precision_is_the_contract_meeting_one():
    """The reference's configs carry no precision key; the build then renders in fp16, the
    16-bit mode within SURVEY §8(c)'s 1e-2 m depth contract (bf16 is selectable)."""
    from scenedino_amd.models import make_model
    conf = {k: v for k, v in MODEL_CONF.items() if k != "precision"}
    assert make_model(conf).precision == "fp16"
    assert make_model(MODEL_CONF).precision == "bf16"
