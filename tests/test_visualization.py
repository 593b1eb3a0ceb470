"""The encoder's visualization API (dinov2_module.py:156,194-201; visualization.py:9-153).

CPU: the restatement against ``tests/golden/visualization.npz``, written by running the
reference's own ``VisualizationModule`` in this container (make_golden.py
``fx_visualization``; pykeops stubbed by the dense equivalent of ``x_i | c_j`` +
``argmax``): the PCA fit under the same seeded RNG (tolerance 1e-5 -- the same op
sequence; 1e-4 absolute across CPUs, whose LAPACK / BLAS builds round the SVD differently),
``transform_pca`` in every (norm, from_dim) the callers
use, the cosine k-means colour map (bit-exact) and centres; tab10 against matplotlib.
GPU: ``demo_script.py:29-78``'s call sequence on ``make_model``'s native encoder (random
weights): encode, inference_rendered_2d, fit_visualization, transform_visualization at
from_dim 0 / 3 / 6, inference_3d on a small grid, transform_visualization of the 3-D
features -- no AttributeError, finite outputs, the colours equal to the centred projection
by the device-fitted state.
"""
import os

import numpy as np
import pytest
import torch

from scenedino_amd.models.backbones.dino.visualization import VisualizationModule, tab10

GOLD = os.path.join(os.path.dirname(__file__), "golden", "visualization.npz")


def _fx():
    return np.load(GOLD)


def test_pca_fit_and_transform_vs_reference():
    d = _fx()
    vis = VisualizationModule(768)
    torch.manual_seed(92)
    vis.fit_pca(torch.from_numpy(d["feats"]), refit=True)
    np.testing.assert_allclose(vis.batch_rgb_mean.numpy(), d["mean"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(vis.batch_rgb_comp.numpy(), d["comp"], rtol=1e-4, atol=1e-4)
    img = torch.from_numpy(d["img"])
    for fd in (0, 3, 6):
        for norm in (False, True):
            np.testing.assert_allclose(vis.transform_pca(img, norm, fd).numpy(),
                                       d[f"t_{fd}_{int(norm)}"], rtol=1e-3, atol=2e-4)


def test_transform_is_centred_projection():
    """transform_pca = (f - mean) @ comp[..., d:d+3], the norm branch dividing first."""
    vis = VisualizationModule(16)
    g = torch.Generator().manual_seed(3)
    vis.batch_rgb_mean = torch.randn(1, 16, generator=g)
    vis.batch_rgb_comp = torch.randn(16, 9, generator=g)
    f = torch.randn(5, 7, 16, generator=g)
    c = f - vis.batch_rgb_mean
    for fd in (0, 3, 6):
        assert torch.allclose(vis.transform_pca(f, False, fd), c @ vis.batch_rgb_comp[:, fd:fd + 3])
        cn = c / c.norm(dim=-1, keepdim=True)
        assert torch.allclose(vis.transform_pca(f, True, fd), cn @ vis.batch_rgb_comp[:, fd:fd + 3])


def test_fit_rejects_batched_input_and_skips_refit():
    vis = VisualizationModule(16)
    with pytest.raises(ValueError):
        vis.fit_pca(torch.randn(2, 10, 16), refit=True)
    vis.fit_pca(torch.randn(50, 16), refit=True)
    comp = vis.batch_rgb_comp.clone()
    vis.fit_pca(torch.randn(50, 16) + 5, refit=False)  # fitted already: kept
    assert torch.equal(vis.batch_rgb_comp, comp)


def test_kmeans_colour_map_vs_reference():
    d = _fx()
    vis = VisualizationModule(768)
    m = vis.fit_transform_kmeans_batch(torch.from_numpy(d["km_in"]))
    assert m.shape == d["km_map"].shape
    np.testing.assert_array_equal(m.numpy(), d["km_map"])
    np.testing.assert_allclose(vis.kmeans_cluster_centers.numpy(), d["km_centers"], rtol=1e-5,
                               atol=1e-6)


def test_tab10_matches_matplotlib():
    mpl = pytest.importorskip("matplotlib")
    cmap = mpl.colormaps["tab10"]
    for n in (8, 19):
        x = (np.arange(n, dtype=np.float32) / np.float32(n - 1))
        np.testing.assert_array_equal(tab10(x), cmap(x)[..., :3])


def test_native_module_exposes_the_api():
    from test_encoder import make
    m = make()
    assert isinstance(m.visualization, VisualizationModule)
    assert m.visualization.n_kmeans_clusters == 8
    f = torch.randn(300, 768)
    m.fit_visualization(f)
    assert m.transform_visualization(f.view(10, 30, 768), from_dim=6).shape == (10, 30, 3)
    m.visualization.n_kmeans_clusters = 4  # trainer_downstream.py:58 sets it from outside
    assert m.fit_transform_kmeans_visualization(f.view(10, 30, 1, 768)).shape == (10, 30, 3)


# ------------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_demo_script_call_sequence_on_native_encoder():
    """demo_script.py:29-78 with demo_utils.utils.inference_rendered_2d (:199-236) and
    inference_3d (:144-186) restated inline, on make_model's native encoder."""
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    from scenedino_amd import _lib
    _lib.load()
    from test_dpt import det_fill
    from test_encoder import MODEL_CONF
    from test_vit import init_vit
    from scenedino_amd.common.ray_sampler import ImageRaySampler
    from scenedino_amd.downstream_head import SemanticHead
    from scenedino_amd.models import make_model
    from scenedino_amd.renderer import NeRFRenderer
    dev = "cuda"
    torch.manual_seed(41)
    # the ViT-S encoder's full feature width (dim_reduction 64 <-> 384) is the head's input
    head = SemanticHead(19, 19, 384, 64).eval()
    net = make_model(MODEL_CONF, downstream_head=head)
    init_vit(net.encoder.encoder.model.vit, 42)
    det_fill(net.encoder.decoder, 43)
    net = net.to(dev).eval()
    H, W = 64, 160
    g = torch.Generator().manual_seed(44)
    images = (torch.rand(1, 1, 3, H, W, generator=g) * 2 - 1).to(dev)
    projs = torch.tensor([[0.7849, 0, -0.0312], [0, 2.9391, 0.2701], [0, 0, 1]],
                         device=dev).view(1, 1, 3, 3)
    poses = torch.eye(4, device=dev).view(1, 1, 4, 4)
    renderer = NeRFRenderer(n_coarse=32, lindisp=True, hard_alpha_cap=False).bind_parallel(net, gpus=None).eval()
    sampler = ImageRaySampler(3, 80, H, W)
    with torch.no_grad():
        net.encode(images, projs, poses, ids_encoder=[0])
        net.set_scale(0)
        # inference_rendered_2d
        rays, _ = sampler.sample(None, poses[:, :], projs[:, :])
        rd = sampler.reconstruct(renderer(rays, want_weights=True, want_alphas=True))
        depth_2d = rd["coarse"]["depth"].squeeze()
        dino_full_2d = net.encoder.expand_dim(rd["coarse"]["dino_features"].squeeze())
        seg_2d = net.downstream_head(dino_full_2d, mode="stego_kmeans")
        assert dino_full_2d.shape == (H, W, 384) and depth_2d.shape == (H, W)
        assert seg_2d is not None and seg_2d.shape[:2] == (H, W)
        net.encoder.fit_visualization(dino_full_2d.flatten(0, -2))
        pcas = [net.encoder.transform_visualization(dino_full_2d, from_dim=fd).permute(2, 0, 1)
                for fd in (0, 3, 6)]
        for p in pcas:
            assert p.shape == (3, H, W) and torch.isfinite(p).all()
        vis = net.encoder.visualization  # fitted on the device, state on the device
        assert vis.batch_rgb_comp.is_cuda and vis.batch_rgb_comp.shape == (384, 9)
        want = (dino_full_2d - vis.batch_rgb_mean) @ vis.batch_rgb_comp[:, 3:6]
        assert torch.allclose(pcas[1].permute(1, 2, 0), want)
        # inference_3d on a small grid (demo: 101 x 51 x 101 at 0.2 m; here 1 m)
        xs = torch.linspace(-10, 10, 21)
        ys = torch.linspace(-5, 5, 11)
        zs = torch.linspace(0, 20, 21)
        gx, gy, gz = torch.meshgrid(xs, ys, zs, indexing="ij")
        xyz = torch.stack((gx, gy, gz), dim=-1).reshape(-1, 3).unsqueeze(0).to(dev)
        dino_full, _, sigma, seg = net(xyz, predict_segmentation=True, prediction_mode="stego_kmeans")
        dino_full_3d = dino_full.reshape(21, 11, 21, -1)
        assert sigma.reshape(21, 11, 21).shape == (21, 11, 21)
        assert seg.reshape(21, 11, 21, -1).argmax(-1).shape == (21, 11, 21)
        pca_3d = net.encoder.transform_visualization(dino_full_3d, from_dim=0)
        assert pca_3d.shape == (21, 11, 21, 3) and torch.isfinite(pca_3d).all()
