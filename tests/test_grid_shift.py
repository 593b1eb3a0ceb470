"""loss_feature_grid_shift (bts.py:197-205, trainer.py:185-198): the trainer draws
``torch.randint(-p/2, p/2, (2,))`` every training step, BTSNet.encode edge-pads the loss
images by 8 and crops them at (8 + s0, 8 + s1) before the gt-encoder pass, and
PatchRaySampler.sample offsets its patches by the same shift.

torchvision (``transforms.Pad(8, padding_mode="edge")``, ``functional.crop``) is not
importable here, so no reference fixture pins the pad + crop: **parity unpinned**; it is
checked bit for bit against an index-clamp restatement of edge padding (out[i, j] =
img[clamp(i + s0), clamp(j + s1)]) and, outside the padded border, torchvision's
zero-filled crop window."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from scenedino_amd.models.bts import shift_loss_images

KN = torch.tensor([[0.7849, 0.0, -0.0312], [0.0, 2.9391, 0.2701], [0.0, 0.0, 1.0]])


def _edge_crop_np(img, s0, s1, h, w):
    """Restatement: edge padding by 8 then a crop at (8 + s0, 8 + s1) of size (h, w); rows /
    columns beyond the padded image are zero (torchvision's tensor crop)."""
    H, W = img.shape[-2:]
    out = np.zeros(img.shape[:-2] + (h, w), img.dtype)
    for i in range(h):
        pi = i + 8 + s0  # row in the padded image
        if not 0 <= pi < H + 16:
            continue
        for j in range(w):
            pj = j + 8 + s1
            if not 0 <= pj < W + 16:
                continue
            out[..., i, j] = img[..., min(max(pi - 8, 0), H - 1), min(max(pj - 8, 0), W - 1)]
    return out


@pytest.mark.parametrize("s0,s1", [(0, 0), (-8, 7), (3, -5), (-1, -1), (7, 0), (12, -11)])
def test_shift_loss_images_restatement(s0, s1):
    g = torch.Generator().manual_seed(s0 * 31 + s1)
    imgs = torch.rand(2, 1, 3, 24, 40, generator=g) * 2 - 1
    out = shift_loss_images(imgs, torch.tensor([s0, s1]), 24, 40)
    ref = _edge_crop_np(imgs.numpy(), s0, s1, 24, 40)
    assert out.shape == imgs.shape
    assert np.array_equal(out.numpy(), ref)


class _RecordingEncoder(torch.nn.Module):
    """Fixed feature grid for the encoder pass; for the gt pass (ground_truth=True) it records
    its input and returns a (n, D, h/8, w/8) DINO map computed from it, so the sampled DINO
    targets depend on the shifted images."""

    def __init__(self, grid, D=64, patch=8):
        super().__init__()
        self.register_buffer("grid", grid)
        self.latent_size = grid.shape[1]
        self.extra_outs = 0
        self.patch = patch
        self.register_buffer("proj", torch.randn(D, 3, generator=torch.Generator().manual_seed(11)))
        self.gt_inputs = []

    def forward(self, x, ground_truth=False):
        if not ground_truth:
            return [self.grid]
        self.gt_inputs.append(x.detach().clone())
        pooled = torch.nn.functional.avg_pool2d(x, self.patch)
        return [torch.einsum("dc,nchw->ndhw", self.proj.to(x.dtype), pooled)]


def _net(grid, device):
    from scenedino_amd.common.positional_encoding import PositionalEncoding
    from scenedino_amd.models import BTSNet
    from scenedino_amd.models.prediction_heads import ResnetFC
    torch.manual_seed(2)
    head = ResnetFC(d_in=grid.shape[1] + 39, d_out=65, n_blocks=0, d_hidden=128)
    conf = {"predict_dino": True, "dino_dims": 64, "learn_empty": False, "code_mode": "z",
            "inv_z": True, "z_near": 3, "z_far": 80, "sample_color": True, "precision": "fp32"}
    return BTSNet(conf, _RecordingEncoder(grid), PositionalEncoding(6, 3, 1.5, True),
                  {"normal_head": head}, final_pred_head="normal_head").to(device)


@pytest.mark.parametrize("shift", [torch.tensor([-3, 5]), torch.tensor([0, 0]), (0, 0), None])
def test_encode_shifts_gt_input_cpu(shift):
    """BTSNet.encode on CPU tensors (the encoder pass and the deferred gt pass are host
    code): the gt-encoder input is the pad + crop of the loss images; a zero shift (tensor or
    tuple) and no shift leave them as they are."""
    g = torch.Generator().manual_seed(4)
    images = torch.rand(2, 1, 3, 24, 40, generator=g) * 2 - 1
    net = _net(torch.randn(2, 256, 6, 20, generator=g), "cpu")
    Ks = KN.view(1, 1, 3, 3).expand(2, 1, 3, 3)
    poses = torch.eye(4).view(1, 1, 4, 4).expand(2, 1, 4, 4)
    net.encode(images, Ks, poses, ids_encoder=[0], ids_render=[0], ids_loss=[0],
               loss_feature_grid_shift=shift)
    assert net.encoder.gt_inputs == []  # deferred until the loss reads it
    lf = net.grid_l_loss_features
    assert lf[0].shape == (2, 1, 64, 3, 5)
    got = net.encoder.gt_inputs[0]
    s = (0, 0) if shift is None else tuple(int(v) for v in shift)
    ref = _edge_crop_np(images[:, 0].numpy(), s[0], s[1], 24, 40)
    assert np.array_equal(got.numpy(), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("amp", [torch.float16, None])
def test_reference_shaped_training_step_with_shift_gpu(amp):
    """One training step shaped like trainer.py:180-260 with loss_feature_grid_shift:
    encode(shift) -> grid_l_loss_features -> PatchRaySampler.sample(shift) -> render
    (want_weights / want_alphas / want_rgb_samps, as the trainer asks) -> loss.backward()
    -> Adam.  The gt-encoder input equals the pad + crop restatement bit for bit, the DINO
    targets equal the oracle patch gather of the shifted gt map, every gradient is finite
    and the head parameters move."""
    from oracle import render_oracle as O
    from scenedino_amd.common.ray_sampler import PatchRaySampler
    from scenedino_amd.renderer import NeRFRenderer
    dev = "cuda"
    NB, H, W, PS, RB, KT = 2, 48, 160, 8, 512, 32
    g = torch.Generator().manual_seed(8)
    images = (torch.rand(NB, 1, 3, H, W, generator=g) * 2 - 1).to(dev)
    grid = torch.randn(NB, 256, H // 2, W // 2, generator=g).to(dev)
    net = _net(grid, dev)
    Ks = KN.view(1, 1, 3, 3).expand(NB, 1, 3, 3).contiguous().to(dev)
    poses = torch.eye(4).view(1, 1, 4, 4).expand(NB, 1, 4, 4).contiguous().to(dev)
    torch.manual_seed(123)
    shift = torch.randint(-PS // 2, PS // 2, (2,))  # trainer.py:186-187 (patch_size // 2)
    if int(shift[0]) == 0 and int(shift[1]) == 0:
        shift = torch.tensor([-2, 3])
    net.train()
    net.encode(images, Ks, poses, ids_encoder=[0], ids_render=[0], ids_loss=[0],
               loss_feature_grid_shift=shift)
    leaf = net.grid_f_features[0].detach().clone().requires_grad_(True)
    net.grid_f_features[0] = leaf
    dino_map = net.grid_l_loss_features[0]
    gt_in = net.encoder.gt_inputs[0].cpu()
    ref = _edge_crop_np(images[:, 0].cpu().numpy(), int(shift[0]), int(shift[1]), H, W)
    assert np.array_equal(gt_in.numpy(), ref)

    sampler = PatchRaySampler(3, 80, RB, PS, snap_to_grid=True, dino_upscaled=False)
    torch.manual_seed(7)
    rays, rgb_gt, dino_gt = sampler.sample(images, poses, Ks, dino_features=dino_map,
                                           loss_feature_grid_shift=shift)
    torch.manual_seed(7)
    patches = sampler._draw(NB, 1, H, W, tuple(dino_map.shape[-2:]), shift)
    o_rays, o_rgb, o_dino = O.patch_sample(images.cpu(), poses.cpu(), Ks.cpu(), patches, PS, PS,
                                           dino=dino_map.cpu(), dino_upscaled=False)
    assert torch.equal(rays.cpu(), o_rays) and torch.equal(rgb_gt.cpu(), o_rgb)
    assert torch.equal(dino_gt.cpu(), o_dino)

    head = net.heads["normal_head"]
    before = [p.detach().clone() for p in head.parameters()]
    opt = torch.optim.Adam(head.parameters(), lr=1e-3)
    wrapper = NeRFRenderer(n_coarse=KT, lindisp=True, hard_alpha_cap=True,
                           eval_batch_size=65536).bind_parallel(net, gpus=None).train()
    with torch.autocast("cuda", dtype=amp or torch.float16, enabled=amp is not None):
        out = wrapper(rays, want_weights=True, want_alphas=True, want_rgb_samps=True)["coarse"]
        npatch = RB // (PS * PS)
        pd = out["dino_features"].float().view(NB, npatch, PS * PS, -1).mean(2)
        loss = ((pd - dino_gt) ** 2).mean() + \
            (out["rgb"].float() - (rgb_gt * 0.5 + 0.5)).abs().mean()
    assert out["rgb_samps"].shape[:2] == (NB, RB) and out["alphas"].shape == (NB, RB, KT)
    opt.zero_grad()
    loss.backward()
    assert leaf.grad is not None and bool(torch.isfinite(leaf.grad).all())
    assert float(leaf.grad.abs().sum()) > 0
    for p in head.parameters():
        assert p.grad is not None and bool(torch.isfinite(p.grad).all())
    opt.step()
    assert all(not torch.equal(p.detach(), b) for p, b in zip(head.parameters(), before))
