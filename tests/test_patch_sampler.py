"""PatchRaySampler (ray_sampler.py:136-377): the host draws the patches
with the reference's own torch.randint calls, sd_patch_rays generates the sampled rays and
gathers the targets.  Fixture tests/golden/patch_sampler.npz = the reference's sampler on
seeded inputs (tests/golden/make_golden.py, fx_patch_sampler).  Rays, colour and DINO
targets: bit-exact."""
import numpy as np
import pytest
import torch

from _helpers import load
from oracle import render_oracle as O
from scenedino_amd.common.ray_sampler import PatchRaySampler

CASES = ["grid", "shift", "upscaled"]


def _case(d, name):
    rb, psy, psx, up, seed, s0, s1, has_shift = (int(x) for x in d[f"{name}_meta"])
    shift = torch.tensor([s0, s1]) if has_shift else None
    dino = torch.from_numpy(d["dino_up"] if up else d["dino"])
    return rb, (psy, psx), bool(up), seed, shift, dino


@pytest.mark.parametrize("name", CASES)
def test_host_draw_and_oracle_match_reference(name):
    d = load("patch_sampler.npz")
    rb, ps, up, seed, shift, dino = _case(d, name)
    images = torch.from_numpy(d["images"])
    n, v, c, h, w = images.shape
    smp = PatchRaySampler(3.0, 80.0, rb, ps, snap_to_grid=True, dino_upscaled=up)
    torch.manual_seed(seed)
    patches = smp._draw(n, v, h, w, tuple(dino.shape[-2:]), shift)
    rays, rgb, dg = O.patch_sample(images, torch.from_numpy(d["poses"]), torch.from_numpy(d["Ks"]),
                                   patches, ps[0], ps[1], dino=dino, dino_upscaled=up)
    assert torch.equal(rays, torch.from_numpy(d[f"{name}_rays"]))
    assert torch.equal(rgb, torch.from_numpy(d[f"{name}_rgb"]))
    assert torch.equal(dg, torch.from_numpy(d[f"{name}_dino"]))


def test_reconstruct_views():
    smp = PatchRaySampler(3.0, 80.0, 128, 8, snap_to_grid=True)
    n, K, D = 2, 16, 8
    rd = {"coarse": {"rgb": torch.zeros(n, 128, 3), "weights": torch.zeros(n, 128, K),
                     "depth": torch.zeros(n, 128), "invalid": torch.zeros(n, 128, K, 1),
                     "dino_features": torch.zeros(n, 128, D)},
          "rgb_gt": torch.zeros(n, 128, 3), "dino_gt": torch.zeros(n, 2, D)}
    out = smp.reconstruct(rd)
    assert out["coarse"]["rgb"].shape == (n, 2, 8, 8, 1, 3)
    assert out["coarse"]["dino_features"].shape == (n, 2, 8, 8, 1, D)
    assert out["dino_gt"].shape == (n, 2, D) and out["rgb_gt"].shape == (n, 2, 8, 8, 3)


def test_not_snapped_raises_like_reference():
    smp = PatchRaySampler(3.0, 80.0, 64, 8, snap_to_grid=False)
    with pytest.raises(NotImplementedError):
        smp._draw(1, 1, 24, 80, None, None)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_device_sampler_bit_exact(name):
    d = load("patch_sampler.npz")
    rb, ps, up, seed, shift, dino = _case(d, name)
    smp = PatchRaySampler(3.0, 80.0, rb, ps, snap_to_grid=True, dino_upscaled=up)
    torch.manual_seed(seed)
    rays, rgb, dg = smp.sample(torch.from_numpy(d["images"]).cuda(), torch.from_numpy(d["poses"]).cuda(),
                               torch.from_numpy(d["Ks"]).cuda(), dino_features=dino.cuda(),
                               loss_feature_grid_shift=shift)
    assert torch.equal(rays.cpu(), torch.from_numpy(d[f"{name}_rays"]))
    assert torch.equal(rgb.cpu(), torch.from_numpy(d[f"{name}_rgb"]))
    assert torch.equal(dg.cpu(), torch.from_numpy(d[f"{name}_dino"]))
    # the global RNG advanced exactly as the reference's did
    torch.manual_seed(seed)
    n, v, c, h, w = d["images"].shape
    smp._draw(n, v, h, w, tuple(dino.shape[-2:]), shift)
    after = torch.rand(4)
    torch.manual_seed(seed)
    smp.sample(torch.from_numpy(d["images"]).cuda(), torch.from_numpy(d["poses"]).cuda(),
               torch.from_numpy(d["Ks"]).cuda(), dino_features=dino.cuda(),
               loss_feature_grid_shift=shift)
    assert torch.equal(torch.rand(4), after)
