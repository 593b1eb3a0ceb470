"""CPU: pin the oracle (C restatement + torch-CPU restatement) against the golden
vectors produced by the reference itself (tests/golden/make_golden.py)."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from _helpers import load
from oracle import coracle
from oracle import render_oracle as O


def test_c_oracle_gen_rays_small():
    d = load("gen_rays_small.npz")
    out = coracle.gen_rays(d["poses"], d["projs"], 24, 80)
    assert np.array_equal(out.reshape(-1, 11), d["rays"][0])


def test_c_oracle_gen_rays_full_sha256():
    j = json.load(open(os.path.join(GOLDEN, "gen_rays_full.json")))
    K = np.array(j["K"], np.float32)[None]
    for name, c in j["cases"].items():
        out = coracle.gen_rays(np.array(c["pose"], np.float32)[None], K, 192, 640)
        assert hashlib.sha256(out.tobytes()).hexdigest() == c["sha256"], name


@pytest.mark.parametrize("K", [8, 32, 64, 128])
@pytest.mark.parametrize("lindisp", [1, 0])
def test_c_oracle_sample_z(K, lindisp):
    d = load("sample_z.npz")
    z = coracle.sample_z(d["rays"], K, d[f"u_{K}"], bool(lindisp))
    assert np.array_equal(z, d[f"z_{K}_{lindisp}"])


def test_torch_oracle_gen_rays_and_z():
    d = load("gen_rays_small.npz")
    rays = O.gen_rays(torch.from_numpy(d["poses"]), torch.from_numpy(d["projs"]), 24, 80)
    assert torch.equal(rays, torch.from_numpy(d["rays"][0]))
    s = load("sample_z.npz")
    z = O.sample_z(torch.from_numpy(s["rays"]), 64, torch.from_numpy(s["u_64"]), True)
    assert torch.equal(z, torch.from_numpy(s["z_64_1"]))


@pytest.mark.parametrize("fx", ["field_query.npz", "field_query_empty.npz"])
def test_torch_oracle_field_query_bit_exact(fx):
    d = load(fx)
    T = torch.from_numpy
    w2c = torch.inverse(T(d["poses"]))
    r = O.field_query(T(d["xyz"]), T(d["grid"]), w2c[:, 0], T(d["Ks"])[:, 0],
                      T(d["images"]) * 0.5 + 0.5, w2c, T(d["Ks"]), T(d["W_in"]), T(d["b_in"]),
                      T(d["W_out"]), T(d["b_out"]),
                      empty_feature=T(d["empty_feature"]) if "empty_feature" in d else None)
    assert torch.equal(r["sigma"], T(d["sigma"])[..., 0])
    assert torch.equal(r["dino"], T(d["dino"]))
    assert torch.equal(r["rgb"], T(d["rgb"]))
    assert torch.equal(r["invalid"].float(), T(d["invalid"]))


@pytest.mark.parametrize("fx", ["render_k32_cap0.npz", "render_k64_cap1.npz",
                                "render_sb2_nv2_k16.npz", "render_sb2_k32_empty.npz"])
def test_torch_oracle_render_matches_reference(fx):
    d = load(fx)
    T = torch.from_numpy
    poses, Ks = T(d["poses"]), T(d["Ks"])
    nv = int(d["nv_render"])
    w2c = torch.inverse(poses)
    sb = poses.shape[0]
    out = O.render(T(d["rays"]).reshape(-1, 11), T(d["u"]), T(d["grid"]), w2c[:, 0], Ks[:, 0],
                   T(d["images"])[:, :nv] * 0.5 + 0.5, w2c[:, :nv], Ks[:, :nv], T(d["W_in"]),
                   T(d["b_in"]), T(d["W_out"]), T(d["b_out"]), sb=sb,
                   hard_alpha_cap=bool(d["hard_cap"]),
                   empty_feature=T(d["empty_feature"]) if "empty_feature" in d else None)
    for k in ("rgb", "depth", "invalid", "weights", "alphas", "z_samps", "rgb_samps",
              "dino_features", "ray_info"):
        ref = T(d[k])
        assert torch.allclose(out[k].reshape(ref.shape), ref, rtol=1e-5, atol=1e-6), k
    ref_if = T(d["invalid_features"])
    assert torch.equal(out["invalid_features"].reshape(ref_if.shape), ref_if)


def test_render_full_subsample_fixture_consistent():
    d = load("render_full_subsample.npz")
    assert d["depth"].shape == d["idx"].shape and d["dino"].shape == (d["idx"].shape[0], 64)
    assert np.isfinite(d["dino"]).all()


@pytest.mark.parametrize("fx", ["render_full_offset_k32.npz", "render_c4_offset.npz"])
def test_torch_oracle_full_frame_offset_fixtures(fx):
    """BASELINE configs[0] (K = 32) and configs[3] (K = 128, 384-d field) full-frame renders
    of the reference (make_golden.fx_render_full_offset_k32 / fx_render_c4_offset): the
    oracle on the fixture's rays of the 192x640 offset-pose frame (rays are independent)."""
    from _fullscene import scene_arrays, KITTI_K
    d = load(fx)
    K = int(d["K"])
    D = int(d["D"]) if "D" in d else 64
    images, grid, (W_in, b_in, W_out, b_out) = scene_arrays(
        int(d["scene_seed"]), D=D, weights=d if "W_in" in d else None)
    Kn = torch.tensor(KITTI_K).view(1, 3, 3)
    pose = torch.from_numpy(d["render_pose"]).view(1, 4, 4)
    rays = O.gen_rays(pose, Kn, 192, 640)
    u = torch.rand(rays.shape[0], K, generator=torch.Generator().manual_seed(int(d["u_seed"])))
    it = torch.from_numpy(d["idx"])
    w2c = torch.eye(4).view(1, 4, 4)
    with torch.no_grad():
        out = O.render(rays[it], u[it], grid, w2c, Kn, images * 0.5 + 0.5, w2c.view(1, 1, 4, 4),
                       Kn.view(1, 1, 3, 3), W_in, b_in, W_out, b_out, sb=1)
    atol = {"depth": 1e-6, "weights": 1e-5, "alphas": 1e-4, "rgb": 1e-5, "dino": 5e-5}
    for k, rk in (("depth", "depth"), ("weights", "weights"), ("alphas", "alphas"),
                  ("rgb", "rgb"), ("dino_features", "dino")):
        ref = torch.from_numpy(d[rk])
        assert torch.allclose(out[k].reshape(ref.shape), ref, rtol=1e-5, atol=atol[rk]), k
    if "invalid" in d:
        assert torch.equal(out["invalid"].reshape(-1).bool(), torch.from_numpy(d["invalid"]).reshape(-1).bool())
