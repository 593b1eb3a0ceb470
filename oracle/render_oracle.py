"""render_oracle -- TEST INFRASTRUCTURE ONLY (the checker / CPU baseline, never shipped).

A pure-PyTorch CPU (fp32) restatement of SceneDINO's volumetric feature-field
render path, written from the reference's behaviour (citations are
/root/reference file:line).  Only tests/, __graft_entry__.smoke() and
bench.py's ``cpu_baseline`` leg may import this module.  It is pinned against
golden vectors produced by the reference itself (tests/golden/make_golden.py,
tests/test_oracle.py).

Layout conventions (same as the reference's tensors):
  rays   (R, 11)  [o(3), d(3), near, far, frame_id, x_ndc, y_ndc]
  grid   (B, C, Hf, Wf) feature grid of the single encoder view per batch element
  w2c_f  (B, 4, 4), K_f (B, 3, 3)   encoder view extrinsics / normalised intrinsics
  imgs   (B, nv, 3, H, W) colour images in [0, 1] (render views)
  w2c_c  (B, nv, 4, 4), K_c (B, nv, 3, 3)
  W_in (d_h, C+39), b_in (d_h), W_out (1+D, d_h), b_out (1+D)
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

EPS = 1e-3  # scenedino/common/cameras/pinhole.py:3


# --------------------------------------------------------------------------
# a1-a3: ray generation  (util.py:113-158, util.py:253-285, ray_sampler.py:439-513)
# --------------------------------------------------------------------------
def gen_rays(poses_c2w, Ks, H, W, z_near=3.0, z_far=80.0, frame_ids=None):
    """poses_c2w (v,4,4), Ks (v,3,3) -> rays (v*H*W, 11), row-major (v, y, x)."""
    v = poses_c2w.shape[0]
    pw, ph = 2.0 / W, 2.0 / H
    x = torch.linspace(-1 + 0.5 * pw, 1 - 0.5 * pw, W, dtype=torch.float32)
    y = torch.linspace(-1 + 0.5 * ph, 1 - 0.5 * ph, H, dtype=torch.float32)
    xs = x.view(1, 1, W).expand(v, H, W)
    ys = y.view(1, H, 1).expand(v, H, W)
    f = torch.stack((Ks[:, 0, 0], Ks[:, 1, 1]), -1).view(v, 1, 1, 2)
    c = torch.stack((Ks[:, 0, 2], Ks[:, 1, 2]), -1).view(v, 1, 1, 2)
    xy_img = torch.stack((xs, ys), -1)
    xy = (xy_img - c) / f
    d = torch.cat((xy, torch.ones_like(xs).unsqueeze(-1)), -1)
    d = d / torch.norm(d, dim=-1, keepdim=True)
    R = poses_c2w[:, None, None, :3, :3]
    dirs = torch.matmul(R, d.unsqueeze(-1))[..., 0]
    o = poses_c2w[:, None, None, :3, 3].expand(v, H, W, 3)
    if frame_ids is None:
        frame_ids = torch.arange(v, dtype=torch.float32)
    fid = frame_ids.view(v, 1, 1, 1).expand(v, H, W, 1)
    nf = torch.tensor([z_near, z_far], dtype=torch.float32).view(1, 1, 1, 2).expand(v, H, W, 2)
    rays = torch.cat((o, dirs, nf, fid, xy_img), -1)
    return rays.reshape(-1, 11)


def patch_sample(images, poses_c2w, Ks, patches, ph, pw, dino=None, dino_upscaled=False,
                 z_near=3.0, z_far=80.0):
    """PatchRaySampler.sample's gathers (ray_sampler.py:171-287) given the drawn patches
    (n, P, 4) = [view, y, x, DINO cell row * dino_w + col]: full-frame rays then the
    patch pixels, the rgb target and the DINO target (per pixel or per patch)."""
    n, v, c, h, w = images.shape
    rays_all, rgb_all, dino_all = [], [], []
    for b in range(n):
        rays = gen_rays(poses_c2w[b], Ks[b], h, w, z_near, z_far).view(v, h, w, 11)
        img = images[b].permute(0, 2, 3, 1)
        rr, cc, dd = [], [], []
        for vv, y, x, cell in patches[b].tolist():
            rr.append(rays[vv, y:y + ph, x:x + pw].reshape(-1, 11))
            cc.append(img[vv, y:y + ph, x:x + pw].reshape(-1, c))
            if dino is not None:
                dn = dino[b].permute(0, 2, 3, 1)
                if dino_upscaled:
                    dd.append(dn[vv, y:y + ph, x:x + pw].reshape(-1, dn.shape[-1]))
                else:
                    dd.append(dn[vv].reshape(-1, dn.shape[-1])[cell].view(1, -1))
        rays_all.append(torch.cat(rr))
        rgb_all.append(torch.cat(cc))
        if dino is not None:
            dino_all.append(torch.cat(dd))
    out = (torch.stack(rays_all), torch.stack(rgb_all))
    return out + ((torch.stack(dino_all),) if dino is not None else ())


# --------------------------------------------------------------------------
# a5: stratified z sampling (nerf.py:121-141), jitter u injected
# --------------------------------------------------------------------------
def sample_z(rays, K, u, lindisp=True):
    near, far = rays[:, 6:7], rays[:, 7:8]
    step = 1.0 / K
    t = torch.linspace(0, 1 - step, K).unsqueeze(0).expand(rays.shape[0], K) + u * step
    if lindisp:
        return 1 / (1 / near * (1 - t) + 1 / far * t)
    return near * (1 - t) + far * t


# --------------------------------------------------------------------------
# a8-a15: per-point field query (bts.py:271-441, bts.py:476-595, pinhole.py:40-112,
#          positional_encoding.py:13-80, resnetfc.py:135-203)
# --------------------------------------------------------------------------
def _project(xyz, w2c, K):
    """xyz (B,P,3); w2c (B,nv,4,4); K (B,nv,3,3) -> xy (B,nv,P,2), z (B,nv,P,1)."""
    B, P, _ = xyz.shape
    ph = torch.cat((xyz, torch.ones(B, P, 1)), -1)  # (B,P,4)
    cam = torch.einsum("bvij,bpj->bvpi", w2c[:, :, :3, :], ph)  # (B,nv,P,3)
    img = torch.einsum("bvij,bvpj->bvpi", K, cam)
    z = img[..., 2:3]
    xy = img[..., :2] / z.clamp_min(EPS)
    return xy, z


def _outside(xy, z):
    return (z <= EPS) | (xy[..., :1] < -1) | (xy[..., :1] > 1) | (xy[..., 1:2] < -1) | (xy[..., 1:2] > 1)


def positional_code(xy, z, d_min=3.0, d_max=80.0, num_freqs=6, freq_factor=1.5):
    """inverse-depth normalisation (positional_encoding.py:13-21) + Fourier code
    (positional_encoding.py:68-80): [x,y,z~, sin(f_j v + phi)] with j-major order."""
    zt = (1 / z.clamp_min(EPS) - 1 / d_max) / (1 / d_min - 1 / d_max)
    zt = 2 * zt - 1
    v = torch.cat((xy, zt), -1)  # (..., 3)
    freqs = freq_factor * 2.0 ** torch.arange(0, num_freqs)
    freqs = torch.repeat_interleave(freqs, 2).view(-1, 1).float()  # (12,1)
    phases = torch.zeros(2 * num_freqs)
    phases[1::2] = math.pi * 0.5
    phases = phases.view(-1, 1)
    # addcmul (positional_encoding.py:76): one fused multiply-add on CPU and GPU builds
    emb = torch.sin(torch.addcmul(phases, v.unsqueeze(-2).expand(*v.shape[:-1], 12, 3), freqs))
    return torch.cat((v, emb.flatten(-2)), -1)  # (..., 39)


def field_query(xyz, grid, w2c_f, K_f, imgs, w2c_c, K_c, W_in, b_in, W_out, b_out,
                with_colors=True, empty_feature=None):
    """xyz (B,P,3) -> dict(sigma (B,P), dino (B,P,D), rgb (B,P,3nv),
    invalid (B,P,nv) bool, invalid_features (B,P) bool).  ``empty_feature`` (C,): the
    learn_empty substitution of bts.py:311-319 (features of points outside the encoder
    frustum replaced by the learned vector)."""
    B, P, _ = xyz.shape
    C = grid.shape[1]
    xy, z = _project(xyz, w2c_f.unsqueeze(1), K_f.unsqueeze(1))  # (B,1,P,*)
    inv_f = _outside(xy, z)[:, 0, :, 0]  # (B,P)
    xy = xy.clamp(-2, 2)
    code = positional_code(xy[:, 0], z[:, 0])  # (B,P,39)
    feat = F.grid_sample(grid, xy.view(B, 1, P, 2), mode="bilinear", padding_mode="border",
                         align_corners=False).view(B, C, P).permute(0, 2, 1)
    if empty_feature is not None:
        feat = torch.where(inv_f.unsqueeze(-1), empty_feature.view(1, 1, C), feat)
    x = torch.cat((feat, code), -1)  # (B,P,C+39)
    h = torch.relu(x @ W_in.t() + b_in)
    out = h @ W_out.t() + b_out
    sigma = F.softplus(out[..., 0])
    dino = out[..., 1:]
    res = {"sigma": sigma, "dino": dino, "invalid_features": inv_f}
    if with_colors:
        nv = imgs.shape[1]
        H, W = imgs.shape[-2:]
        xyc, zc = _project(xyz, w2c_c, K_c)  # (B,nv,P,*)
        xyc = xyc.clamp(-2, 2)
        inv_c = _outside(xyc, zc)[..., 0]  # (B,nv,P)
        col = F.grid_sample(imgs.reshape(B * nv, 3, H, W), xyc.reshape(B * nv, 1, P, 2),
                            mode="bilinear", padding_mode="border", align_corners=False)
        col = col.view(B, nv, 3, P).permute(0, 3, 1, 2).reshape(B, P, nv * 3)
        inv = inv_c.permute(0, 2, 1) | inv_f.unsqueeze(-1)  # (B,P,nv)
        res["rgb"] = col
        res["invalid"] = inv
    return res


# --------------------------------------------------------------------------
# a6, a16: alpha compositing (nerf.py:246-253, nerf.py:343-405)
# --------------------------------------------------------------------------
def composite(z, sigma, dino, rgb, hard_alpha_cap=False):
    """z, sigma (R,K); dino (R,K,D); rgb (R,K,3nv) -> weights, alphas, depth, dino, rgb."""
    deltas = torch.cat((z[:, 1:] - z[:, :-1], 1e10 * torch.ones_like(z[:, :1])), -1)
    alphas = 1 - torch.exp(-deltas.abs() * torch.relu(sigma))
    if hard_alpha_cap:
        alphas = alphas.clone()
        alphas[:, -1] = 1
    T = torch.cumprod(torch.cat((torch.ones_like(alphas[:, :1]), 1 - alphas + 1e-10), -1), -1)
    w = alphas * T[:, :-1]
    return {
        "weights": w,
        "alphas": alphas,
        "depth": (w * z).sum(-1),
        "dino": (dino * w.unsqueeze(-1)).sum(-2),
        "rgb": (w.unsqueeze(-1) * rgb).sum(-2),
    }


def render(rays, u, grid, w2c_f, K_f, imgs, w2c_c, K_c, W_in, b_in, W_out, b_out,
           sb, lindisp=True, hard_alpha_cap=False, chunk_rays=None, empty_feature=None):
    """Full coarse render.  rays (SB*B', 11); grid (SB,C,h,w); per-superbatch cameras.
    Returns the reference's ``coarse`` dict layout (nerf.py:541-598)."""
    R = rays.shape[0]
    K = u.shape[1]
    z = sample_z(rays, K, u, lindisp)
    Rb = R // sb
    pts = (rays[:, None, :3] + z.unsqueeze(2) * rays[:, None, 3:6]).reshape(sb, Rb * K, 3)
    nv = imgs.shape[1]
    D = W_out.shape[0] - 1
    sig = torch.empty(sb, Rb * K)
    din = torch.empty(sb, Rb * K, D)
    col = torch.empty(sb, Rb * K, 3 * nv)
    inv = torch.empty(sb, Rb * K, nv, dtype=torch.bool)
    invf = torch.empty(sb, Rb * K, dtype=torch.bool)
    step = (chunk_rays or Rb) * K
    for s0 in range(0, Rb * K, step):
        sl = slice(s0, min(s0 + step, Rb * K))
        r = field_query(pts[:, sl], grid, w2c_f, K_f, imgs, w2c_c, K_c, W_in, b_in, W_out, b_out,
                        empty_feature=empty_feature)
        sig[:, sl], din[:, sl], col[:, sl] = r["sigma"], r["dino"], r["rgb"]
        inv[:, sl], invf[:, sl] = r["invalid"], r["invalid_features"]
    c = composite(z, sig.view(R, K), din.view(R, K, D), col.view(R, K, 3 * nv), hard_alpha_cap)
    return {
        "rgb": c["rgb"].view(sb, Rb, 3 * nv),
        "depth": c["depth"].view(sb, Rb),
        "invalid": inv.view(sb, Rb, K, nv).float(),
        "ray_info": rays[:, 8:].reshape(sb, Rb, 3),
        "weights": c["weights"].view(sb, Rb, K),
        "alphas": c["alphas"].view(sb, Rb, K),
        "z_samps": z.view(sb, Rb, K),
        "rgb_samps": col.view(sb, Rb, K, 3 * nv),
        "dino_features": c["dino"].view(sb, Rb, D),
        "invalid_features": invf.view(sb, Rb, K, 1),
    }
