"""Full-image ray sampler (mirror of scenedino.common.ray_sampler.ImageRaySampler,
/root/reference/scenedino/common/ray_sampler.py:421-607).

Ray generation runs in the bit-exact ``sd_gen_rays`` gfx950 kernel (replacing
util.unproj_map + util.gen_rays, util.py:113-158 / 253-285).  Output layout is the
reference's: (n, v*H*W, 11) = [o(3), d(3), near, far, frame_id, x_ndc, y_ndc],
row-major over (v, y, x).
"""
from __future__ import annotations

from math import isqrt

import torch

from .. import _lib


class RaySampler:
    def __init__(self, z_near: float, z_far: float) -> None:
        self.z_near = z_near
        self.z_far = z_far

    def sample(self, images, poses, projs):
        raise NotImplementedError

    def reconstruct(self, render_dict):
        raise NotImplementedError


class ImageRaySampler(RaySampler):
    def __init__(self, z_near: float, z_far: float, height: int | None = None,
                 width: int | None = None, channels: int = 3, norm_dir: bool = True,
                 dino_upscaled: bool = False) -> None:
        super().__init__(z_near, z_far)
        self.height, self.width = height, width
        self.channels = channels
        self.norm_dir = norm_dir
        self.dino_upscaled = dino_upscaled
        self._ids_cache = {}

    def sample(self, images, poses, projs, image_ids=None, dino_features=None,
               dino_artifacts=None):
        if not self.norm_dir:
            raise NotImplementedError("norm_dir=False is not used by any caller")
        n, v = poses.shape[:2]
        device = poses.device
        if images is not None:
            self.channels = images.shape[2]
        if self.height is None:
            self.height, self.width = images.shape[-2:]
        h, w = self.height, self.width
        if image_ids is None:
            key = (v, str(device))
            ids = self._ids_cache.get(key)
            if ids is None:
                ids = self._ids_cache[key] = torch.arange(v, device=device, dtype=torch.float32)
        else:
            ids = torch.tensor(image_ids, device=device, dtype=torch.float32)
        all_rays, all_rgb, all_dino = [], [], []
        for n_ in range(n):
            rays = _lib.gen_rays(poses[n_].reshape(-1, 4, 4).float().contiguous(),
                                 projs[n_].reshape(-1, 3, 3).float().contiguous(), ids, h, w,
                                 self.z_near, self.z_far)
            all_rays.append(rays.view(-1, 11))
            if images is not None:
                all_rgb.append(images[n_].view(-1, self.channels, h, w).permute(0, 2, 3, 1)
                               .reshape(-1, self.channels))
            if dino_features is not None:
                dc, ph, pw = dino_features.shape[-3:]
                all_dino.append(dino_features[n_].view(-1, dc, ph, pw).permute(0, 2, 3, 1)
                                .reshape(-1, dc))
        # a single frame is a view, not a copy (torch.stack would copy the rays)
        all_rays = all_rays[0].unsqueeze(0) if n == 1 else torch.stack(all_rays)
        if images is not None:
            all_rgb = all_rgb[0].unsqueeze(0) if n == 1 else torch.stack(all_rgb)
        else:
            all_rgb = None
        if dino_features is not None:
            return all_rays, all_rgb, torch.stack(all_dino)
        return all_rays, all_rgb

    def reconstruct(self, render_dict, channels=None, dino_channels=None):
        H, W = self.height, self.width
        n = v_in = None
        for name, part in render_dict.items():
            if not isinstance(part, dict) or "rgb" not in part:
                continue
            channels = self.channels if channels is None else channels
            n, n_pts, v_c = part["rgb"].shape
            v_in = n_pts // (H * W)
            v_r = v_c // channels
            k = part["weights"].shape[-1]
            part["rgb"] = part["rgb"].view(n, v_in, H, W, v_r, channels)
            part["weights"] = part["weights"].view(n, v_in, H, W, k)
            part["depth"] = part["depth"].view(n, v_in, H, W)
            part["invalid"] = part["invalid"].view(n, v_in, H, W, k, v_r)
            if "invalid_features" in part:
                part["invalid_features"] = part["invalid_features"].view(n, v_in, H, W, k, v_r)
            if "alphas" in part:
                part["alphas"] = part["alphas"].view(n, v_in, H, W, k)
            if "z_samps" in part:
                part["z_samps"] = part["z_samps"].view(n, v_in, H, W, k)
            if "rgb_samps" in part:
                part["rgb_samps"] = part["rgb_samps"].view(n, v_in, H, W, k, v_r, channels)
            if "ray_info" in part:
                part["ray_info"] = part["ray_info"].view(n, v_in, H, W, part["ray_info"].shape[-1])
            if "extras" in part:
                part["extras"] = part["extras"].view(n, v_in, H, W, part["extras"].shape[-1])
            if "dino_features" in part:
                part["dino_features"] = part["dino_features"].view(
                    n, v_in, H, W, 1, part["dino_features"].shape[-1])
            render_dict[name] = part
        if "rgb_gt" in render_dict:
            render_dict["rgb_gt"] = render_dict["rgb_gt"].view(n, v_in, H, W, channels)
        if "dino_gt" in render_dict:
            g = render_dict["dino_gt"]
            d = g.shape[-1]
            if self.dino_upscaled:
                render_dict["dino_gt"] = g.view(n, v_in, H, W, d)
            else:
                ps = isqrt((n * v_in * H * W * d) // g.numel())
                render_dict["dino_gt"] = g.view(n, v_in, H // ps, W // ps, d)
            if "dino_artifacts" in render_dict:  # ray_sampler.py:599-605
                art = render_dict["dino_artifacts"]
                ps = isqrt((n * v_in * H * W * d) // art.numel())
                render_dict["dino_artifacts"] = art.view(n, v_in, H // ps, W // ps, d)
        return render_dict
