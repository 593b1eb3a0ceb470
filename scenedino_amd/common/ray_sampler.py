"""Ray samplers (mirrors of scenedino.common.ray_sampler.ImageRaySampler,
/root/reference/scenedino/common/ray_sampler.py:421-607, and PatchRaySampler, :136-377).

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


class PatchRaySampler(RaySampler):
    """Training batches of square-grid patches (ray_sampler.py:136-377).

    ``sample`` draws the patch positions with exactly the reference's torch.randint calls
    (global CPU generator, same order: per frame view / row / column), so a seeded run picks
    the same patches; the rays of only the sampled pixels, the rgb target and the DINO
    target are then produced on the device by ``sd_patch_rays`` (rays bit-exact with
    util.gen_rays).  ``snap_to_grid=False`` raises NotImplementedError after drawing, as the
    reference does (:234-235)."""

    def __init__(self, z_near: float, z_far: float, ray_batch_size: int, patch_size,
                 channels: int = 3, snap_to_grid: bool = False, dino_upscaled: bool = False):
        super().__init__(z_near, z_far)
        self.ray_batch_size = ray_batch_size
        self.channels = channels
        self.snap_to_grid = snap_to_grid
        self.dino_upscaled = dino_upscaled
        if isinstance(patch_size, int):
            self.patch_size_x, self.patch_size_y = patch_size, patch_size
        elif isinstance(patch_size, (tuple, list)):
            self.patch_size_y, self.patch_size_x = patch_size[0], patch_size[1]
        else:
            raise ValueError("Invalid format for patch size")
        assert (ray_batch_size % (self.patch_size_x * self.patch_size_y)) == 0
        self._patch_count = self.ray_batch_size // (self.patch_size_x * self.patch_size_y)
        self._ids_cache = {}
        self._ring = [None, None]  # pinned host staging of the drawn patches (+ copy event)
        self._slot = 0

    def _draw(self, n, v, h, w, dino_hw, loss_feature_grid_shift):
        """The reference's per-frame randint draws (:215-226) -> (n, patches, 4) int32:
        [view, y, x, DINO cell row * dino_w + col] (:228-245)."""
        psy, psx, pc = self.patch_size_y, self.patch_size_x, self._patch_count
        shift = None
        if loss_feature_grid_shift is not None:
            shift = [int(t) for t in loss_feature_grid_shift]
        out = torch.empty(n, pc, 4, dtype=torch.int32)
        for n_ in range(n):
            cv = torch.randint(0, v, (pc,))
            if self.snap_to_grid:
                if shift is not None:
                    cy = torch.randint(0, h // psy - 1, (pc,))
                    cx = torch.randint(0, w // psx - 1, (pc,))
                else:
                    cy = torch.randint(0, h // psy, (pc,))
                    cx = torch.randint(0, w // psx, (pc,))
            else:
                torch.randint(0, h - psy, (pc,))
                torch.randint(0, w - psx, (pc,))
                raise NotImplementedError
            if shift is not None:
                y = (shift[0] % psy) + psy * cy
                x = (shift[1] % psx) + psx * cx
                gy = cy + (1 if shift[0] < 0 else 0)
                gx = cx + (1 if shift[1] < 0 else 0)
            else:
                y, x, gy, gx = psy * cy, psx * cx, cy, cx
            dw = dino_hw[1] if dino_hw is not None else 0
            out[n_] = torch.stack((cv, y, x, gy * dw + gx), 1).to(torch.int32)
        return out

    def _upload(self, patches, device):
        """Host -> device copy of the drawn patches through a 2-slot pinned ring: a copy from
        pageable memory would block the host until the stream drained (a device sync per
        training step); a slot is reused only after its previous copy has completed."""
        slot = self._slot
        self._slot ^= 1
        ent = self._ring[slot]
        if ent is None or ent[0].shape != patches.shape:
            ent = self._ring[slot] = [torch.empty(patches.shape, dtype=patches.dtype,
                                                  pin_memory=True), None]
        if ent[1] is not None:
            ent[1].synchronize()
        ent[0].copy_(patches)
        out = ent[0].to(device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(device))
        ent[1] = ev
        return out

    def sample(self, images, poses, projs, image_ids=None, dino_features=None,
               loss_feature_grid_shift=None):
        patches = self.draw(images, dino_features, loss_feature_grid_shift)
        if images.device.type != "cuda":
            raise RuntimeError("PatchRaySampler: the device sampler needs CUDA (HIP) tensors")
        patches = self._upload(patches, images.device)
        return self.sample_patches(patches, images, poses, projs, image_ids, dino_features)

    def draw(self, images, dino_features=None, loss_feature_grid_shift=None):
        """The host half of ``sample``: the reference's randint draws as a (n, patches, 4)
        int32 CPU tensor (``sample_patches`` takes them once they are on the device)."""
        n, v, c, h, w = images.shape
        dino_hw = tuple(dino_features.shape[-2:]) if dino_features is not None else None
        return self._draw(n, v, h, w, dino_hw, loss_feature_grid_shift)

    def sample_patches(self, patches, images, poses, projs, image_ids=None, dino_features=None):
        """The device half of ``sample``: rays / colour (and DINO) targets of the drawn
        patches (a device int32 tensor from ``draw``).  No host synchronisation and no
        host-to-device copy: a training step can be captured into a HIP graph from here on
        (the patch draws stay on the host, copied into the graph's input buffer each step)."""
        n, v, c, h, w = images.shape
        self.channels = c
        device = images.device
        psy, psx, pc = self.patch_size_y, self.patch_size_x, self._patch_count
        dino_hw = tuple(dino_features.shape[-2:]) if dino_features is not None else None
        if image_ids is None:
            key = (v, str(device))
            ids = self._ids_cache.get(key)
            if ids is None:
                ids = self._ids_cache[key] = torch.arange(v, device=device, dtype=torch.float32)
        else:
            ids = torch.tensor(image_ids, device=device, dtype=torch.float32)
        npts = pc * psy * psx
        poses_f = poses.float().contiguous()
        Ks_f = projs.float().contiguous()
        imgs = images.float().contiguous()
        rays = torch.empty(n, npts, 11, device=device)
        rgb = torch.empty(n, npts, c, device=device)
        a = _lib.SdPatchArgs(
            poses=poses_f.data_ptr(), Ks=Ks_f.data_ptr(), frame_ids=ids.data_ptr(),
            patches=patches.data_ptr(), images=imgs.data_ptr(), rays=rays.data_ptr(),
            rgb_out=rgb.data_ptr(), B=n, V=v, H=h, W=w, n_patches=pc, ph=psy, pw=psx,
            channels=c, z_near=float(self.z_near), z_far=float(self.z_far))
        dino_gt = None
        if dino_features is not None:
            dc = dino_features.shape[2]
            dino = dino_features.float().contiguous()
            dino_gt = torch.empty(n, npts if self.dino_upscaled else pc, dc, device=device)
            a.dino, a.dino_out = dino.data_ptr(), dino_gt.data_ptr()
            a.dino_c, a.dino_h, a.dino_w = dc, dino_hw[0], dino_hw[1]
            a.dino_upscaled = int(bool(self.dino_upscaled))
        _lib.patch_rays(a, rays)
        if dino_features is not None:
            return rays, rgb, dino_gt
        return rays, rgb

    def reconstruct(self, render_dict, channels=None, dino_channels=None):
        """:289-377: reshape the flat patch batch into (n, patches, ph, pw, ...) views."""
        psy, psx, pc = self.patch_size_y, self.patch_size_x, self._patch_count
        n = None
        for name, part in render_dict.items():
            if not isinstance(part, dict) or "rgb" not in part:
                continue
            channels = self.channels if channels is None else channels
            rgb_gt = render_dict["rgb_gt"]
            dino_gt = render_dict["dino_gt"]
            n, n_pts, v_c = part["rgb"].shape
            v = v_c // channels
            k = part["weights"].shape[-1]
            part["rgb"] = part["rgb"].view(n, pc, psy, psx, v, channels)
            part["weights"] = part["weights"].view(n, pc, psy, psx, k)
            part["depth"] = part["depth"].view(n, pc, psy, psx)
            part["invalid"] = part["invalid"].view(n, pc, psy, psx, k, v)
            if "alphas" in part:
                part["alphas"] = part["alphas"].view(n, pc, psy, psx, k)
            if "z_samps" in part:
                part["z_samps"] = part["z_samps"].view(n, pc, psy, psx, k)
            if "rgb_samps" in part:
                part["rgb_samps"] = part["rgb_samps"].view(n, pc, psy, psx, k, v, channels)
            if "ray_info" in part:
                part["ray_info"] = part["ray_info"].view(n, pc, psy, psx, part["ray_info"].shape[-1])
            if "extras" in part:
                part["extras"] = part["extras"].view(n, pc, psy, psx, part["extras"].shape[-1])
            if "dino_features" in part:
                part["dino_features"] = part["dino_features"].view(
                    n, pc, psy, psx, 1, part["dino_features"].shape[-1])
            render_dict[name] = part
        render_dict["rgb_gt"] = rgb_gt.view(n, pc, psy, psx, channels)
        d = dino_gt.shape[-1]
        if self.dino_upscaled:
            render_dict["dino_gt"] = dino_gt.view(n, pc, psy, psx, d)
        else:
            render_dict["dino_gt"] = dino_gt.view(n, pc, d)
        if "dino_artifacts" in render_dict:
            render_dict["dino_artifacts"] = render_dict["dino_artifacts"].view(n, pc, d)
        return render_dict


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
