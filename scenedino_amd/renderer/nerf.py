"""NeRF volume renderer, MI355X-native.

Mirror of scenedino.renderer.nerf.NeRFRenderer / _RenderWrapper
(/root/reference/scenedino/renderer/nerf.py:12-658): same constructor, ``from_conf``
keys, mutable attributes, persistent buffers (``iter_idx``, ``last_sched``),
``bind_parallel`` and output dictionary.

Hot path:
  * ``sample_coarse``  -> ``sd_sample_z`` (bit-exact given the jitter; perf mode
    draws the jitter from an on-device counter RNG seeded from torch's CPU RNG);
  * ``composite``      -> for a BTSNet from this package, ONE fused kernel
    (``sd_render_fused``: points, projection, code, gather, MFMA MLP, colours and
    alpha compositing); for any other field callable, the reference's chunked model
    calls followed by the ``sd_composite`` kernel.

Parity hook: set ``renderer.z_jitter = u`` (tensor (SB*B, K) in [0,1)) to replace
the reference's ``torch.rand_like`` draw (nerf.py:134) with given values.
"""
from __future__ import annotations

import os

import torch

from .. import _lib, autograd


class _RenderWrapper(torch.nn.Module):
    def __init__(self, net, renderer, simple_output):
        super().__init__()
        self.net = net
        self.renderer = renderer
        self.simple_output = simple_output

    def forward(self, rays, want_weights=False, want_alphas=False, want_z_samps=False,
                want_rgb_samps=False, sample_from_dist=None):
        if rays.shape[0] == 0:
            return (torch.zeros(0, 3, device=rays.device), torch.zeros(0, device=rays.device))
        outputs = self.renderer(
            self.net, rays,
            want_weights=want_weights and not self.simple_output,
            want_alphas=want_alphas and not self.simple_output,
            want_z_samps=want_z_samps and not self.simple_output,
            want_rgb_samps=want_rgb_samps and not self.simple_output,
            sample_from_dist=sample_from_dist)
        if self.simple_output:
            part = outputs["fine"] if self.renderer.using_fine else outputs["coarse"]
            return part["rgb"], part["depth"]
        return outputs


class NeRFRenderer(torch.nn.Module):
    def __init__(self, n_coarse=128, n_fine=0, n_fine_depth=0, noise_std=0.0, depth_std=0.01,
                 eval_batch_size=100000, white_bkgd=False, lindisp=False, sched=None,
                 hard_alpha_cap=False, render_mode="volumetric", surface_sigmoid_scale=.1,
                 render_flow=False, normalize_dino=False):
        super().__init__()
        self.n_coarse, self.n_fine = n_coarse, n_fine
        self.n_fine_depth = n_fine_depth
        self.noise_std = noise_std
        self.depth_std = depth_std
        self.eval_batch_size = eval_batch_size
        self.white_bkgd = white_bkgd
        self.lindisp = lindisp
        self.using_fine = n_fine > 0
        self.sched = sched if (sched is None or len(sched) > 0) else None
        self.register_buffer("iter_idx", torch.tensor(0, dtype=torch.long), persistent=True)
        self.register_buffer("last_sched", torch.tensor(0, dtype=torch.long), persistent=True)
        self.hard_alpha_cap = hard_alpha_cap
        assert render_mode in ("volumetric", "surface", "neus")
        self.render_mode = render_mode
        self.only_surface_color = render_mode == "surface"
        self.surface_sigmoid_scale = surface_sigmoid_scale
        self.render_flow = render_flow
        self.normalize_dino = normalize_dino
        self.z_jitter = None          # parity hook (see module docstring)
        # debug flag: the reference's per-call NaN guard (nerf.py:428-432; host sync)
        self.check_nan = os.environ.get("SCENEDINO_AMD_NAN_CHECK", "0") == "1"
        self._rng_offset = 0
        # index of this call's first ray within its frame: the in-kernel z jitter is keyed
        # by the ray's frame index, so a row band rendered alone (ray-tile sharding) draws
        # the same depths as the whole frame would
        self.ray_offset = 0
        self._want = None             # per-forward: which per-sample outputs are written
        self._z_seed = None           # per-forward: in-kernel z sampling seed

    # -- sampling -------------------------------------------------------------
    def _jitter_seed(self):
        return int(torch.randint(0, 2**62, (1,)).item())  # CPU generator: no device sync

    def sample_coarse(self, rays):
        rays = rays.float().contiguous()
        u = self.z_jitter
        if u is not None:
            u = u.to(device=rays.device, dtype=torch.float32).contiguous()
            return _lib.sample_z(rays, self.n_coarse, self.lindisp, u=u)
        return _lib.sample_z(rays, self.n_coarse, self.lindisp, seed=self._jitter_seed())

    def _z_to_steps_linear(self, rays, z_steps):
        near, far = rays[:, 6:7], rays[:, 7:8]
        if not self.lindisp:
            return near * (1 - z_steps) + far * z_steps
        return 1 / (1 / near * (1 - z_steps) + 1 / far * z_steps)

    def sample_fine(self, rays, weights):
        """Importance sampling (nerf.py:181-212); not used by shipped configs."""
        B = rays.shape[0]
        w = weights.detach() + 1e-5
        pdf = w / torch.sum(w, -1, keepdim=True)
        cdf = torch.cat([torch.zeros_like(pdf[:, :1]), torch.cumsum(pdf, -1)], -1)
        u = torch.rand(B, self.n_fine - self.n_fine_depth, device=rays.device)
        inds = torch.clamp_min(torch.searchsorted(cdf, u, right=True).float() - 1.0, 0.0)
        z_steps = (inds + torch.rand_like(inds)) / self.n_coarse
        return self._z_to_steps_linear(rays, z_steps)

    def sample_fine_depth(self, rays, depth):
        z = depth.unsqueeze(1).repeat((1, self.n_fine_depth))
        z = z + torch.randn_like(z) * self.depth_std
        return torch.max(torch.min(z, rays[:, 7:8]), rays[:, 6:7])

    def sample_coarse_from_dist(self, rays, weights, z_samp):
        """nerf.py:143-179; not used by shipped configs."""
        B = rays.shape[0]
        w = weights.detach() + 1e-5
        pdf = w / torch.sum(w, -1, keepdim=True)
        cdf = torch.cat([torch.zeros_like(pdf[:, :1]), torch.cumsum(pdf, -1)], -1)
        u = torch.rand(B, self.n_coarse, device=rays.device)
        ids = torch.clamp(torch.searchsorted(cdf, u, right=True) - 1, 0, self.n_coarse - 1)
        interp = torch.rand_like(ids, dtype=torch.float32)
        if self.lindisp:
            z_samp = 1 / z_samp
        centers = 0.5 * (z_samp[:, 1:] + z_samp[:, :-1])
        borders = torch.cat((z_samp[:, :1], centers, z_samp[:, -1:]), dim=-1)
        z = torch.gather(borders, -1, ids) * (1 - interp) + torch.gather(borders, -1, ids + 1) * interp
        return 1 / z if self.lindisp else z

    # -- compositing ----------------------------------------------------------
    def composite(self, model, rays, z_samp, coarse=True, sb=0):
        """Returns the reference's 10-tuple (nerf.py:438-449)."""
        with torch.profiler.record_function("renderer_composite"):
            if self.render_mode != "volumetric":
                raise NotImplementedError("render_mode surface/neus is not used by shipped configs")
            if self.training and self.noise_std > 0.0:
                raise NotImplementedError("sigma noise (training) is outside the inference hot path")
            # z_samp None: the fused kernel draws the depths itself (forward() decided,
            # seed in self._z_seed); the (B, K) depth array is never materialised
            B = rays.shape[0]
            K = z_samp.shape[1] if z_samp is not None else self.n_coarse
            r_dim = rays.shape[-1]
            sbn = sb if sb > 0 else 1
            want = getattr(self, "_want", None) or {}
            if self._fused_ok(model, K):
                o = model.render_fused(rays, z_samp, sbn, self.hard_alpha_cap,
                                       want_weights=want.get("weights", True),
                                       want_alphas=want.get("alphas", True),
                                       want_rgb_samps=want.get("rgb_samps", False),
                                       K=K, z_seed=self._z_seed, lindisp=self.lindisp,
                                       z_offset=self.ray_offset * K)
                weights, alphas = o["weights"], o["alphas"]
                rgb_final, depth_final = o["rgb"], o["depth"]
                invalid = o["invalid"]
                rgbs = o["rgb_samps"]
                state_dicts = {"invalid_features": o["invalid_f"].view(B, K, 1),
                               "dino_features": o["dino"]}
            else:
                weights, alphas, rgb_final, depth_final, invalid, rgbs, state_dicts = \
                    self._composite_generic(model, rays, z_samp, coarse, sb)
            if self.white_bkgd:
                if weights is None:
                    raise RuntimeError("white_bkgd needs the per-sample weights")
                rgb_final = rgb_final + 1 - weights.sum(dim=1).unsqueeze(-1)
            if self.check_nan:
                self._nan_guard(weights, rgb_final, depth_final, alphas, invalid, z_samp)
            ray_info = rays[:, None, 8:] if r_dim > 8 else None
            return (weights, rgb_final, depth_final, alphas, invalid, z_samp, rgbs, ray_info,
                    None, state_dicts)

    @staticmethod
    def _nan_guard(weights, rgb_final, depth_final, alphas, invalid, z_samp):
        """The reference's NaN check of every composite call (nerf.py:428-432): print the
        offending tensor and exit().  Behind ``check_nan`` (a debug flag, env
        SCENEDINO_AMD_NAN_CHECK=1) because each check is a device -> host sync; tensors the
        fused path does not produce (None) are skipped."""
        for name, x in [("weights", weights), ("rgb_final", rgb_final),
                        ("depth_final", depth_final), ("alphas", alphas), ("invalid", invalid),
                        ("z_samp", z_samp)]:
            if x is not None and torch.is_floating_point(x) and bool(torch.isnan(x).any()):
                print(f"Detected NaN in {name} ({x.dtype}):")
                print(x)
                exit()

    def _fused_ok(self, model, K):
        return (hasattr(model, "render_fused") and not getattr(model, "use_viewdirs", False)
                and model.fused_supported(K))

    def _composite_generic(self, model, rays, z_samp, coarse, sb):
        B, K = z_samp.shape
        r_dim = rays.shape[-1]
        points = (rays[:, None, :3] + z_samp.unsqueeze(2) * rays[:, None, 3:6]).reshape(-1, 3)
        ray_info = rays[:, None, 8:].expand(-1, K, -1) if r_dim > 8 else None
        if sb > 0:
            points = points.reshape(sb, -1, 3)
            if ray_info is not None:
                ray_info = ray_info.reshape(sb, -1, ray_info.shape[-1])
            dim, bs = 1, (self.eval_batch_size - 1) // sb + 1
        else:
            dim, bs = 0, self.eval_batch_size
        if getattr(model, "wants_single_chunk", None) is not None and model.wants_single_chunk():
            bs = points.shape[dim]  # the model's training path: one launch per kernel per pass
        chunks = torch.split(points, bs, dim=dim)
        infos = torch.split(ray_info, bs, dim=dim) if ray_info is not None else [None] * len(chunks)
        rgbs_all, inv_all, sig_all, sds = [], [], [], []
        hooks = hasattr(model, "begin_pass") and hasattr(model, "end_pass")
        if hooks:
            model.begin_pass()
        try:
            for pnts, info in zip(chunks, infos):
                rgbs, invalid, sigmas, extras, sd = model(pnts, coarse=coarse, only_density=False,
                                                          ray_info=info,
                                                          render_flow=self.render_flow)
                if extras is not None:
                    raise NotImplementedError("field extras are not used by shipped configs")
                rgbs_all.append(rgbs); inv_all.append(invalid); sig_all.append(sigmas)
                if sd is not None:
                    sds.append(sd)
        finally:
            if hooks:
                model.end_pass()
        # (one chunk -- the training path -- is used as is: torch.cat copies even one tensor)
        cat = lambda xs: xs[0] if len(xs) == 1 else torch.cat(xs, dim=dim)
        rgbs = cat(rgbs_all).reshape(B, K, -1).float().contiguous()
        invalid = cat(inv_all).reshape(B, K, -1)
        sigmas = cat(sig_all).reshape(B, K).float().contiguous()
        state_dicts = {k: cat([s[k] for s in sds]) for k in sds[0]} if sds else None
        if state_dicts is not None:
            state_dicts = {k: v.reshape(B, K, *v.shape[2:]) for k, v in state_dicts.items()}
        feat = state_dicts["dino_features"].float().contiguous() if state_dicts else None
        # sd_composite; with autograd (sd_composite_bwd) when the field output carries grad
        weights, alphas, depth, feat_out, rgb_out = autograd.composite(
            z_samp, sigmas, feat, rgbs, self.hard_alpha_cap)
        if state_dicts is not None:
            state_dicts["dino_features"] = feat_out
        return weights, alphas, rgb_out, depth, invalid, rgbs, state_dicts

    # -- forward --------------------------------------------------------------
    def forward(self, model, rays, want_weights=False, want_alphas=False, want_z_samps=False,
                want_rgb_samps=False, sample_from_dist=None):
        with torch.profiler.record_function("renderer_forward"):
            if self.sched is not None and self.last_sched.item() > 0:
                self.n_coarse = self.sched[1][self.last_sched.item() - 1]
                self.n_fine = self.sched[2][self.last_sched.item() - 1]
            assert len(rays.shape) == 3
            sbs = rays.shape[0]
            r_dim = rays.shape[-1]
            rays = rays.reshape(-1, r_dim)
            # per-sample outputs nobody asked for are not written by the fused kernel;
            # the fine pass and white_bkgd need the weights
            self._want = {"weights": want_weights or self.using_fine or self.white_bkgd,
                          "alphas": want_alphas, "rgb_samps": want_rgb_samps}
            self._z_seed = None
            if (sample_from_dist is None and self.z_jitter is None and not want_z_samps
                    and not self.using_fine and self._fused_ok(model, self.n_coarse)):
                # z sampled inside the fused kernel (same RNG stream as sd_sample_z)
                z_coarse = None
                self._z_seed = self._jitter_seed()
            elif sample_from_dist is None:
                z_coarse = self.sample_coarse(rays)
            else:
                pw, pz = sample_from_dist
                n = pw.shape[-1]
                z_coarse = self.sample_coarse_from_dist(rays, pw.reshape(-1, n), pz.reshape(-1, n))
                z_coarse, _ = torch.sort(z_coarse, dim=-1)
            cc = self.composite(model, rays, z_coarse, coarse=True, sb=sbs)
            outputs = {"coarse": self._format_outputs(cc, sbs, want_weights, want_alphas,
                                                      want_z_samps, want_rgb_samps)}
            outputs["state_dict"] = cc[-1]
            if self.using_fine:
                samps = [z_coarse]
                if self.n_fine - self.n_fine_depth > 0:
                    samps.append(self.sample_fine(rays, cc[0].detach()))
                if self.n_fine_depth > 0:
                    samps.append(self.sample_fine_depth(rays, cc[2]))
                z_comb, _ = torch.sort(torch.cat(samps, dim=-1), dim=-1)
                fc = self.composite(model, rays, z_comb.contiguous(), coarse=False, sb=sbs)
                outputs["fine"] = self._format_outputs(fc, sbs, want_weights, want_alphas,
                                                       want_z_samps, want_rgb_samps)
            self._want, self._z_seed = None, None
            return outputs

    def _format_outputs(self, rendered, superbatch_size, want_weights=False, want_alphas=False,
                        want_z_samps=False, want_rgb_samps=False):
        (weights, rgb_final, depth, alphas, invalid, z_samps, rgb_samps, ray_info, extras,
         state_dict) = rendered
        n_smps = invalid.shape[1]
        out_d_rgb = rgb_final.shape[-1]
        out_d_i = invalid.shape[-1]
        if superbatch_size > 0:
            rgb_final = rgb_final.reshape(superbatch_size, -1, out_d_rgb)
            depth = depth.reshape(superbatch_size, -1)
            invalid = invalid.reshape(superbatch_size, -1, n_smps, out_d_i)
        ret = {"rgb": rgb_final, "depth": depth, "invalid": invalid}
        if ray_info is not None:
            ret["ray_info"] = ray_info.reshape(superbatch_size, -1, ray_info.shape[-1])
        if want_weights:
            ret["weights"] = weights.reshape(superbatch_size, -1, n_smps)
        if want_alphas:
            ret["alphas"] = alphas.reshape(superbatch_size, -1, n_smps)
        if want_z_samps:
            ret["z_samps"] = z_samps.reshape(superbatch_size, -1, n_smps)
        if want_rgb_samps:
            ret["rgb_samps"] = rgb_samps.reshape(superbatch_size, -1, n_smps, out_d_rgb)
        if state_dict is not None and "dino_features" in state_dict:
            d = state_dict["dino_features"].shape[-1]
            ret["dino_features"] = state_dict["dino_features"].reshape(superbatch_size, -1, d)
        if state_dict is not None and "invalid_features" in state_dict:
            ret["invalid_features"] = state_dict["invalid_features"].reshape(
                superbatch_size, -1, n_smps, out_d_i)
        return ret

    def sched_step(self, steps=1):
        if self.sched is None:
            return
        self.iter_idx += steps
        while (self.last_sched.item() < len(self.sched[0])
               and self.iter_idx.item() >= self.sched[0][self.last_sched.item()]):
            self.n_coarse = self.sched[1][self.last_sched.item()]
            self.n_fine = self.sched[2][self.last_sched.item()]
            self.last_sched += 1

    @classmethod
    def from_conf(cls, conf, white_bkgd=False, eval_batch_size=100000):
        return cls(conf.get("n_coarse", 128), conf.get("n_fine", 0),
                   n_fine_depth=conf.get("n_fine_depth", 0), noise_std=conf.get("noise_std", 0.0),
                   depth_std=conf.get("depth_std", 0.01),
                   white_bkgd=conf.get("white_bkgd", white_bkgd),
                   lindisp=conf.get("lindisp", True),
                   eval_batch_size=conf.get("eval_batch_size", eval_batch_size),
                   sched=conf.get("sched", None), hard_alpha_cap=conf.get("hard_alpha_cap", False),
                   render_mode=conf.get("render_mode", "volumetric"),
                   surface_sigmoid_scale=conf.get("surface_sigmoid_scale", 1),
                   render_flow=conf.get("render_flow", False),
                   normalize_dino=conf.get("normalize_dino", False))

    def bind_parallel(self, net, gpus=None, simple_output=False):
        wrapped = _RenderWrapper(net, self, simple_output=simple_output)
        if gpus is not None and len(gpus) > 1:
            wrapped = torch.nn.DataParallel(wrapped, gpus, dim=1)
        return wrapped
