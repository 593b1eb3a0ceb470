"""SceneDINO encoder module, MI355X build (the image encoder feeding the
rendered field).

Mirror of scenedino/models/backbones/dino/dinov2_module.py:19-222 (``build_*`` helpers,
``DINOv2Module`` with the same constructor / ``from_conf`` arguments, attribute names
``encoder`` / ``decoder`` / ``gt_encoder`` / ``dim_reduction`` and therefore the same
``encoder.*`` checkpoint keys).  The prediction pass -- ViT (csrc/sdhip_vit.hip) ->
DPT decoder (same kernels, NHWC bf16) -> NCHW f32 feature grid -- is one HIP graph per
(input shape, parameter version): the intermediate token grids go to the decoder in its
NHWC operand layout without a transposition, and the ~170 launches of a 192x640 frame are
replayed by one graph launch (the DPT's last convolution is launched after the replay so
that it writes the caller's fresh output tensor).

The loss-side downsampler (``downsampler_arch``: ``featup`` = PatchSalienceDownsampler on
the sd_salience kernels, ``bilinear``) is built as in the reference (same
``encoder.downsampler.*`` checkpoint keys).  Out of scope (training-loss machinery, SURVEY
§8 "out"): the feature-upsampling GT wrappers of ``mode="upsample-gt"`` (upsampler.py,
kornia).  ``VisualizationModule`` (PCA / cosine k-means colouring of feature maps, the
demo's and the validation panels' ``fit_visualization`` / ``transform_visualization``) is
built as in the reference, as plain device tensor ops (visualization.py).
"""
from __future__ import annotations

import os
from typing import List, Optional, Tuple

import torch
import torch.nn.functional as F
from torch import nn

from .dim_reduction import MlpDimReduction, NoDimReduction
from .downsampler import BilinearDownsampler, PatchSalienceDownsampler
from .dpt_head import DPTHead
from .visualization import VisualizationModule
from .vit import DINOv2Encoder, _param_key, vit_forward


def _get(conf, key, default=None):
    if isinstance(conf, dict):
        return conf.get(key, default)
    if hasattr(conf, "get"):
        return conf.get(key, default)
    return getattr(conf, key, default)


class OrthogonalLinearDimReduction(nn.Module):
    """dim_reduction.py:28-36 (parameters ``bias`` / ``weights``): a (reduced -> full)
    affine map, L2-normalised.  Runs as device tensor ops (not on the shipped configs'
    path, which use ``mlp``)."""

    def __init__(self, full_channels, reduced_channels):
        super().__init__()
        self.bias = nn.Parameter(torch.zeros(full_channels))
        self.weights = nn.Parameter(torch.eye(full_channels, reduced_channels))

    def transform_expand(self, features):
        return F.normalize(features @ self.weights.transpose(0, 1) + self.bias, dim=-1)


class NoDecoder(nn.Module):
    """decoder.py:8-33: the final (L2-normalised) token grid resized to the image and
    renormalised."""

    _MODES = {"nearest": "nearest", "bilinear": "bilinear", "bicubic": "bicubic"}

    def __init__(self, image_size, interpolation, normalize_features):
        super().__init__()
        if interpolation not in self._MODES:
            raise NotImplementedError(f'Interpolation mode "{interpolation}" not implemented!')
        self.image_size = tuple(image_size)
        self.mode = self._MODES[interpolation]
        self.normalize_features = normalize_features

    def forward(self, x):
        f = x[-1]
        kw = {} if self.mode == "nearest" else {"align_corners": False, "antialias": True}
        r = F.interpolate(f, size=self.image_size, mode=self.mode, **kw)
        if self.normalize_features:
            r = r / torch.linalg.norm(r, dim=1, keepdim=True)
        return [r]


def build_encoder(backbone: str, image_size: Tuple[int, int], intermediate_features: List[int],
                  key_features: bool, version: str):
    """dinov2_module.py:19-28."""
    if backbone not in ("vit-s", "vit-b"):
        raise NotImplementedError(f"encoder backbone {backbone!r}")
    return DINOv2Encoder(backbone, image_size, intermediate_features=intermediate_features,
                         key_features=key_features, version=version)


def build_decoder(decoder_arch: str, patch_size: int, image_size: Tuple[int, int],
                  latent_size: int, num_ch_enc, decoder_out_dim: int):
    """dinov2_module.py:31-56 (``spf`` is CUDA-only in the reference and not shipped)."""
    if decoder_arch in ("nearest", "bilinear", "bicubic"):
        return NoDecoder(image_size, interpolation=decoder_arch, normalize_features=True)
    if decoder_arch == "dpt":
        return DPTHead(embed_dims=latent_size, post_process_channels=num_ch_enc,
                       readout_type="ignore", patch_size=patch_size, d_out=decoder_out_dim,
                       expand_channels=False)
    raise NotImplementedError(f"decoder_arch {decoder_arch!r}")


def build_downsampler(arch: str, dim: int, patch_size: int):
    """dinov2_module.py:59-66."""
    if arch == "featup":
        return PatchSalienceDownsampler(dim, patch_size=patch_size, normalize_features=True)
    if arch == "bilinear":
        return BilinearDownsampler(patch_size=patch_size)
    raise NotImplementedError(f"downsampler {arch!r}")


def build_dim_reduction(arch: str, full_channels: int, reduced_channels: int):
    """dinov2_module.py:79-88."""
    if arch == "none":
        return NoDimReduction(full_channels, reduced_channels)
    if arch == "mlp":
        return MlpDimReduction(full_channels, reduced_channels, latent_channels=128)
    if arch == "orthogonal-linear":
        return OrthogonalLinearDimReduction(full_channels, reduced_channels)
    raise NotImplementedError(f"dim_reduction_arch {arch!r}")


class DINOv2Module(nn.Module):
    """dinov2_module.py:91-222."""

    def __init__(self, mode: str, decoder_arch: str, upsampler_arch: Optional[str],
                 downsampler_arch: Optional[str], encoder_arch: str, encoder_freeze: bool,
                 flip_avg_gt: bool, dim_reduction_arch: str, num_ch_enc,
                 intermediate_features: List[int], decoder_out_dim: int, dino_pca_dim: int,
                 image_size: Tuple[int, int], key_features: bool, dino_version: str,
                 separate_gt_version: Optional[str]):
        super().__init__()
        self.encoder = build_encoder(encoder_arch, image_size, intermediate_features,
                                     key_features, dino_version)
        self.flip_avg_gt = flip_avg_gt
        self.encoder_frozen = bool(encoder_freeze or separate_gt_version is None)
        if self.encoder_frozen:
            for p in self.encoder.parameters():
                p.requires_grad = False
        self.decoder = build_decoder(decoder_arch, self.encoder.patch_size, image_size,
                                     self.encoder.latent_size, num_ch_enc, decoder_out_dim)
        if separate_gt_version is None:
            self.gt_encoder = self.encoder
        else:
            self.gt_encoder = build_encoder(encoder_arch, image_size, [], key_features,
                                            separate_gt_version)
            for p in self.gt_encoder.parameters():
                p.requires_grad = False
        if mode == "downsample-prediction":
            if upsampler_arch is not None:
                raise ValueError("downsample-prediction takes no upsampler_arch")
            self.downsampler_arch = downsampler_arch
            self.gt_wrapper = None
        elif mode == "upsample-gt":
            raise NotImplementedError("mode 'upsample-gt' (feature-upsampling GT wrappers of "
                                      "the training loss) is outside the MI355X hot path")
        else:
            raise NotImplementedError(f"mode {mode!r}")
        self.mode = mode
        self.downsampler = None
        if mode == "downsample-prediction" and downsampler_arch is not None:
            self.downsampler = build_downsampler(downsampler_arch, self.gt_encoder.latent_size,
                                                 self.gt_encoder.patch_size)
        self.extra_outs = 0
        self.latent_size = decoder_out_dim
        self.dino_pca_dim = dino_pca_dim
        self.dim_reduction = build_dim_reduction(dim_reduction_arch, self.encoder.latent_size,
                                                 dino_pca_dim)
        self.visualization = VisualizationModule(self.encoder.latent_size)
        self.use_graph = True
        self._graph = None
        # DPT level fronts on side streams beside the ViT (SCENEDINO_AMD_DPT_OVERLAP=1 at
        # construction; same kernels and results as the one-stream order).  Off by default:
        # measured slower (ViT-S/16 + DPT 1.14 -> 1.23 ms, profiles/r4_dpt_overlap_ab.txt) --
        # the side streams' full-chip convolutions hold every CU's LDS and delay the
        # latency-bound ViT launches on the critical path
        self.overlap_levels = os.environ.get("SCENEDINO_AMD_DPT_OVERLAP", "0") == "1"
        if self.overlap_levels and int(os.environ.get("SD_SPLITK_WG", "0") or 0) > 0:
            # the cross-workgroup split-K tiles share one ticket / partial workspace per device:
            # split launches on the side streams and on the main stream would corrupt it
            raise ValueError("SCENEDINO_AMD_DPT_OVERLAP=1 and SD_SPLITK_WG>0 cannot be combined")
        self._side = None

    # -- prediction pass --------------------------------------------------------
    def _decode(self, x, last: bool = True):
        """ViT -> decoder, eager.  DPT: NHWC bf16 token grids straight into the decoder
        (``last=False``: stop before the DPT's final convolution, see _predict)."""
        enc = self.encoder
        if enc.resize is not None:
            x = F.interpolate(x, size=enc.resize, mode="bilinear", align_corners=False,
                              antialias=True)
        vit = enc.model
        if isinstance(self.decoder, DPTHead):
            if not (x.is_cuda and self.overlap_levels):
                grids, final = vit_forward(vit.vit, x, vit.packed(), vit.intermediate, nhwc=True)
                return self.decoder.forward_nhwc(grids + [final], last=last)
            # the DPT's per-level fronts (projection, resize, 3x3 conv) on side streams as
            # soon as their token grids exist, overlapping the later ViT blocks (latency-bound
            # 481-token launches that leave most CUs idle); joined before the fusion chain
            main = torch.cuda.current_stream(x.device)
            # (re)pack the decoder weights on the main stream first: the side streams only
            # wait on main, so a pack made inside the first level front (side stream 0) would
            # race the other fronts' reads
            self.decoder._pack()
            if self._side is None or self._side[0] != x.device:
                self._side = (x.device, [torch.cuda.Stream(device=x.device) for _ in range(3)])
            side = self._side[1]
            levels = [None] * (len(vit.intermediate) + 1)

            def on_grid(i, g):
                if i >= len(side):
                    return
                s = side[i]
                s.wait_stream(main)
                with torch.cuda.stream(s):
                    levels[i] = self.decoder.forward_level(i, g)
                if not torch.cuda.is_current_stream_capturing():  # eager: cross-stream lifetimes
                    g.record_stream(s)
                    levels[i].record_stream(main)

            grids, final = vit_forward(vit.vit, x, vit.packed(), vit.intermediate, nhwc=True,
                                       on_grid=on_grid)
            for i, s in enumerate(side):
                if levels[i] is not None:
                    main.wait_stream(s)
            return self.decoder.forward_nhwc(grids + [final], last=last, levels=levels)
        grids, final = vit_forward(vit.vit, x, vit.packed(), vit.intermediate)
        return self.decoder(grids + [final])

    def _predict(self, x):
        if not self.use_graph or not x.is_cuda:
            return self._decode(x)
        dpt = isinstance(self.decoder, DPTHead)
        dkey = _param_key(self.decoder)  # also validates the decoder's packed weights below
        key = (tuple(x.shape), str(x.device), _param_key(self.encoder), dkey)
        if self._graph is None or self._graph[0] != key:
            self._graph = None
            static_in = x.detach().float().contiguous().clone()
            side = torch.cuda.Stream(device=x.device)
            side.wait_stream(torch.cuda.current_stream(x.device))
            with torch.cuda.stream(side):  # warm-up (packing, allocations) outside capture
                self._decode(static_in, last=not dpt)
            torch.cuda.current_stream(x.device).wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                outs = self._decode(static_in, last=not dpt)
            self._graph = (key, graph, static_in, outs)
        _, graph, static_in, outs = self._graph
        static_in.copy_(x)
        graph.replay()
        if dpt:  # the final convolution writes a fresh output (no copy of a graph buffer)
            return self.decoder.forward_last(outs, key=dkey)
        return [o.clone() for o in outs]

    def forward(self, x, ground_truth: bool = False):
        """dinov2_module.py:158-183."""
        if ground_truth:
            with torch.no_grad():
                gt_0 = self.gt_encoder(x)[-1]
                if self.flip_avg_gt:
                    gt_f = self.gt_encoder(x.flip([-1]))[-1]
                    return [F.normalize(gt_f.flip([-1]) + gt_0, dim=1)]
                return [gt_0]
        if torch.is_grad_enabled() and self.training:
            # The reference runs the DPT decoder with autograd (only the ViT sits under
            # no_grad when encoder_freeze, dinov2_module.py:176-183) and trains it in its own
            # Adam group (trainer.py:567-570).  These kernels have no backward: refuse
            # rather than silently leave the decoder (or ViT) parameters without gradients.
            trainable = [n for n, p in self.named_parameters() if p.requires_grad and
                         (n.startswith("decoder.") or (n.startswith("encoder.") and
                                                       not self.encoder_frozen))]
            if trainable:
                raise NotImplementedError(
                    "scenedino_amd DINOv2Module: the ViT / DPT kernels are forward-only; "
                    f"{len(trainable)} trainable encoder/decoder parameters (e.g. {trainable[0]}) "
                    "would get no gradient.  Train with the reference backbone (dropin keeps "
                    "scenedino.models.backbones for training) or freeze them (requires_grad_(False)).")
        with torch.no_grad():
            return self._predict(x)

    def downsample(self, x, mode="patch"):
        """dinov2_module.py:185-189."""
        if self.downsampler is None:
            return None
        return self.downsampler(x, mode)

    def expand_dim(self, features):
        """dinov2_module.py:191-192."""
        return self.dim_reduction.transform_expand(features)

    def fit_visualization(self, features, refit=True):
        """dinov2_module.py:194-195."""
        return self.visualization.fit_pca(features, refit)

    def transform_visualization(self, features, norm=False, from_dim=0):
        """dinov2_module.py:197-198."""
        return self.visualization.transform_pca(features, norm, from_dim)

    def fit_transform_kmeans_visualization(self, features):
        """dinov2_module.py:200-201."""
        return self.visualization.fit_transform_kmeans_batch(features)

    @classmethod
    def from_conf(cls, conf):
        """dinov2_module.py:203-222 (same keys and defaults)."""
        return cls(
            mode=_get(conf, "mode"),
            decoder_arch=_get(conf, "decoder_arch"),
            upsampler_arch=_get(conf, "upsampler_arch", None),
            downsampler_arch=_get(conf, "downsampler_arch", None),
            encoder_arch=_get(conf, "encoder_arch"),
            encoder_freeze=_get(conf, "encoder_freeze"),
            flip_avg_gt=_get(conf, "flip_avg_gt", False),
            dim_reduction_arch=_get(conf, "dim_reduction_arch"),
            num_ch_enc=_get(conf, "num_ch_enc", None),
            intermediate_features=_get(conf, "intermediate_features", []),
            decoder_out_dim=_get(conf, "decoder_out_dim"),
            dino_pca_dim=_get(conf, "dino_pca_dim"),
            image_size=_get(conf, "image_size"),
            key_features=_get(conf, "key_features"),
            dino_version=_get(conf, "version", "reg"),
            separate_gt_version=_get(conf, "separate_gt_version", None),
        )
