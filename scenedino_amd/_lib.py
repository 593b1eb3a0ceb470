"""ctypes binding of libsdhip.so (the C ABI declared in include/sdhip.h).

The product path has no fallback: if the shared library is missing or a call
fails, this module raises.  Only raw device pointers, sizes and the current HIP
stream cross the boundary.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# SDHIP_LIB: alternative build of the same library (diagnostic builds only)
LIB_PATH = os.environ.get("SDHIP_LIB") or os.path.join(_HERE, "libsdhip.so")
ABI_VERSION = 11
CAM_WORDS = 36  # floats per camera record (include/sdhip.h SD_CAM_WORDS)

SD_F32 = 0
SD_BF16 = 1
SD_F16 = 2
TORCH_DTYPE = {SD_F32: torch.float32, SD_BF16: torch.bfloat16, SD_F16: torch.float16}
SD_OF_TORCH = {v: k for k, v in TORCH_DTYPE.items()}
# element type of the render / field kernels' grid operands (the NHWC grid, the projected
# grid P) and of every MLP operand upstream of sigma, per precision mode: f16 in both 16-bit
# modes -- the bf16 mode keeps bf16 for the DINO output layer only (include/sdhip.h sd_mlp,
# csrc/sdhip_render.h RMode; SURVEY §8(c)'s 1e-2 m depth contract)
FIELD_DTYPE = {SD_F32: SD_F32, SD_BF16: SD_F16, SD_F16: SD_F16}

_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32


class SdMlp(ctypes.Structure):
    _fields_ = [
        ("w_in", _vp), ("b_in_h", _vp), ("w_sig_h", _vp), ("b_sigma", ctypes.c_float),
        ("w_out", _vp), ("b_dino", _vp),
        ("C", _i32), ("D", _i32), ("dtype", _i32), ("d_hidden", _i32),
        ("b_empty_h", _vp), ("proj_flags", _i32), ("pad_mlp", _i32),
    ]


class SdFrameArgs(ctypes.Structure):
    """sd_frame_args (include/sdhip.h): sd_frame_inputs' operands."""
    _fields_ = [("img_nchw", _vp), ("N", _i64), ("H", _i64), ("W", _i64), ("out_nhwc4", _vp),
                ("w2c", _vp), ("s_w", _i64), ("Ks", _vp), ("s_k", _i64), ("n", _i64),
                ("out_cam", _vp)]


class SdHead(ctypes.Structure):
    _fields_ = [
        ("w_pe", _vp), ("w_sig", _vp), ("w_out", _vp), ("b_dino", _vp),
        ("b_sigma", ctypes.c_float), ("D", _i32), ("dtype", _i32),
    ]


class SdRenderArgs(ctypes.Structure):
    _fields_ = [
        ("rays", _vp), ("ray_dim", _i64), ("R", _i64), ("rays_per_sb", _i64), ("K", _i32),
        ("z", _vp),
        ("grid", _vp), ("Hf", _i32), ("Wf", _i32),
        ("cam_f", _vp),
        ("img", _vp), ("nv", _i32), ("Hc", _i32), ("Wc", _i32),
        ("cam_c", _vp),
        ("hard_alpha_cap", _i32),
        ("depth", _vp), ("dino", _vp), ("rgb", _vp),
        ("weights", _vp), ("alphas", _vp), ("invalid", _vp), ("invalid_f", _vp),
        ("rgb_samps", _vp),
        ("z_lindisp", _i32), ("z_seed", ctypes.c_uint64), ("z_offset", ctypes.c_uint64),
        ("work", _vp),
        ("ld_depth", _i64), ("ld_dino", _i64), ("ld_rgb", _i64),
        ("grid_dtype", _i32), ("pad1", _i32),
    ]


class SdFieldArgs(ctypes.Structure):
    _fields_ = [
        ("xyz", _vp), ("B", _i64), ("P", _i64),
        ("grid", _vp), ("Hf", _i32), ("Wf", _i32),
        ("cam_f", _vp),
        ("img", _vp), ("nv", _i32), ("Hc", _i32), ("Wc", _i32),
        ("cam_c", _vp),
        ("sigma", _vp), ("dino", _vp), ("rgb", _vp), ("invalid", _vp), ("invalid_f", _vp),
        ("dino_dtype", _i32), ("grid_dtype", _i32), ("tile_order", _vp),
    ]


class SdSegHead(ctypes.Structure):
    _fields_ = [
        ("w1", _vp), ("b1", _vp), ("w2", _vp), ("b2", _vp),
        ("wl", _vp), ("bl", _vp), ("bo", _vp), ("wm", _vp), ("bm", _vp), ("bn1", _vp),
        ("wn2", _vp), ("centres", _vp), ("assign", _vp),
        ("n_clusters", _i32), ("d_in", _i32), ("d_latent", _i32), ("d_full", _i32),
        ("d_code", _i32), ("w2_f8", _vp), ("w2_f8_scale", ctypes.c_float), ("pad0", _i32),
        ("wg", _vp), ("g2", _vp), ("b2sq", ctypes.c_float), ("frag_layout", _i32),
    ]


class SdGemmArgs(ctypes.Structure):
    _fields_ = [
        ("a", _vp), ("lda", _i64), ("w", _vp), ("bias", _vp), ("M", _i64), ("N", _i64),
        ("K", _i64), ("epi", _i32), ("out", _vp), ("ldo", _i64), ("gamma", _vp),
        ("q", _vp), ("k", _vp), ("vt", _vp),
        ("tokens", _i32), ("heads", _i32), ("head_dim", _i32), ("tokens_pad", _i32),
        ("pos", _vp), ("patches", _i32),
        ("res", _vp), ("res2", _vp),
        ("conv", _i32), ("H", _i32), ("W", _i32), ("Cin", _i32), ("stride", _i32), ("OH", _i32),
        ("OW", _i32), ("relu_in", _i32),
        ("shuf_k", _i32), ("in_h", _i32), ("in_w", _i32),
    ]


class SdPatchArgs(ctypes.Structure):
    """sd_patch_args (include/sdhip.h): PatchRaySampler batch."""
    _fields_ = [
        ("poses", _vp), ("Ks", _vp), ("frame_ids", _vp), ("patches", _vp), ("images", _vp),
        ("dino", _vp), ("rays", _vp), ("rgb_out", _vp), ("dino_out", _vp),
        ("B", _i64), ("V", _i64), ("H", _i64), ("W", _i64),
        ("n_patches", _i32), ("ph", _i32), ("pw", _i32), ("channels", _i32),
        ("dino_c", _i32), ("dino_h", _i32), ("dino_w", _i32), ("dino_upscaled", _i32),
        ("z_near", ctypes.c_float), ("z_far", ctypes.c_float),
    ]


class SdMlpTrainArgs(ctypes.Structure):
    """sd_mlp_train_args (include/sdhip.h): fused training MLP."""
    _fields_ = [
        ("x", _vp), ("N", _i64), ("ldx", _i32), ("kx", _i32), ("dtype", _i32), ("D", _i32),
        ("C", _i32), ("lddx", _i32), ("dx_dtype", _i32), ("pad", _i32), ("w1f", _vp), ("w2f", _vp), ("b_out", _vp), ("h", _vp),
        ("sigma", _vp), ("dino", _vp), ("d_sigma", _vp), ("d_dino", _vp), ("wtf", _vp),
        ("wxf", _vp), ("dy", _vp), ("dh", _vp), ("dx", _vp), ("xyz", _vp), ("cam_f", _vp),
        ("dgrid", _vp), ("P", _i64), ("Hf", _i32), ("Wf", _i32),
    ]


class SdWgradArgs(ctypes.Structure):
    """sd_wgrad_args (include/sdhip.h): training-MLP weight gradients."""
    _fields_ = [("a", _vp), ("b", _vp), ("N", _i64), ("lda", _i32), ("ldb", _i32),
                ("Ma", _i32), ("Nb", _i32), ("dtype", _i32), ("nparts", _i32), ("part", _vp)]


class SdMlpWgradArgs(ctypes.Structure):
    """sd_mlp_wgrad_args (include/sdhip.h): both training-MLP weight gradients."""
    _fields_ = [("x", _vp), ("dh", _vp), ("dy", _vp), ("h", _vp), ("N", _i64), ("ldx", _i32),
                ("kx", _i32), ("D", _i32), ("dtype", _i32), ("nparts", _i32), ("pad", _i32),
                ("work", _vp), ("dw_in", _vp), ("db_in", _vp), ("dw_out", _vp), ("db_out", _vp)]


class SdSalienceArgs(ctypes.Structure):
    """sd_salience_args (include/sdhip.h): PatchSalienceDownsampler forward / backward."""
    _fields_ = [
        ("x", _vp), ("w", _vp), ("b", _vp), ("pw", _vp), ("pb", _vp), ("N", _i64),
        ("S", _i32), ("C", _i32), ("normalize", _i32), ("pad", _i32),
        ("out", _vp), ("sal", _vp), ("wmap", _vp), ("ynorm", _vp),
        ("g_out", _vp), ("g_sal", _vp), ("g_wmap", _vp),
        ("gx", _vp), ("gw_part", _vp), ("gpw_part", _vp), ("gpb_part", _vp), ("gb_part", _vp),
    ]


class SdSscArgs(ctypes.Structure):
    """sd_ssc_args (include/sdhip.h): SSCBench scoring configuration."""
    _fields_ = [
        ("sigma_cutoff", ctypes.c_float), ("additional_invalids", _i32), ("inv_zmax", _i32),
        ("n_sizes", _i32), ("crop_x", _i32 * 4), ("crop_y0", _i32 * 4), ("crop_y1", _i32 * 4),
        ("n_pred_labels", _i32), ("pred_lut", ctypes.c_uint8 * 256),
        ("target_lut", ctypes.c_uint8 * 256), ("target_known", ctypes.c_uint8 * 256),
        ("n_target_labels", _i32),
    ]


(SD_EPI_BF16, SD_EPI_GELU, SD_EPI_F32, SD_EPI_RESID, SD_EPI_QKV, SD_EPI_PATCH, SD_EPI_SHUF,
 SD_EPI_NCHW) = range(8)

# (name, argtypes) of every exported entry point; tests check the .so exports all.
SIGNATURES = {
    "sd_last_error": [],
    "sd_abi_version": [],
    "sd_field_dtype": [ctypes.c_int],
    "sd_reserve_cus": [ctypes.c_int32],
    "sd_spin": [ctypes.c_int32, ctypes.c_float, _vp],
    "sd_ln_gemm": [ctypes.POINTER(SdGemmArgs), _vp, _vp, _vp, ctypes.c_float, _vp],
    "sd_gen_rays": [_vp, _vp, _vp, _i64, _i64, _i64, ctypes.c_float, ctypes.c_float, _vp, _vp],
    "sd_sample_z": [_vp, _i64, _i64, _i64, ctypes.c_int, _vp, ctypes.c_uint64, ctypes.c_uint64,
                    _vp, _vp],
    "sd_patch_rays": [ctypes.POINTER(SdPatchArgs), _vp],
    "sd_pack_grid": [_vp, _i64, _i64, _i64, _i64, ctypes.c_int, _vp, _vp],
    "sd_pack_image": [_vp, _i64, _i64, _i64, _vp, _vp],
    "sd_cam_records": [_vp, _i64, _vp, _i64, _i64, _vp, _vp],
    "sd_frame_inputs": [_vp, _i64, _i64, _i64, _vp, _vp, _i64, _vp, _i64, _i64, _vp, _vp],
    "sd_render_fused": [ctypes.POINTER(SdRenderArgs), ctypes.POINTER(SdMlp), _vp],
    "sd_field_query": [ctypes.POINTER(SdFieldArgs), ctypes.POINTER(SdMlp), _vp],
    "sd_field_gather": [_vp, _i64, _i64, _vp, _i32, _i32, _i32, _vp, _vp, _i32, _i32, _i32, _vp,
                        _vp, _i32, _vp, _vp, _vp, _vp],
    "sd_field_gather_bwd": [_vp, _i64, _i64, _vp, _i32, _i64, _i32, _i32, _i32, _vp, _vp, _vp],
    "sd_unpack_grid": [_vp, _i64, _i64, _i64, _i64, _vp, _vp],
    "sd_composite_bwd": [_vp, _vp, _vp, _i64, _vp, _i64, _i64, _i32, _i32, _vp, _vp, _vp, _vp,
                         _vp, _vp, _vp, _vp, _vp],
    "sd_project_grid": [_vp, _i64, _i64, _i64, ctypes.POINTER(SdMlp), _vp, _vp],
    "sd_project_grid_nhwc": [_vp, _i64, _i64, _i64, ctypes.POINTER(SdMlp), _vp, _vp],
    "sd_project_grid_nhwc_inputs": [_vp, _i64, _i64, _i64, ctypes.POINTER(SdMlp), _vp,
                                    ctypes.POINTER(SdFrameArgs), _vp],
    "sd_cast_grid": [_vp, _i64, ctypes.c_int, _vp, _vp],
    "sd_render_proj": [ctypes.POINTER(SdRenderArgs), ctypes.POINTER(SdHead), _vp],
    "sd_render_proj_work_bytes": [_i64, _i32],
    "sd_render_tile_cap": [_i32],
    "sd_composite": [_vp, _vp, _vp, _i64, _vp, _i64, _i64, _i32, _i32, _vp, _vp, _vp, _vp, _vp,
                     _vp],
    "sd_voxel_points": [ctypes.POINTER(ctypes.c_double), ctypes.c_double, _i64, _i64, _i64,
                        ctypes.POINTER(ctypes.c_double), _vp, _vp],
    "sd_grow3": [_vp, _i64, _i64, _i64, _vp, _vp],
    "sd_seg_query": [_vp, _i32, _i64, ctypes.POINTER(SdSegHead), _vp, ctypes.c_float, _vp, _vp,
                     _vp, _vp],
    "sd_voxel_fov": [ctypes.POINTER(ctypes.c_double), ctypes.c_double, _i64, _i64, _i64,
                     ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), _i32, _i32,
                     _vp, _vp],
    "sd_ssc_confusion": [_vp, _vp, _vp, _vp, _i64, _i64, _i64, ctypes.POINTER(SdSscArgs), _vp,
                         _vp],
    "sd_mlp_train_fwd": [ctypes.POINTER(SdMlpTrainArgs), _vp],
    "sd_mlp_train_bwd": [ctypes.POINTER(SdMlpTrainArgs), _vp],
    "sd_wgrad": [ctypes.POINTER(SdWgradArgs), _vp],
    "sd_mlp_train_wgrad": [ctypes.POINTER(SdMlpWgradArgs), _vp],
    "sd_mlp_train_wgrad_work": [_i32],
    "sd_salience_fwd": [ctypes.POINTER(SdSalienceArgs), _vp],
    "sd_salience_bwd": [ctypes.POINTER(SdSalienceArgs), _vp],
    "sd_gemm": [ctypes.POINTER(SdGemmArgs), _vp],
    "sd_gemm_resid_ln": [ctypes.POINTER(SdGemmArgs), _vp, _vp, ctypes.c_float, _vp, _vp, _vp],
    "sd_attention": [_vp, _vp, _vp, _i32, _i32, _i32, _i32, _i32, ctypes.c_float, _vp, _vp],
    "sd_vit_mlp": [_vp, _vp, _i64, _i32, _i32, _vp, _vp, ctypes.c_float, _vp, _vp, _vp, _vp, _vp,
                   _vp],
    "sd_layernorm": [_vp, _i64, _i32, _vp, _vp, ctypes.c_float, _vp, _i32, _vp],
    "sd_patchify": [_vp, _i32, _i32, _i32, _i32, _i32, ctypes.POINTER(ctypes.c_float),
                    ctypes.POINTER(ctypes.c_float), _vp, _vp, _vp, _vp, _i32, _vp],
    "sd_tokens_to_grid": [_vp, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp],
    "sd_tokens_to_nhwc": [_vp, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp],
    "sd_layernorm_nhwc": [_vp, _i32, _i32, _i32, _vp, _vp, ctypes.c_float, _i32, _i32, _i32, _vp, _vp],
    "sd_upsample2x": [_vp, _i32, _i32, _i32, _i32, _vp, _vp],
}

_lib = None


def load(path: str = LIB_PATH):
    """Load libsdhip.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(
            f"scenedino_amd: HIP library {path} is missing. Build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950).")
    lib = ctypes.CDLL(path)
    for name, argt in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argt
        fn.restype = ctypes.c_int
    lib.sd_last_error.restype = ctypes.c_char_p
    lib.sd_render_proj_work_bytes.restype = ctypes.c_int64
    lib.sd_mlp_train_wgrad_work.restype = ctypes.c_int64
    if lib.sd_abi_version() != ABI_VERSION:
        raise RuntimeError("scenedino_amd: libsdhip.so ABI version mismatch; rebuild it")
    _lib = lib
    return lib


def _check(rc: int, what: str):
    if rc != 0:
        msg = _lib.sd_last_error().decode(errors="replace") if _lib else ""
        raise RuntimeError(f"scenedino_amd: {what} failed (rc={rc}): {msg}")


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_of(t: torch.Tensor):
    if t.device.type != "cuda":
        raise RuntimeError("scenedino_amd: HIP kernels need tensors on a ROCm (cuda) device; "
                           f"got {t.device}")
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _req(t: torch.Tensor, name: str, dtype=torch.float32):
    if t.dtype != dtype:
        raise TypeError(f"scenedino_amd: {name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"scenedino_amd: {name} must be contiguous")
    return t


# ---------------------------------------------------------------------------
# thin wrappers (torch tensors in, torch tensors out; all on the same device)
# ---------------------------------------------------------------------------
def gen_rays(poses_c2w, Ks, frame_ids, H, W, z_near, z_far):
    lib = load()
    v = poses_c2w.shape[0]
    out = torch.empty(v, H, W, 11, device=poses_c2w.device, dtype=torch.float32)
    _check(lib.sd_gen_rays(ptr(_req(poses_c2w, "poses")), ptr(_req(Ks, "Ks")),
                           ptr(_req(frame_ids, "frame_ids")), v, H, W, float(z_near),
                           float(z_far), ptr(out), stream_of(out)), "sd_gen_rays")
    return out


def mlp_train_fwd(args: SdMlpTrainArgs, ref_tensor):
    lib = load()
    _check(lib.sd_mlp_train_fwd(ctypes.byref(args), stream_of(ref_tensor)), "sd_mlp_train_fwd")


def mlp_train_bwd(args: SdMlpTrainArgs, ref_tensor):
    lib = load()
    _check(lib.sd_mlp_train_bwd(ctypes.byref(args), stream_of(ref_tensor)), "sd_mlp_train_bwd")


def wgrad(a, b, Ma, Nb, nparts=None):
    """sum_p a[p, :Ma]^T b[p, :Nb] over the rows of two 16-bit (N, *) matrices (sd_wgrad):
    (Ma, Nb) f32."""
    lib = load()
    N = a.shape[0]
    MaP, NbP = (Ma + 31) // 32 * 32, (Nb + 31) // 32 * 32
    if nparts is None:  # ~2 workgroups per CU over the column splits (5 tiles each)
        splits = (NbP // 32 + 4) // 5
        nparts = max(1, min(512 // splits, (N + 511) // 512))
    part = torch.empty(nparts, MaP, NbP, device=a.device)
    g = SdWgradArgs(a=a.data_ptr(), b=b.data_ptr(), N=N, lda=a.stride(0), ldb=b.stride(0),
                    Ma=Ma, Nb=Nb, dtype=SD_OF_TORCH[a.dtype], nparts=nparts,
                    part=part.data_ptr())
    _check(lib.sd_wgrad(ctypes.byref(g), stream_of(a)), "sd_wgrad")
    return part.sum(0)[:Ma, :Nb]


def mlp_train_wgrad(x, dh, dy, h, kx, D, nparts=None):
    """Both weight gradients of the training MLP (sd_mlp_train_wgrad) from the 16-bit rows
    of sd_mlp_train_fwd / _bwd: (dw_in (128, kx - 1), db_in (128), dw_out (1 + D, 128),
    db_out (1 + D)) f32, lin_out rows in the parameter order (out_0 first)."""
    lib = load()
    N, ldx = x.shape
    dev = x.device
    if nparts is None:  # one workgroup per CU
        nparts = max(1, min(torch.cuda.get_device_properties(dev).multi_processor_count,
                            (N + 31) // 32))
    work = torch.empty(int(lib.sd_mlp_train_wgrad_work(nparts)), device=dev)
    dw_in = torch.empty(128, kx - 1, device=dev)
    db_in = torch.empty(128, device=dev)
    dw_out = torch.empty(1 + D, 128, device=dev)
    db_out = torch.empty(1 + D, device=dev)
    g = SdMlpWgradArgs(x=x.data_ptr(), dh=dh.data_ptr(), dy=dy.data_ptr(), h=h.data_ptr(), N=N,
                       ldx=ldx, kx=kx, D=D, dtype=SD_OF_TORCH[x.dtype], nparts=nparts,
                       work=work.data_ptr(), dw_in=dw_in.data_ptr(), db_in=db_in.data_ptr(),
                       dw_out=dw_out.data_ptr(), db_out=db_out.data_ptr())
    _check(lib.sd_mlp_train_wgrad(ctypes.byref(g), stream_of(x)), "sd_mlp_train_wgrad")
    return dw_in, db_in, dw_out, db_out


def salience_fwd(args: SdSalienceArgs, ref_tensor):
    lib = load()
    _check(lib.sd_salience_fwd(ctypes.byref(args), stream_of(ref_tensor)), "sd_salience_fwd")


def salience_bwd(args: SdSalienceArgs, ref_tensor):
    lib = load()
    _check(lib.sd_salience_bwd(ctypes.byref(args), stream_of(ref_tensor)), "sd_salience_bwd")


def patch_rays(args: SdPatchArgs, ref_tensor):
    lib = load()
    _check(lib.sd_patch_rays(ctypes.byref(args), stream_of(ref_tensor)), "sd_patch_rays")


def sample_z(rays, K, lindisp, u=None, seed=0, offset=0, out=None):
    lib = load()
    R, rd = rays.shape
    z = out if out is not None else torch.empty(R, K, device=rays.device, dtype=torch.float32)
    if u is not None:
        _req(u, "u")
        if tuple(u.shape) != (R, K):
            raise ValueError(f"jitter u must be ({R},{K}), got {tuple(u.shape)}")
    _check(lib.sd_sample_z(ptr(_req(rays, "rays")), R, rd, K, int(bool(lindisp)), ptr(u),
                           ctypes.c_uint64(seed & (2**64 - 1)),
                           ctypes.c_uint64(offset & (2**64 - 1)), ptr(z), stream_of(z)),
           "sd_sample_z")
    return z


def channels_last(g: torch.Tensor) -> bool:
    """(B, C, H, W) tensor whose storage is NHWC (the native encoder's grid layout)."""
    return g.dim() == 4 and not g.is_contiguous() and g.permute(0, 2, 3, 1).is_contiguous()


def pack_grid(grid, dtype):
    """(B, C, H, W) f32 grid -> NHWC (B, H, W, C) in dtype: sd_pack_grid transposes an NCHW
    grid; a channels-last one is returned as its NHWC view (f32) or cast (sd_cast_grid)."""
    lib = load()
    B, C, H, W = grid.shape
    if channels_last(grid):
        nhwc = _req(grid.permute(0, 2, 3, 1), "grid")
        if dtype == SD_F32:
            return nhwc
        out = torch.empty(B, H, W, C, device=grid.device, dtype=TORCH_DTYPE[dtype])
        _check(lib.sd_cast_grid(ptr(nhwc), nhwc.numel(), dtype, ptr(out), stream_of(out)),
               "sd_cast_grid")
        return out
    grid = grid.contiguous()
    out = torch.empty(B, H, W, C, device=grid.device, dtype=TORCH_DTYPE[dtype])
    _check(lib.sd_pack_grid(ptr(_req(grid, "grid")), B, C, H, W, dtype, ptr(out),
                            stream_of(out)), "sd_pack_grid")
    return out


def pack_image(img_nchw):
    lib = load()
    N, c3, H, W = img_nchw.shape
    assert c3 == 3, "colour images must have 3 channels"
    out = torch.empty(N, H, W, 4, device=img_nchw.device, dtype=torch.float32)
    _check(lib.sd_pack_image(ptr(_req(img_nchw, "images")), N, H, W, ptr(out), stream_of(out)),
           "sd_pack_image")
    return out


def _cam_operands(poses_w2c, Ks):
    w = poses_w2c.float().reshape(-1, 4, 4)
    k = Ks.float().reshape(-1, 3, 3)
    if w.stride()[1:] != (4, 1):
        w = w.contiguous()
    if k.stride()[1:] != (3, 1):
        k = k.contiguous()
    n = w.shape[0]
    if k.shape[0] != n:
        raise ValueError("poses and intrinsics must have the same number of views")
    return w, k, n, (w.stride(0) if n > 1 else 16), (k.stride(0) if n > 1 else 9)


def frame_inputs(img_nchw, poses_w2c, Ks):
    """pack_image(img_nchw) and cam_records(poses_w2c, Ks) in one launch (sd_frame_inputs)."""
    lib = load()
    N, c3, H, W = img_nchw.shape
    assert c3 == 3, "colour images must have 3 channels"
    w, k, n, sw, sk = _cam_operands(poses_w2c, Ks)
    img = torch.empty(N, H, W, 4, device=img_nchw.device, dtype=torch.float32)
    cam = torch.empty(*poses_w2c.shape[:-2], CAM_WORDS, device=w.device, dtype=torch.float32)
    _check(lib.sd_frame_inputs(ptr(_req(img_nchw, "images")), N, H, W, ptr(img), ptr(w), sw,
                               ptr(k), sk, n, ptr(cam), stream_of(img)), "sd_frame_inputs")
    return img, cam


def cam_records(poses_w2c, Ks):
    """(..., 4, 4) w2c and (..., 3, 3) K -> (..., CAM_WORDS) camera records (one launch)."""
    lib = load()
    lead = poses_w2c.shape[:-2]
    w = poses_w2c.float().reshape(-1, 4, 4)
    k = Ks.float().reshape(-1, 3, 3)
    if w.stride()[1:] != (4, 1):
        w = w.contiguous()
    if k.stride()[1:] != (3, 1):
        k = k.contiguous()
    n = w.shape[0]
    if k.shape[0] != n:
        raise ValueError("poses and intrinsics must have the same number of views")
    out = torch.empty(*lead, CAM_WORDS, device=w.device, dtype=torch.float32)
    _check(lib.sd_cam_records(ptr(w), w.stride(0) if n > 1 else 16, ptr(k),
                              k.stride(0) if n > 1 else 9, n, ptr(out), stream_of(out)),
           "sd_cam_records")
    return out


def render_fused(args: SdRenderArgs, mlp: SdMlp, ref_tensor):
    lib = load()
    _check(lib.sd_render_fused(ctypes.byref(args), ctypes.byref(mlp), stream_of(ref_tensor)),
           "sd_render_fused")


SD_PROJ_EXACT_GRID = 1
SD_SEG_FRAG32 = 0  # sd_seg_head.frag_layout (include/sdhip.h)
SD_SEG_FRAG16 = 1


def _with_flags(mlp: SdMlp, exact_grid: bool) -> SdMlp:
    """A copy of the MLP record with sd_mlp.proj_flags for one projection call."""
    m = SdMlp.from_buffer_copy(mlp)
    m.proj_flags = SD_PROJ_EXACT_GRID if exact_grid else 0
    return m


def project_grid(grid, mlp: SdMlp, dtype, exact_grid: bool = False):
    """P = W_in[:, :C] . grid + b_in per pixel: (B, Hf, Wf, 128) in FIELD_DTYPE[dtype] (f16
    for both 16-bit modes; plain NHWC, 256 B per pixel).  grid (B, C, Hf, Wf) f32, NCHW or
    channels-last.  exact_grid: the grid as a hi + lo f16 operand pair (SD_PROJ_EXACT_GRID)."""
    lib = load()
    mlp = _with_flags(mlp, exact_grid)
    B, C, H, W = grid.shape
    out = torch.empty(B, H, W, 128, device=grid.device, dtype=TORCH_DTYPE[FIELD_DTYPE[dtype]])
    if channels_last(grid):
        _check(lib.sd_project_grid_nhwc(ptr(_req(grid.permute(0, 2, 3, 1), "grid")), B, H, W,
                                        ctypes.byref(mlp), ptr(out), stream_of(out)),
               "sd_project_grid_nhwc")
        return out
    _check(lib.sd_project_grid(ptr(_req(grid.contiguous(), "grid")), B, H, W, ctypes.byref(mlp),
                               ptr(out), stream_of(out)), "sd_project_grid")
    return out


def project_grid_inputs(grid, mlp: SdMlp, dtype, img_nchw, poses_w2c, Ks, exact_grid: bool = False):
    """project_grid(grid) and frame_inputs(img_nchw, poses_w2c, Ks) in one launch
    (sd_project_grid_nhwc_inputs; channels-last grids -- others take the two calls).
    Returns (P, packed image, camera records)."""
    if not channels_last(grid):
        img, cam = frame_inputs(img_nchw, poses_w2c, Ks)
        return project_grid(grid, mlp, dtype, exact_grid), img, cam
    lib = load()
    mlp = _with_flags(mlp, exact_grid)
    B, C, H, W = grid.shape
    N, c3, Hc, Wc = img_nchw.shape
    assert c3 == 3, "colour images must have 3 channels"
    w, k, n, sw, sk = _cam_operands(poses_w2c, Ks)
    out = torch.empty(B, H, W, 128, device=grid.device, dtype=TORCH_DTYPE[FIELD_DTYPE[dtype]])
    img = torch.empty(N, Hc, Wc, 4, device=img_nchw.device, dtype=torch.float32)
    cam = torch.empty(*poses_w2c.shape[:-2], CAM_WORDS, device=w.device, dtype=torch.float32)
    fa = SdFrameArgs(img_nchw=ptr(_req(img_nchw, "images")), N=N, H=Hc, W=Wc, out_nhwc4=ptr(img),
                     w2c=ptr(w), s_w=sw, Ks=ptr(k), s_k=sk, n=n, out_cam=ptr(cam))
    _check(lib.sd_project_grid_nhwc_inputs(ptr(_req(grid.permute(0, 2, 3, 1), "grid")), B, H, W,
                                           ctypes.byref(mlp), ptr(out), ctypes.byref(fa),
                                           stream_of(out)), "sd_project_grid_nhwc_inputs")
    return out, img, cam


def render_proj_work_bytes(R: int, D: int) -> int:
    return int(load().sd_render_proj_work_bytes(R, D))


def render_tile_cap(nbytes: int) -> int:
    """Test hook (sd_render_tile_cap): cap the tile buffers, returns the previous cap."""
    return int(load().sd_render_tile_cap(int(nbytes)))


def render_proj(args: SdRenderArgs, head: SdHead, ref_tensor):
    lib = load()
    _check(lib.sd_render_proj(ctypes.byref(args), ctypes.byref(head), stream_of(ref_tensor)),
           "sd_render_proj")


def field_query(args: SdFieldArgs, mlp: SdMlp, ref_tensor):
    lib = load()
    _check(lib.sd_field_query(ctypes.byref(args), ctypes.byref(mlp), stream_of(ref_tensor)),
           "sd_field_query")


def voxel_fov(origin, voxel_size, dims, T, cam_k, img_w, img_h, device):
    """SSCBench field-of-view mask (sd_voxel_fov): (nx*ny*nz,) uint8 0/1 on device."""
    lib = load()
    nx, ny, nz = (int(d) for d in dims)
    o = (ctypes.c_double * 3)(*[float(v) for v in origin])
    Tm = torch.as_tensor(T, dtype=torch.float64).reshape(-1, 4)[:3].flatten().tolist()
    t = (ctypes.c_double * 12)(*Tm)
    km = (ctypes.c_double * 9)(*torch.as_tensor(cam_k, dtype=torch.float64)
                               .reshape(3, 3).flatten().tolist())
    out = torch.empty(nx * ny * nz, device=device, dtype=torch.uint8)
    _check(lib.sd_voxel_fov(o, float(voxel_size), nx, ny, nz, t, km, int(img_w), int(img_h),
                            ptr(out), stream_of(out)), "sd_voxel_fov")
    return out


def ssc_confusion(pred, sigma, target, fov, args: SdSscArgs, conf):
    """One frame's SSCBench confusion matrices (sd_ssc_confusion) into ``conf``
    ((n_sizes*256 + 1,) int32 viewed as uint32, device)."""
    lib = load()
    nx, ny, nz = (int(d) for d in pred.shape)
    _check(lib.sd_ssc_confusion(ptr(pred), ptr(sigma), ptr(target), ptr(fov), nx, ny, nz,
                                ctypes.byref(args), ptr(conf), stream_of(conf)),
           "sd_ssc_confusion")


def voxel_points(origin, voxel_size, dims, T, device):
    """SSCBench voxel-centre grid (sd_voxel_points): (nx*ny*nz, 3) float32 on device.
    origin (3,), T (4, 4) or (3, 4): host numbers (float64)."""
    lib = load()
    nx, ny, nz = (int(d) for d in dims)
    o = (ctypes.c_double * 3)(*[float(v) for v in origin])
    Tm = torch.as_tensor(T, dtype=torch.float64).reshape(-1, 4)[:3].flatten().tolist()
    t = (ctypes.c_double * 12)(*Tm)
    out = torch.empty(nx * ny * nz, 3, device=device, dtype=torch.float32)
    _check(lib.sd_voxel_points(o, float(voxel_size), nx, ny, nz, t, ptr(out), stream_of(out)),
           "sd_voxel_points")
    return out


def grow3(sig):
    """3x3x3 max filter of a (nx, ny, nz) f32 density grid (sd_grow3): F.max_pool3d(
    sig[None], 3, 1, 1)[0] of evaluate_model_sscbench.py:755-756."""
    lib = load()
    _req(sig, "sig")
    if sig.dim() != 3:
        raise ValueError("grow3: sig must be (nx, ny, nz)")
    out = torch.empty_like(sig)
    _check(lib.sd_grow3(ptr(sig), sig.shape[0], sig.shape[1], sig.shape[2], ptr(out),
                        stream_of(sig)), "sd_grow3")
    return out


def seg_query(dino, rec: SdSegHead, sigma=None, voxel_size=0.2, want_labels=True,
              want_seg=False, want_full=False):
    """Folded transform_expand + stego k-means head (sd_seg_query) on dino (P, 64) f32 or
    bf16.  Returns (labels int32 (P) | None, seg uint8 (P) | None, dino_full (P, d_full) |
    None)."""
    lib = load()
    dt = SD_BF16 if dino.dtype == torch.bfloat16 else SD_F32
    _req(dino, "dino", torch.bfloat16 if dt == SD_BF16 else torch.float32)
    P = dino.shape[0]
    dev = dino.device
    labels = torch.empty(P, device=dev, dtype=torch.int32) if want_labels else None
    seg = torch.empty(P, device=dev, dtype=torch.uint8) if want_seg else None
    full = torch.empty(P, rec.d_full, device=dev) if want_full else None
    if want_seg:
        if sigma is None or sigma.numel() != P:
            raise ValueError("seg_query: want_seg needs sigma (P,)")
        _req(sigma, "sigma")
    _check(lib.sd_seg_query(ptr(dino), dt, P, ctypes.byref(rec), ptr(sigma), float(voxel_size),
                            ptr(labels), ptr(seg), ptr(full), stream_of(dino)), "sd_seg_query")
    return labels, seg, full


def composite(z, sigma, feat, rgb, hard_alpha_cap, want_weights=True):
    lib = load()
    R, K = z.shape
    dev = z.device
    F = feat.shape[-1] if feat is not None else 0
    Cc = rgb.shape[-1] if rgb is not None else 0
    weights = torch.empty(R, K, device=dev)
    alphas = torch.empty(R, K, device=dev)
    depth = torch.empty(R, device=dev)
    feat_out = torch.empty(R, F, device=dev) if feat is not None else None
    rgb_out = torch.empty(R, Cc, device=dev) if rgb is not None else None
    _check(lib.sd_composite(ptr(_req(z, "z")), ptr(_req(sigma, "sigma")),
                            ptr(feat if feat is None else _req(feat, "feat")), F,
                            ptr(rgb if rgb is None else _req(rgb, "rgb")), Cc, R, K,
                            int(bool(hard_alpha_cap)), ptr(weights), ptr(alphas), ptr(depth),
                            ptr(feat_out), ptr(rgb_out), stream_of(depth)), "sd_composite")
    return weights, alphas, depth, feat_out, rgb_out


def field_gather(xyz, grid_nhwc, cam_f, img=None, cam_c=None, colors=True,
                 dtype=torch.float32):
    """sd_field_gather: xyz (B,P,3), grid_nhwc (B,Hf,Wf,C) f32 -> x (B,P,C+40) = [feat|code|1],
    invalid_f (B,P) bool, rgb (B,P,3nv) | None, invalid (B,P,nv) | None."""
    lib = load()
    B, P, _ = xyz.shape
    _, Hf, Wf, C = grid_nhwc.shape
    dev = xyz.device
    x = torch.empty(B, P, C + 40, device=dev, dtype=dtype)
    invf = torch.empty(B, P, device=dev, dtype=torch.bool)
    nv, Hc, Wc = 0, 0, 0
    if colors:  # img: pack_image output (B*nv, Hc, Wc, 4); cam_c (B, nv, CAM_WORDS)
        nv, Hc, Wc = cam_c.shape[1], img.shape[1], img.shape[2]
    rgb = torch.empty(B, P, 3 * nv, device=dev) if colors else None
    inv = torch.empty(B, P, nv, device=dev) if colors else None
    _check(lib.sd_field_gather(ptr(_req(xyz, "xyz")), B, P, ptr(_req(grid_nhwc, "grid")), C, Hf,
                               Wf, ptr(_req(cam_f, "cam_f")), ptr(img), nv, Hc, Wc, ptr(cam_c),
                               ptr(x), SD_OF_TORCH[dtype], ptr(invf), ptr(rgb), ptr(inv),
                               stream_of(x)),
           "sd_field_gather")
    return x, invf, rgb, inv


def field_gather_bwd(xyz, dx, cam_f, Hf, Wf, C, dgrid=None):
    """sd_field_gather_bwd: dx (B,P,>=C) f32 / f16 / bf16 rows -> dgrid (B,Hf,Wf,C) f32
    (zeros, or accumulated into the given dgrid)."""
    lib = load()
    B, P, _ = xyz.shape
    if dx.dtype not in (torch.float32, torch.float16, torch.bfloat16):
        dx = dx.float()
    dx = dx.contiguous()
    if dgrid is None:
        dgrid = torch.zeros(B, Hf, Wf, C, device=xyz.device)
    _req(dgrid, "dgrid")
    _check(lib.sd_field_gather_bwd(ptr(_req(xyz, "xyz")), B, P, ptr(dx), SD_OF_TORCH[dx.dtype],
                                   dx.shape[-1], C, Hf, Wf,
                                   ptr(_req(cam_f, "cam_f")), ptr(dgrid), stream_of(dgrid)),
           "sd_field_gather_bwd")
    return dgrid


def unpack_grid(grid_nhwc):
    """sd_unpack_grid: (B,H,W,C) f32 -> (B,C,H,W) f32."""
    lib = load()
    B, H, W, C = grid_nhwc.shape
    out = torch.empty(B, C, H, W, device=grid_nhwc.device)
    _check(lib.sd_unpack_grid(ptr(_req(grid_nhwc, "grid")), B, C, H, W, ptr(out),
                              stream_of(out)), "sd_unpack_grid")
    return out


def composite_bwd(z, sigma, feat, rgb, hard_alpha_cap, g_depth, g_feat, g_rgb, g_weights,
                  g_alphas, need_feat=True, need_rgb=False):
    """sd_composite_bwd -> d_sigma (R,K), d_feat (R,K,F) | None, d_rgb (R,K,Cc) | None."""
    lib = load()
    R, K = z.shape
    F = feat.shape[-1] if feat is not None else 0
    Cc = rgb.shape[-1] if rgb is not None else 0
    g = [None if t is None else _req(t.float().contiguous(), n) for t, n in
         ((g_depth, "g_depth"), (g_feat, "g_feat"), (g_rgb, "g_rgb"), (g_weights, "g_weights"),
          (g_alphas, "g_alphas"))]
    if feat is None:
        g[1] = None
    if rgb is None:
        g[2] = None
    d_sigma = torch.empty(R, K, device=z.device)
    d_feat = torch.empty(R, K, F, device=z.device) if (need_feat and g[1] is not None) else None
    d_rgb = torch.empty(R, K, Cc, device=z.device) if (need_rgb and g[2] is not None) else None
    _check(lib.sd_composite_bwd(ptr(_req(z, "z")), ptr(_req(sigma, "sigma")),
                                ptr(feat if feat is None else _req(feat, "feat")), F,
                                ptr(rgb if rgb is None else _req(rgb, "rgb")), Cc, R, K,
                                int(bool(hard_alpha_cap)), *[ptr(t) for t in g], ptr(d_sigma),
                                ptr(d_feat), ptr(d_rgb), stream_of(d_sigma)), "sd_composite_bwd")
    return d_sigma, d_feat, d_rgb


# ---------------------------------------------------------------------------
# ViT encoder kernels (sdhip_vit.hip)
# ---------------------------------------------------------------------------
def gemm(a, w, bias, epi, out=None, gamma=None, qkv=None, tokens=0, heads=0, pos=None,
         patches=0, grid_out=None, ln=None, copy_out=None):
    """sd_gemm: a (M, K) bf16 (row stride a.stride(0)), w (N, K) bf16 contiguous.
    SD_EPI_RESID with grid_out (B, tokens - 1, N)-shaped bf16: also writes the updated rows
    without each image's class token there (tokens_to_nhwc's output, no extra launch).
    SD_EPI_RESID with ln = (ln_w, ln_b, eps, ln_out, ws): sd_gemm_resid_ln -- ln_out (M, N)
    bf16 = LayerNorm of the updated rows (bit-equal to layernorm()), ws a zeroed int32
    workspace of >= ceil(M / 32) words (left zeroed)."""
    lib = load()
    M, K = a.shape
    N = w.shape[0]
    if a.dtype != torch.bfloat16 or w.dtype != torch.bfloat16 or a.stride(1) != 1:
        raise TypeError("sd_gemm: a, w must be bf16 with unit inner stride")
    _req(w, "w", torch.bfloat16)
    g = SdGemmArgs(a=a.data_ptr(), lda=a.stride(0), w=w.data_ptr(),
                   bias=bias.data_ptr() if bias is not None else None, M=M, N=N, K=K, epi=epi,
                   out=out.data_ptr() if out is not None else None,
                   ldo=out.stride(-2) if out is not None else 0,
                   gamma=gamma.data_ptr() if gamma is not None else None)
    if qkv is not None:
        q, k, vt = qkv
        g.q, g.k, g.vt = q.data_ptr(), k.data_ptr(), vt.data_ptr()
        g.tokens, g.heads, g.head_dim, g.tokens_pad = tokens, heads, q.shape[-1], k.shape[-2]
    if pos is not None:
        g.pos, g.patches = pos.data_ptr(), patches
    if copy_out is not None:  # SD_EPI_RESID: an f32 copy of the updated rows (same strides)
        _req(copy_out, "copy_out")
        if epi != SD_EPI_RESID or copy_out.shape != out.shape or copy_out.stride() != out.stride():
            raise ValueError("sd_gemm: copy_out is an SD_EPI_RESID copy shaped / strided as out")
        g.k = copy_out.data_ptr()
    if grid_out is not None:
        _req(grid_out, "grid_out", torch.bfloat16)
        if grid_out.numel() != (M // tokens) * (tokens - 1) * N:
            raise ValueError("sd_gemm: grid_out must hold (M / tokens) x (tokens - 1) x N values")
        g.q, g.tokens = grid_out.data_ptr(), tokens
    if ln is not None:
        ln_w, ln_b, eps, ln_out, ws = ln
        _req(ln_out, "ln_out", torch.bfloat16)
        _req(ws, "ln_ws", torch.int32)
        if ln_out.numel() != M * N or ws.numel() < (M + 31) // 32:
            raise ValueError("sd_gemm_resid_ln: ln_out must hold M x N values, ws ceil(M / 32)")
        _check(lib.sd_gemm_resid_ln(ctypes.byref(g), ptr(_req(ln_w, "ln_w")), ptr(_req(ln_b, "ln_b")),
                                    float(eps), ptr(ln_out), ptr(ws), stream_of(a)), "sd_gemm_resid_ln")
        return
    _check(lib.sd_gemm(ctypes.byref(g), stream_of(a)), "sd_gemm")


def vit_mlp(x_ln, x, ln_w, ln_b, eps, fc1_w, fc1_b, fc2_w, fc2_b, gamma=None):
    """sd_vit_mlp: x += gamma * (fc2(gelu(fc1(LN(x_ln)))) + fc2_b) in place (f32 atomics);
    x_ln a separate f32 copy of x, C = 384."""
    lib = load()
    M, C = x.shape
    _req(x_ln, "x_ln")
    _req(x, "x")
    _req(fc1_w, "fc1_w", torch.bfloat16)
    _req(fc2_w, "fc2_w", torch.bfloat16)
    _check(lib.sd_vit_mlp(ptr(x_ln), ptr(x), M, C, fc1_w.shape[0], ptr(_req(ln_w, "ln_w")),
                          ptr(_req(ln_b, "ln_b")), float(eps), ptr(fc1_w), ptr(_req(fc1_b, "fc1_b")),
                          ptr(fc2_w), ptr(fc2_b) if fc2_b is not None else None,
                          ptr(gamma) if gamma is not None else None, stream_of(x)), "sd_vit_mlp")


def ln_gemm(x, ln_w, ln_b, eps, w, bias, epi, out=None, qkv=None, tokens=0, heads=0):
    """sd_ln_gemm: LN(x) w^T + bias with the epilogue epi; x (M, C) f32, w (N, C) bf16."""
    lib = load()
    M, C = x.shape
    N = w.shape[0]
    _req(x, "x")
    _req(w, "w", torch.bfloat16)
    g = SdGemmArgs(a=None, lda=C, w=w.data_ptr(), bias=bias.data_ptr() if bias is not None else None,
                   M=M, N=N, K=C, epi=epi, out=out.data_ptr() if out is not None else None,
                   ldo=out.stride(-2) if out is not None else 0)
    if qkv is not None:
        q, k, vt = qkv
        g.q, g.k, g.vt = q.data_ptr(), k.data_ptr(), vt.data_ptr()
        g.tokens, g.heads, g.head_dim, g.tokens_pad = tokens, heads, q.shape[-1], k.shape[-2]
    _check(lib.sd_ln_gemm(ctypes.byref(g), ptr(x), ptr(_req(ln_w, "ln_w")), ptr(_req(ln_b, "ln_b")),
                          float(eps), stream_of(x)), "sd_ln_gemm")


def attention(q, k, vt, scale, out):
    lib = load()
    B, H, T, hd = q.shape
    _check(lib.sd_attention(ptr(q), ptr(k), ptr(vt), B, H, T, k.shape[-2], hd, float(scale),
                            ptr(out), stream_of(q)), "sd_attention")


def layernorm(x, w, b, eps, out):
    lib = load()
    rows, C = x.shape
    _check(lib.sd_layernorm(ptr(_req(x, "x")), rows, C, ptr(w), ptr(b), float(eps), ptr(out),
                            int(out.dtype == torch.float32), stream_of(x)), "sd_layernorm")


def patchify(img, p, Kp, mean, std, patches, cls, pos, x):
    lib = load()
    B, _, H, W = img.shape
    m = (ctypes.c_float * 3)(*[float(v) for v in mean])
    sd = (ctypes.c_float * 3)(*[float(v) for v in std])
    _check(lib.sd_patchify(ptr(_req(img, "img")), B, H, W, p, Kp, m, sd, ptr(patches), ptr(cls),
                           ptr(pos), ptr(x), x.shape[-1], stream_of(img)), "sd_patchify")


def tokens_to_grid(x, B, T, C, n_prefix, gh, gw, l2norm):
    lib = load()
    out = torch.empty(B, C, gh, gw, device=x.device, dtype=torch.float32)
    _check(lib.sd_tokens_to_grid(ptr(_req(x, "x")), B, T, C, n_prefix, gh, gw, int(bool(l2norm)),
                                 ptr(out), stream_of(x)), "sd_tokens_to_grid")
    return out


# ---------------------------------------------------------------------------
# DPT decoder helpers
# ---------------------------------------------------------------------------
def conv3x3(x, w, bias, stride=1, relu_in=False, epi=None, out=None, res=None, res2=None):
    """Implicit-GEMM 3x3 convolution, padding 1: x (B, H, W, Cin) bf16 NHWC, w (Cout, 9 Cin)
    bf16 (k order ky, kx, ci) -> (B, OH, OW, Cout) bf16 (or f32 NCHW with epi=SD_EPI_NCHW)."""
    lib = load()
    B, H, W, Cin = x.shape
    _req(x, "x", torch.bfloat16)
    _req(w, "w", torch.bfloat16)
    Cout = w.shape[0]
    OH, OW = (H - 1) // stride + 1, (W - 1) // stride + 1
    epi = SD_EPI_BF16 if epi is None else epi
    M = B * OH * OW
    if out is None:
        out = (torch.empty(B, Cout, OH, OW, device=x.device) if epi == SD_EPI_NCHW else
               torch.empty(B, OH, OW, Cout, device=x.device,
                           dtype=torch.float32 if epi == SD_EPI_F32 else torch.bfloat16))
    g = SdGemmArgs(a=x.data_ptr(), lda=9 * Cin, w=w.data_ptr(),
                   bias=bias.data_ptr() if bias is not None else None, M=M, N=Cout, K=9 * Cin,
                   epi=epi, out=out.data_ptr(), ldo=Cout,
                   res=res.data_ptr() if res is not None else None,
                   res2=res2.data_ptr() if res2 is not None else None,
                   conv=1, H=H, W=W, Cin=Cin, stride=stride, OH=OH, OW=OW,
                   relu_in=int(bool(relu_in)), tokens=OH * OW)
    _check(lib.sd_gemm(ctypes.byref(g), stream_of(x)), "sd_gemm(conv3x3)")
    return out


def linear_nhwc(x, w, bias, epi=None, out=None, shuf=None, res=None):
    """1x1 convolution / ConvTranspose2d(k, stride k) on NHWC bf16 x (B, H, W, Cin):
    w (N, Cin) bf16.  shuf=k: SD_EPI_SHUF into (B, H k, W k, N / k^2)."""
    lib = load()
    B, H, W, Cin = x.shape
    _req(x, "x", torch.bfloat16)
    _req(w, "w", torch.bfloat16)
    N = w.shape[0]
    M = B * H * W
    if shuf is not None:
        epi = SD_EPI_SHUF
        out = torch.empty(B, H * shuf, W * shuf, N // (shuf * shuf), device=x.device,
                          dtype=torch.bfloat16) if out is None else out
    else:
        epi = SD_EPI_BF16 if epi is None else epi
        out = torch.empty(B, H, W, N, device=x.device, dtype=torch.bfloat16) if out is None else out
    g = SdGemmArgs(a=x.data_ptr(), lda=Cin, w=w.data_ptr(),
                   bias=bias.data_ptr() if bias is not None else None, M=M, N=N, K=Cin, epi=epi,
                   out=out.data_ptr(), ldo=N, res=res.data_ptr() if res is not None else None,
                   shuf_k=shuf or 0, in_h=H, in_w=W)
    _check(lib.sd_gemm(ctypes.byref(g), stream_of(x)), "sd_gemm(1x1)")
    return out


def layernorm_nhwc(x, w, b, eps, B, T, C, n_prefix, gh, gw, l2norm):
    """sd_layernorm_nhwc: LayerNorm of the non-prefix token rows of x (B T, C) f32 straight
    into a (B, gh, gw, C) bf16 grid (= layernorm(out_f32) + tokens_to_nhwc, one launch)."""
    lib = load()
    out = torch.empty(B, gh, gw, C, device=x.device, dtype=torch.bfloat16)
    _check(lib.sd_layernorm_nhwc(ptr(_req(x, "x")), B, T, C, ptr(_req(w, "w")), ptr(_req(b, "b")),
                                 float(eps), n_prefix, gh * gw, int(bool(l2norm)), ptr(out),
                                 stream_of(x)), "sd_layernorm_nhwc")
    return out


def tokens_to_nhwc(x, B, T, C, n_prefix, gh, gw, l2norm):
    lib = load()
    out = torch.empty(B, gh, gw, C, device=x.device, dtype=torch.bfloat16)
    _check(lib.sd_tokens_to_nhwc(ptr(_req(x, "x")), B, T, C, n_prefix, gh * gw, int(bool(l2norm)),
                                 ptr(out), stream_of(x)), "sd_tokens_to_nhwc")
    return out


def upsample2x(x):
    lib = load()
    B, H, W, C = x.shape
    out = torch.empty(B, 2 * H, 2 * W, C, device=x.device, dtype=torch.bfloat16)
    _check(lib.sd_upsample2x(ptr(_req(x, "x", torch.bfloat16)), B, H, W, C, ptr(out),
                             stream_of(x)), "sd_upsample2x")
    return out


def reserve_cus(n: int) -> int:
    """sd_reserve_cus: leave n CUs to other kernels (RCCL beside the render); previous value."""
    return int(load().sd_reserve_cus(int(n)))


def spin(nblocks: int, us: float, stream=None) -> None:
    """sd_spin (diagnostic): nblocks single-wave workgroups holding CUs for us microseconds."""
    s = stream if stream is not None else torch.cuda.current_stream()
    _check(load().sd_spin(int(nblocks), float(us), ctypes.c_void_p(s.cuda_stream)), "sd_spin")
