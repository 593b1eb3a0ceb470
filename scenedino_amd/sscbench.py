"""SSCBench-KITTI-360 voxel query, MI355X build.

Mirrors the hot part of sscbench/evaluate_model_sscbench.py and sscbench/point_utils.py:
  * ``read_calib`` / ``get_cam_k``          point_utils.py:84-157 (calibration constants)
  * ``generate_point_grid``                  point_utils.py:17-82 -> sd_voxel_points (the
                                             voxel centres; bit-exact, GPU-resident)
  * ``predict_grid``                         evaluate_model_sscbench.py:829-854
  * ``downsample_and_predict``               evaluate_model_sscbench.py:660-758 at
                                             factor 1 (VOXEL_SIZE 0.2): one fused query of
                                             all voxels (sd_field_query without colours +
                                             sd_seg_query with the alpha-weighted class pick)
                                             instead of 4 chunks of 128x128x32, then the
                                             3x3x3 max-pool "grow" of the densities.
IoU bookkeeping, ply export and statistics stay the reference's (out of scope).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from . import _lib

VOXEL_SIZE = 0.2          # evaluate_model_sscbench.py:50
USE_ALPHA_WEIGHTING = True  # :59
USE_GROW = True           # :60
VOX_ORIGIN = (0.0, -25.6, -2.0)
SCENE_SIZE = (51.2, 51.2, 6.4)


def read_calib():
    """point_utils.py:84-137: {"P2": 3x4 projection, "Tr": 4x4 velodyne->camera}."""
    P = np.array([552.554261, 0.0, 682.049453, 0.0, 0.0, 552.554261, 238.769549, 0.0,
                  0.0, 0.0, 1.0, 0.0]).reshape(3, 4)
    cam2velo = np.array([0.04307104361, -0.08829286498, 0.995162929, 0.8043914418,
                         -0.999004371, 0.007784614041, 0.04392796942, 0.2993489574,
                         -0.01162548558, -0.9960641394, -0.08786966659,
                         -0.1770225824]).reshape(3, 4)
    c2v = np.concatenate([cam2velo, np.array([0, 0, 0, 1]).reshape(1, 4)], axis=0)
    tr = np.identity(4)
    tr[:3, :4] = np.linalg.inv(c2v)[:3, :]
    return {"P2": P, "Tr": tr}


def get_cam_k():
    return read_calib()["P2"][:3, :3]


def grid_dims(scene_size=SCENE_SIZE, voxel_size=VOXEL_SIZE):
    """vol_dim = ceil(scene_size / voxel_size) (point_utils.py:52)."""
    return tuple(int(v) for v in np.ceil(np.asarray(scene_size) / voxel_size).astype(int))


def generate_point_grid(cam_E, vox_origin=VOX_ORIGIN, voxel_size=VOXEL_SIZE,
                        scene_size=SCENE_SIZE, device="cuda"):
    """Voxel centres in the camera frame, (nx*ny*nz, 3) float32 on ``device`` -- the
    reference's ``torch.tensor(pts).float()`` of generate_point_grid's first output
    (evaluate_model_sscbench.py:270-278), bit for bit."""
    dims = grid_dims(scene_size, voxel_size)
    return _lib.voxel_points(vox_origin, voxel_size, dims, np.asarray(cam_E, np.float64), device)


def predict_grid(data_batch, net, points, prediction_mode=None):
    """evaluate_model_sscbench.py:829-854 (the reference-contract per-chunk call)."""
    points = points.reshape(1, -1, 3)
    kw = {"predict_segmentation": True}
    if prediction_mode is not None:
        kw["prediction_mode"] = prediction_mode
    dino_feat, invalid, sigmas, segs = net.forward(points, **kw)
    return sigmas, segs, dino_feat


def query_voxels(net, pts, dims, prediction_mode="stego_kmeans", grow=USE_GROW):
    """GPU-resident body of downsample_and_predict at factor 1 for an encoded ``net``:
    pts (nx*ny*nz, 3) -> sigmas (nx, ny, nz) f32 (grown if ``grow``) and segs
    (nx, ny, nz) uint8 on the device."""
    nx, ny, nz = dims
    sigma, seg = net.predict_voxels(pts.reshape(1, -1, 3), voxel_size=VOXEL_SIZE,
                                    prediction_mode=prediction_mode)
    sigmas = sigma.reshape(nx, ny, nz)
    if grow:  # :755-756
        sigmas = F.max_pool3d(sigmas.unsqueeze(0), kernel_size=3, stride=1, padding=1).squeeze(0)
    return sigmas, seg.reshape(nx, ny, nz)


def slab_range(nx: int, rank: int, world: int) -> tuple[int, int]:
    """x-slab [x0, x1) of the voxel grid rendered by ``rank`` (C5 splits the
    256 x-planes, [32 g, 32 g + 32) on 8 GPUs); slabs differ by at most one plane."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    base, extra = divmod(nx, world)
    x0 = rank * base + min(rank, extra)
    return x0, x0 + base + (1 if rank < extra else 0)


def query_voxels_slab(predict, pts, dims, rank, world, grow=USE_GROW):
    """This rank's x-slab of query_voxels.  ``predict(points (P, 3)) -> (sigma (P,),
    seg (P,))`` evaluates the field + head on a contiguous run of voxel centres (the flat
    index (ix ny + iy) nz + iz keeps every x-plane contiguous).  The 3x3x3 grow max-pool
    needs one neighbouring x-plane on each side: those halo planes are queried too and
    dropped after pooling, so the gathered slabs equal the unsharded result bit for bit.
    Returns sigmas (x1 - x0, ny, nz), segs (x1 - x0, ny, nz)."""
    nx, ny, nz = dims
    x0, x1 = slab_range(nx, rank, world)
    h0 = max(x0 - 1, 0) if grow else x0
    h1 = min(x1 + 1, nx) if grow else x1
    plane = ny * nz
    sig, seg = predict(pts[h0 * plane:h1 * plane])
    sig = sig.reshape(h1 - h0, ny, nz)
    if grow:
        sig = F.max_pool3d(sig.unsqueeze(0), kernel_size=3, stride=1, padding=1).squeeze(0)
    lo = x0 - h0
    return (sig[lo:lo + x1 - x0].contiguous(),
            seg.reshape(h1 - h0, ny, nz)[lo:lo + x1 - x0].contiguous())


def gather_slabs(sigmas, segs, dims, group=None):
    """All-gather every rank's x-slab (equal slabs: world divides nx) into the full
    (nx, ny, nz) grids on every rank: one all_gather_into_tensor per output."""
    import torch.distributed as dist
    nx, ny, nz = dims
    world = dist.get_world_size(group)
    if nx % world:
        raise ValueError("gather_slabs needs world | nx (equal slabs)")
    full_s = torch.empty(nx, ny, nz, dtype=sigmas.dtype, device=sigmas.device)
    full_g = torch.empty(nx, ny, nz, dtype=segs.dtype, device=segs.device)
    dist.all_gather_into_tensor(full_s, sigmas, group=group)
    dist.all_gather_into_tensor(full_g, segs, group=group)
    return full_s, full_g


def downsample_and_predict(data, net, pts, factor, prediction_mode, vis=False, feat_vis=False):
    """evaluate_model_sscbench.py:660-758 (factor 1, no visualisation outputs): returns
    numpy ``sigmas`` (256, 256, 32), ``segs`` (256, 256, 32) and ``None``."""
    if factor != 1 or vis or feat_vis:
        raise NotImplementedError("downsample_and_predict: factor 1 (VOXEL_SIZE 0.2) without "
                                  "visualisation outputs")
    if not USE_ALPHA_WEIGHTING:
        raise NotImplementedError("USE_ALPHA_WEIGHTING=False")
    device = pts.device
    images = torch.stack(data["imgs"], dim=0).unsqueeze(0).to(device).float()
    poses = torch.tensor(np.stack(data["poses"], 0)).unsqueeze(0).to(device).float()
    projs = torch.tensor(np.stack(data["projs"], 0)).unsqueeze(0).to(device).float()
    poses = torch.inverse(poses[:, :1]) @ poses
    net.compute_grid_transforms(projs, poses)
    net.encode(images, projs, poses, ids_encoder=[0], ids_render=[0],
               images_alt=images * 0.5 + 0.5)
    net.set_scale(0)
    sigmas, segs = query_voxels(net, pts.reshape(-1, 3), (256, 256, 32), prediction_mode)
    return sigmas.cpu().numpy(), segs.cpu().numpy().astype(np.float64), None
