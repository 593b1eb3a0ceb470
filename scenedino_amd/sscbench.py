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
  * ``get_fov_mask``                         point_utils.py:6-15 -> sd_voxel_fov
  * ``SSCBenchScores``                       the scoring loop, evaluate_model_sscbench.py:284-299
                                             (accumulators), :366-367 / 452-456 / 492 /
                                             496-525 (per frame, one sd_ssc_confusion pass
                                             on the device) and :532-609 (tables, Hungarian
                                             re-assignment, mIoU, the printed report)
Ply export, statistics, alpha cut-off search and the sigma trade-off plot stay the
reference's (visualisation / plotting, out of scope).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

VOXEL_SIZE = 0.2          # evaluate_model_sscbench.py:50
USE_ALPHA_WEIGHTING = True  # :59
USE_GROW = True           # :60
SIGMA_CUTOFF = 0.2        # :57
USE_ADDITIONAL_INVALIDS = True  # :52
SIZES = (12.8, 25.6, 51.2)  # :49
IMG_W, IMG_H = 1408, 376  # generate_point_grid defaults (point_utils.py:17)
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
        sigmas = _lib.grow3(sigmas.contiguous())  # = F.max_pool3d(kernel 3, stride 1, pad 1)
    return sigmas, seg.reshape(nx, ny, nz)


def slab_range(nx: int, rank: int, world: int) -> tuple[int, int]:
    """x-slab [x0, x1) of the voxel grid rendered by ``rank`` (C5 splits the
    256 x-planes, [32 g, 32 g + 32) on 8 GPUs); slabs differ by at most one plane."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    base, extra = divmod(nx, world)
    x0 = rank * base + min(rank, extra)
    return x0, x0 + base + (1 if rank < extra else 0)


def query_voxels_slab(predict, pts, dims, rank, world, grow=USE_GROW, grow_fn=None):
    """This rank's x-slab of query_voxels.  ``predict(points (P, 3)) -> (sigma (P,),
    seg (P,))`` evaluates the field + head on a contiguous run of voxel centres (the flat
    index (ix ny + iy) nz + iz keeps every x-plane contiguous).  The 3x3x3 grow max-pool
    needs one neighbouring x-plane on each side: those halo planes are queried too and
    dropped after pooling, so the gathered slabs equal the unsharded result bit for bit.
    ``grow_fn`` (default sd_grow3) maps a (planes, ny, nz) density block to its 3x3x3 max
    filter.  Returns sigmas (x1 - x0, ny, nz), segs (x1 - x0, ny, nz)."""
    nx, ny, nz = dims
    x0, x1 = slab_range(nx, rank, world)
    h0 = max(x0 - 1, 0) if grow else x0
    h1 = min(x1 + 1, nx) if grow else x1
    plane = ny * nz
    sig, seg = predict(pts[h0 * plane:h1 * plane])
    sig = sig.reshape(h1 - h0, ny, nz)
    if grow:
        sig = (grow_fn or _lib.grow3)(sig.contiguous())
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


# ---------------------------------------------------------------------------
# scoring (evaluate_model_sscbench.py:284-609)
# ---------------------------------------------------------------------------
# sscbench/label_maps.yaml
SSCBENCH_TO_LABEL = {0: 0, 1: 1, 2: 2, 3: 3, 4: 4, 5: 5, 6: 6, 7: 7, 8: 8, 9: 8, 10: 12, 11: 9,
                     12: 10, 13: 11, 14: 12, 15: 13, 16: 14, 17: 9, 18: 15, 19: 0, 255: 255}
CITYSCAPES_TO_LABEL = {0: 7, 1: 8, 2: 9, 3: 9, 4: 10, 5: 13, 6: 15, 7: 14, 8: 11, 9: 12,
                       10: 0, 11: 6, 12: 0, 13: 1, 14: 4, 15: 5, 16: 5, 17: 3, 18: 2}
LABELS = {0: "unlabeled", 1: "car", 2: "bicycle", 3: "motorcycle", 4: "truck",
          5: "other-vehicle", 6: "person", 7: "road", 8: "sidewalk", 9: "building", 10: "fence",
          11: "vegetation", 12: "terrain", 13: "pole", 14: "traffic-sign", 15: "other-object"}
WEIGHTS = {1: 2.85, 2: 0.01, 3: 0.01, 4: 0.16, 5: 5.75, 6: 0.02, 7: 14.98, 8: 6.43, 9: 20.00,
           10: 0.96, 11: 41.99, 12: 9.15, 13: 0.22, 14: 0.06, 15: 0.28}
ROW_LABELS = ["IoU", "Precision", "Recall", "mIoU"] + [LABELS[i] for i in range(1, 16)]


def get_fov_mask(device="cuda"):
    """point_utils.get_fov_mask (:6-15): (256, 256, 32) bool, voxels whose centre projects
    into the 1408 x 376 image in front of the camera (sd_voxel_fov, bit-exact)."""
    dims = grid_dims()
    m = _lib.voxel_fov(VOX_ORIGIN, VOXEL_SIZE, dims, read_calib()["Tr"], get_cam_k(), IMG_W,
                       IMG_H, device)
    return m.view(torch.bool).reshape(dims)


def crop_bounds(size):
    """:496-501: range ``size`` keeps x in [0, n) and y in [128 - n // 2, 128 + n // 2),
    n = int(size // 0.2) (Python's float floor division, as the reference)."""
    n = int(size // 0.2)
    return n, 128 - n // 2, 128 + n // 2


def counts_from_confusion(C):
    """The per-range numbers the reference accumulates (compute_occupancy_numbers :908-925,
    compute_occupancy_numbers_segmentation :862-886, compute_occupancy_recall_segmentation
    :889-905) from one 16 x 16 confusion matrix: every one of them is a sum of its entries."""
    C = np.asarray(C, np.int64)
    d = np.diag(C)[1:]
    fp_seg = C[:, 1:].sum(0) - d
    fn_seg = C[1:, :].sum(1) - d
    return {"tp": int(C[1:, 1:].sum()), "fp": int(C[0, 1:].sum()), "tn": int(C[0, 0]),
            "fn": int(C[1:, 0].sum()),
            "tp_seg": d.astype(np.float64), "fp_seg": fp_seg.astype(np.float64),
            "tn_seg": (C.sum() - d - fp_seg - fn_seg).astype(np.float64),
            "fn_seg": fn_seg.astype(np.float64),
            "confusion_seg": C.astype(np.float64),
            "tp_recall_seg": C[1:, 1:].sum(1).astype(np.float64),
            "sum_recall_seg": C[1:, :].sum(1).astype(np.float64)}


class SSCBenchScores:
    """The SSCBench scoring loop of evaluate_model_sscbench.py on the device.

    ``add_frame(sigmas, segs, voxel_gt, fov_mask)`` is one iteration of the main loop after
    ``downsample_and_predict`` (:366-367 convert_voxels of both label maps, :452-456 the
    additional invalids, :492 ``segs[sigmas < SIGMA_CUTOFF] = 0``, :496-525 the per-range
    counts): one ``sd_ssc_confusion`` launch adds the frame's per-range confusion matrices to
    a device accumulator, with no host round trip.  ``results()`` returns the reference's
    ``results[size]`` dicts (:284-299), ``tables()`` the "direct" / "hungarian" tables of
    :539-584 and ``report()`` the printed result string (:586-609).

    A label without a lookup-table entry makes the reference's dict lookup raise; here it is
    counted on the device and ``results()`` raises (``check_each_frame=True`` raises in
    ``add_frame`` instead, at the cost of one synchronisation per frame).
    """

    def __init__(self, sizes=SIZES, sigma_cutoff=SIGMA_CUTOFF,
                 additional_invalids=USE_ADDITIONAL_INVALIDS, device="cuda",
                 check_each_frame=False):
        if not 1 <= len(sizes) <= 4:
            raise ValueError("SSCBenchScores: 1..4 evaluation ranges")
        self.sizes = tuple(sizes)
        self.device = torch.device(device)
        self.check_each_frame = check_each_frame
        a = _lib.SdSscArgs()
        a.sigma_cutoff = float(sigma_cutoff)
        a.additional_invalids = int(bool(additional_invalids))
        a.inv_zmax = 7  # identify_additional_invalids (:821)
        a.n_sizes = len(self.sizes)
        for i, size in enumerate(self.sizes):
            a.crop_x[i], a.crop_y0[i], a.crop_y1[i] = crop_bounds(size)
        a.n_pred_labels = len(CITYSCAPES_TO_LABEL)
        for k, v in CITYSCAPES_TO_LABEL.items():
            a.pred_lut[k] = v
        for v in range(256):
            a.target_lut[v] = SSCBENCH_TO_LABEL.get(v, 255)
            a.target_known[v] = 1 if v in SSCBENCH_TO_LABEL else 0
        a.n_target_labels = len(SSCBENCH_TO_LABEL)
        self._args = a
        nbins = len(self.sizes) * 256 + 1
        self._frame = torch.zeros(nbins, dtype=torch.int32, device=self.device)
        self._acc = torch.zeros(nbins, dtype=torch.int64, device=self.device)
        self.n_frames = 0

    @staticmethod
    def _u8(x, device):
        t = torch.as_tensor(x, device=device)
        if t.dtype == torch.bool:
            t = t.to(torch.uint8)
        elif t.dtype != torch.uint8:
            t = t.to(torch.int64)
            # values outside 0..255 are labels without a mapping: 254 is not a key either
            t = torch.where((t < 0) | (t > 255), torch.full_like(t, 254), t).to(torch.uint8)
        return t.contiguous()  # class ids outside the table count as unmapped in the kernel

    def frame_confusion(self, sigmas, segs, voxel_gt, fov_mask):
        """Launch the frame's scoring pass; returns the device (n_sizes*256 + 1,) uint32
        counts (as int32) it wrote (valid until the next call)."""
        dev = self.device
        segs_t = torch.as_tensor(segs, device=dev)
        if segs_t.is_floating_point():  # downsample_and_predict returns float64 class ids
            segs_t = segs_t.to(torch.int64)
        segs_t = self._u8(segs_t, dev)
        gt = self._u8(voxel_gt, dev)
        fov = self._u8(fov_mask, dev)
        sig = torch.as_tensor(sigmas, device=dev, dtype=torch.float32).contiguous()
        shape = tuple(segs_t.shape)
        if len(shape) != 3 or any(tuple(t.shape) != shape for t in (gt, fov, sig)):
            raise ValueError("SSCBenchScores: sigmas / segs / voxel_gt / fov_mask must share "
                             "one (nx, ny, nz) shape")
        _lib.ssc_confusion(segs_t, sig, gt, fov, self._args, self._frame)
        return self._frame

    def add_frame(self, sigmas, segs, voxel_gt, fov_mask):
        f = self.frame_confusion(sigmas, segs, voxel_gt, fov_mask)
        self._acc += f.to(torch.int64) & 0xFFFFFFFF
        self.n_frames += 1
        if self.check_each_frame and int(f[-1].item()) != 0:
            raise KeyError("SSCBenchScores: a label without a mapping in label_maps.yaml")

    def confusions(self):
        """{size: accumulated 16 x 16 confusion matrix (int64 numpy)}."""
        acc = self._acc.cpu().numpy()
        if acc[-1] != 0:
            raise KeyError(f"SSCBenchScores: {int(acc[-1])} voxel labels without a mapping in "
                           "label_maps.yaml (the reference's convert_voxels raises)")
        return {size: acc[i * 256:(i + 1) * 256].reshape(16, 16)
                for i, size in enumerate(self.sizes)}

    def results(self):
        """The reference's ``results`` dict (:284-299) after the frames added so far."""
        return {size: counts_from_confusion(c) for size, c in self.confusions().items()}

    def tables(self):
        """:539-584 for mode "direct" and "hungarian": {"table": (19, n_sizes) float32,
        "miou", "weighted_miou" (of the last range), "reassignment"}."""
        from scipy.optimize import linear_sum_assignment
        conf = self.confusions()
        res = {size: counts_from_confusion(c) for size, c in conf.items()}
        out = {}
        for mode in ("direct", "hungarian"):
            table = np.zeros((len(ROW_LABELS), len(self.sizes)), dtype=np.float32)
            assign = None
            if mode == "hungarian":  # :541, on the full (last) range
                assign = linear_sum_assignment(res[self.sizes[-1]]["confusion_seg"], maximize=True)
            miou = wmiou = float("nan")
            with np.errstate(divide="ignore", invalid="ignore"):
                for i, size in enumerate(self.sizes):
                    r = res[size]
                    tp, fp, fn = r["tp"], r["fp"], r["fn"]
                    table[0, i] = np.float64(tp) / (tp + fp + fn)
                    table[1, i] = np.float64(tp) / (tp + fp)
                    table[2, i] = np.float64(tp) / (tp + fn)
                    cm = r["confusion_seg"]
                    if mode == "hungarian":
                        cm = cm[np.argsort(assign[1]), :]
                    d = np.diag(cm)
                    denom = cm.sum(0) + cm.sum(1) - d
                    per_class = d[1:] / denom[1:]
                    miou = np.mean(np.nan_to_num(per_class))
                    w = np.array(list(WEIGHTS.values()))
                    wmiou = np.sum(w * np.nan_to_num(per_class)) / np.sum(w)
                    table[3, i] = miou
                    table[4:, i] = per_class
            out[mode] = {"table": table, "miou": float(miou), "weighted_miou": float(wmiou),
                         "reassignment": None if assign is None else np.argsort(assign[1])}
        return out

    def report(self, ply_checkname="none"):
        """The result string the reference prints (:586-609)."""
        tabs = self.tables()
        headers = [f"{s}m" for s in self.sizes]
        out = ""
        for mode in ("direct", "hungarian"):
            t = tabs[mode]
            out += f"\n# Benchmark Results for '{ply_checkname}' / Mode: {mode}\n"
            out += "\n|               | " + " | ".join(headers) + " |\n"
            out += "|---------------|-------|-------|-------|\n"
            for i, name in enumerate(ROW_LABELS):
                out += f"| {name:<13} | " + " | ".join(f"{v * 100:5.2f}" for v in t["table"][i]) + " |\n"
                if i == 2:
                    out += "|---------------|-------|-------|-------|\n"
            out += "\n"
            if mode == "hungarian":
                out += f"Reassignment: {t['reassignment']}\n"
            out += f"Mean IoU: {t['miou'] * 100:.2f}\n"
            out += f"Weighted Mean IoU: {t['weighted_miou'] * 100:.2f}\n\n"
        return out
