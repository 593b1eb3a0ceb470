"""ssc_oracle -- TEST INFRASTRUCTURE ONLY (the checker, never shipped).

numpy CPU restatement of the SSCBench scoring loop of
sscbench/evaluate_model_sscbench.py (citations are /root/reference file:line).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it.

Pinned by tests/golden/ssc_scoring.json: tests/golden/make_golden.py executes the
reference's own ``convert_voxels``, ``identify_additional_invalids``,
``compute_occupancy_numbers``, ``compute_occupancy_numbers_segmentation`` and
``compute_occupancy_recall_segmentation`` (function bodies taken from the reference file)
and the reference's ``generate_point_grid`` / ``cam2pix`` for the FOV mask, on the seeded
frames of tests/_ssc_inputs.py.  The final table (:532-609: IoU / precision / recall,
Hungarian re-assignment, per-class IoU, mIoU, weighted mIoU) lives inside the reference's
``main()`` and is restated here only (parity unpinned beyond the pinned counts it reads).
"""
from __future__ import annotations

import numpy as np

SIZES = (12.8, 25.6, 51.2)   # evaluate_model_sscbench.py:49
SIGMA_CUTOFF = 0.2           # :57

# sscbench/label_maps.yaml
SSCBENCH_TO_LABEL = {0: 0, 1: 1, 2: 2, 3: 3, 4: 4, 5: 5, 6: 6, 7: 7, 8: 8, 9: 8, 10: 12, 11: 9,
                     12: 10, 13: 11, 14: 12, 15: 13, 16: 14, 17: 9, 18: 15, 19: 0, 255: 255}
CITYSCAPES_TO_LABEL = {0: 7, 1: 8, 2: 9, 3: 9, 4: 10, 5: 13, 6: 15, 7: 14, 8: 11, 9: 12, 10: 0,
                       11: 6, 12: 0, 13: 1, 14: 4, 15: 5, 16: 5, 17: 3, 18: 2}
LABEL_IDS = list(range(16))
WEIGHTS = [2.85, 0.01, 0.01, 0.16, 5.75, 0.02, 14.98, 6.43, 20.00, 0.96, 41.99, 9.15, 0.22,
           0.06, 0.28]
ROW_LABELS = ["IoU", "Precision", "Recall", "mIoU", "car", "bicycle", "motorcycle", "truck",
              "other-vehicle", "person", "road", "sidewalk", "building", "fence", "vegetation",
              "terrain", "pole", "traffic-sign", "other-object"]


def convert_voxels(arr, map_dict):
    """evaluate_model_sscbench.py:857-859 (dict lookup per voxel; raises on unknown keys)."""
    keys = np.array(sorted(map_dict))
    a = np.asarray(arr).astype(np.int64)
    if not np.isin(a, keys).all():
        raise KeyError("convert_voxels: label without a mapping")
    lut = np.zeros(int(keys.max()) + 1, np.int64)
    for k, v in map_dict.items():
        lut[k] = v
    return lut[a]


def identify_additional_invalids(target):
    """:814-827: empty voxels below z = 7 with no labelled voxel strictly underneath."""
    nx, ny, nz = target.shape
    t = np.concatenate([np.zeros([nx, ny, 1]), target], axis=2)
    inv = np.cumsum(np.logical_and(t != 255, t != 0), axis=2)[:, :, :nz] == 0
    inv[:, :, 7:] = 0
    inv[target != 0] = 0
    return inv


def crop_bounds(size, ny=256):
    """:496-501: x in [0, n), y in [128 - n // 2, 128 + n // 2), n = int(size // 0.2)."""
    n = int(size // 0.2)
    return n, 128 - n // 2, 128 + n // 2


def confusion(y_pred, y_true, fov_mask):
    """bincount(16 y_true + y_pred) over y_true != 255 inside the FOV (:862-886)."""
    mask = np.logical_and(y_true != 255, fov_mask).flatten()
    yp = y_pred.flatten()[mask].astype(np.int64)
    yt = y_true.flatten()[mask].astype(np.int64)
    return np.bincount(16 * yt + yp, minlength=256).reshape(16, 16)


def frame_confusions(sigmas, segs, voxel_gt, fov_mask, sizes=SIZES, additional_invalids=True,
                     sigma_cutoff=SIGMA_CUTOFF):
    """One frame of the main loop (:366-367, 452-456, 492, 496-501): per-range 16 x 16
    confusion matrices (int64)."""
    segs = convert_voxels(segs, CITYSCAPES_TO_LABEL)
    target = convert_voxels(voxel_gt, SSCBENCH_TO_LABEL)
    if additional_invalids:
        target = target.copy()
        target[identify_additional_invalids(target) == 1] = 255
    segs = segs.copy()
    segs[sigmas < sigma_cutoff] = 0
    out = []
    for size in sizes:
        n, y0, y1 = crop_bounds(size)
        out.append(confusion(segs[:n, y0:y1, :], target[:n, y0:y1, :], fov_mask[:n, y0:y1, :]))
    return np.stack(out)


def counts_from_confusion(C):
    """The per-frame numbers of compute_occupancy_numbers (:908-925),
    compute_occupancy_numbers_segmentation (:862-886) and
    compute_occupancy_recall_segmentation (:889-905), all sums of one confusion matrix."""
    C = np.asarray(C, np.int64)
    tp = C[1:, 1:].sum(); fp = C[0, 1:].sum(); fn = C[1:, 0].sum(); tn = C[0, 0]
    d = np.diag(C)[1:]
    tp_seg = d
    fp_seg = C[:, 1:].sum(0) - d
    fn_seg = C[1:, :].sum(1) - d
    tn_seg = C.sum() - tp_seg - fp_seg - fn_seg
    tp_rec = C[1:, 1:].sum(1)
    sum_rec = C[1:, :].sum(1)
    return {"tp": int(tp), "fp": int(fp), "tn": int(tn), "fn": int(fn),
            "tp_seg": tp_seg, "fp_seg": fp_seg, "tn_seg": tn_seg, "fn_seg": fn_seg,
            "confusion_seg": C, "tp_recall_seg": tp_rec, "sum_recall_seg": sum_rec}


def results_tables(conf_by_size, sizes=SIZES):
    """:539-609 over accumulated confusion matrices {size: (16, 16)}: for mode "direct" and
    "hungarian" the (19, 3) table, mIoU and weighted mIoU (of the last range, as printed)."""
    from scipy.optimize import linear_sum_assignment
    out = {}
    for mode in ("direct", "hungarian"):
        table = np.zeros((19, len(sizes)), dtype=np.float32)
        if mode == "hungarian":
            assign = linear_sum_assignment(conf_by_size[sizes[-1]].astype(np.float64),
                                           maximize=True)
        miou = wmiou = None
        with np.errstate(divide="ignore", invalid="ignore"):
            for i, size in enumerate(sizes):
                c = counts_from_confusion(conf_by_size[size])
                tp, fp, fn = float(c["tp"]), float(c["fp"]), float(c["fn"])
                table[0, i] = tp / (tp + fp + fn)
                table[1, i] = tp / (tp + fp)
                table[2, i] = tp / (tp + fn)
                cm = conf_by_size[size].astype(np.float64)
                if mode == "hungarian":
                    cm = cm[np.argsort(assign[1]), :]
                d = np.diag(cm)
                denom = cm.sum(0) + cm.sum(1) - d
                per_class = d[1:] / denom[1:]
                miou = np.mean(np.nan_to_num(per_class))
                w = np.array(WEIGHTS)
                wmiou = np.sum(w * np.nan_to_num(per_class)) / np.sum(w)
                table[3, i] = miou
                table[4:, i] = per_class
        out[mode] = {"table": table, "miou": float(miou), "weighted_miou": float(wmiou),
                     "reassignment": (np.argsort(assign[1]) if mode == "hungarian" else None)}
    return out


def fov_mask(T, cam_k, dims=(256, 256, 32), origin=(0.0, -25.6, -2.0), vox=0.2,
             img_w=1408, img_h=376):
    """get_fov_mask / generate_point_grid (point_utils.py:6-82) with cam2pix
    (fusion.py:222-232) vectorised in fp64: vox2world's f32 centres, the f64 rigid transform
    as a sequential sum, pixel = round-half-even(x fx / z + cx) with f32 intrinsics."""
    nx, ny, nz = dims
    xv, yv, zv = np.meshgrid(range(nx), range(ny), range(nz), indexing="ij")
    c = np.stack([xv.reshape(-1), yv.reshape(-1), zv.reshape(-1)], 1).astype(np.float32)
    o32 = np.asarray(origin).astype(np.float32).astype(np.float64)
    p = ((o32[None] + vox * c.astype(np.float64)) + vox * 0.5).astype(np.float32).astype(np.float64)
    T = np.asarray(T, np.float64)
    cam = [((T[j, 0] * p[:, 0] + T[j, 1] * p[:, 1]) + T[j, 2] * p[:, 2]) + T[j, 3]
           for j in range(3)]
    k = np.asarray(cam_k).astype(np.float32).astype(np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        px = np.rint(cam[0] * k[0, 0] / cam[2] + k[0, 2])
        py = np.rint(cam[1] * k[1, 1] / cam[2] + k[1, 2])
    m = (px >= 0) & (px < img_w) & (py >= 0) & (py < img_h) & (cam[2] > 0)
    return m.reshape(dims)
