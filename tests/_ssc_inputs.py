"""Seeded synthetic SSCBench frames (shared by tests/golden/make_golden.py and the tests).

numpy's PCG64 stream is stable across platforms, so the fixture stores only the counts
the reference produced for these inputs, not the 2M-voxel inputs themselves."""
from __future__ import annotations

import numpy as np

DIMS = (256, 256, 32)
TARGET_KEYS = list(range(20)) + [255]


def make_frame(seed: int, dims=DIMS):
    """-> sigmas (f32), segs (uint8 cityscapes classes 0..18), voxel_gt (uint8 raw SSCBench
    labels incl. 255), all (nx, ny, nz).  Ground truth is column-structured (empty space
    above a labelled surface, unlabelled gaps) so the additional-invalid scan matters."""
    rng = np.random.default_rng(1000 + seed)
    nx, ny, nz = dims
    p = np.full(len(TARGET_KEYS), 0.25 / 19)
    p[0], p[-1] = 0.6, 0.15
    gt = rng.choice(np.array(TARGET_KEYS, np.uint8), size=dims, p=p / p.sum())
    ground = rng.integers(0, 9, size=(nx, ny, 1))
    z = np.arange(nz)[None, None, :]
    gt = np.where(z > ground + 3, np.uint8(0), gt).astype(np.uint8)
    segs = rng.integers(0, 19, size=dims).astype(np.uint8)
    sigmas = rng.exponential(0.6, size=dims).astype(np.float32)
    return sigmas, segs, gt
