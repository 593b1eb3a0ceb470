"""Tap-box statistics of the tile render kernel (k_render_tile, sdhip_tile.hip) for the
C2 bench frame: per 8-ray group, the staged texel count th * pitch(tw) of the union of its
bilinear tap boxes, and the share of groups over a given tile capacity.  CPU only."""
import math
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from oracle import render_oracle as O  # noqa: E402


def pitch(tw):
    r = tw & 7
    return tw + (3 if r == 7 else 2 if r == 0 else 1 if r == 1 else 0)


def stats(offset):
    pose = torch.eye(4)
    rp = bench.offset_render_pose(pose) if offset else pose
    K = torch.tensor(bench.KITTI_K)
    rays = O.gen_rays(rp.view(1, 4, 4), K.view(1, 3, 3), bench.H, bench.W).numpy()
    Ks = bench.K_SAMPLES
    g = np.random.default_rng(0)
    t = np.linspace(0, 1 - 1 / Ks, Ks, dtype=np.float32)[None] + g.random((len(rays), Ks), dtype=np.float32) / Ks
    near, far = rays[:, 6:7], rays[:, 7:8]
    z = 1 / ((1 / near) * (1 - t) + (1 / far) * t)
    p = rays[:, None, :3] + z[..., None] * rays[:, None, 3:6]
    Kn = K.numpy()
    i = p @ Kn.T
    zd = np.maximum(i[..., 2], 1e-3)
    x = np.clip(i[..., 0] / zd, -2, 2)
    y = np.clip(i[..., 1] / zd, -2, 2)
    Wf, Hf = bench.WF, bench.HF
    ix = np.clip(((x + 1) * Wf - 1) / 2, 0, Wf - 1)
    iy = np.clip(((y + 1) * Hf - 1) / 2, 0, Hf - 1)
    x0 = np.floor(ix).astype(np.int32)
    y0 = np.floor(iy).astype(np.int32)
    G = len(rays) // 8
    x0 = x0.reshape(G, -1)
    y0 = y0.reshape(G, -1)
    tw = x0.max(1) + 2 - x0.min(1)
    th = y0.max(1) + 2 - y0.min(1)
    ntex = th * np.vectorize(pitch)(tw)
    return ntex


for off in (False, True):
    n = stats(off)
    caps = [96, 120, 136, 152, 177, 200, 240]
    print("offset" if off else "identity", "p50/p90/p99/max", np.percentile(n, [50, 90, 99]).astype(int), n.max(),
          " over cap:", {c: f"{(n > c).mean() * 100:.2f}%" for c in caps})
