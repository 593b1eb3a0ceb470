"""Diagnostic: measured errors of the 16-bit tile renders against the reference's full-frame
renders of configs[0] (K = 32, whole frame) and configs[3] (K = 128, 384-d head, every 61st
ray) -- the numbers behind tests/test_gpu_parity.py's bounds.
usage: python tools/parity_full.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from _fullscene import render_offset_fixture  # noqa: E402


def rel_l2(a, b):
    a = torch.as_tensor(a).double().cpu().reshape(-1)
    b = torch.as_tensor(np.asarray(b)).double().reshape(-1)
    return float((a - b).norm() / b.norm())


def main():
    for name in ("render_full_offset_k32", "render_c4_offset"):
        d = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"), allow_pickle=False)
        idx = torch.from_numpy(d["idx"])
        for prec in ("bf16", "fp16"):
            c = render_offset_fixture(d, prec, "cuda", **({"whole_frame": True} if "c4" in name else {}))
            dep = c["depth"][0].cpu()[idx].double()
            ref = torch.from_numpy(np.asarray(d["depth"])).double().reshape(dep.shape)
            w = c["weights"][0].cpu()[idx].double()
            wr = torch.from_numpy(np.asarray(d["weights"])).double().reshape(w.shape)
            print(f"{name:24s} {prec}: depth max |d| {float((dep - ref).abs().max()):.3e} m, "
                  f"depth rel-L2 {rel_l2(dep, ref):.2e}, weights max |d| {float((w - wr).abs().max()):.2e}, "
                  f"dino rel-L2 {rel_l2(c['dino_features'][0].cpu()[idx], d['dino']):.2e}", flush=True)


if __name__ == "__main__":
    main()
