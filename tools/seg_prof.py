"""Diagnostic: per-phase cycle shares of k_seg_head from an SG_PROF=1 variant build
(tools/seg_variants.sh prof -DSG_PROF=1; run with SDHIP_LIB=scenedino_amd/_exp/prof.so)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from scenedino_amd import _lib  # noqa: E402
from scenedino_amd.seg_pack import PackedSegHead  # noqa: E402
from scenedino_amd.models.backbones.dino import MlpDimReduction  # noqa: E402
from scenedino_amd.downstream_head import SemanticHead  # noqa: E402

NAMES = ["layer1", "norm(gram)", "L path", "M loop misc", "M landed", "M frag+mfma issue",
         "M epilogue+Wn2", "k-means"]
lib = _lib.load()
f = lib.sd_seg_prof
f.argtypes = [ctypes.c_void_p, ctypes.c_int]
torch.manual_seed(0)
dev = "cuda"
dr = MlpDimReduction(768, 64, 128).to(dev).eval()
sh = SemanticHead(19, 19, 768, 64).to(dev).eval()
pk = PackedSegHead(dr, sh.stego_head, sh.stego_cluster_head)
x = torch.randn(256 * 256 * 32, 64, device=dev).to(torch.bfloat16)  # C5 passes bf16 codes
buf = (ctypes.c_ulonglong * 16)()
_lib.seg_query(x, pk.rec, want_labels=True)
torch.cuda.synchronize()
f(buf, 1)
for _ in range(5):
    _lib.seg_query(x, pk.rec, want_labels=True)
torch.cuda.synchronize()
f(buf, 0)
waves = buf[15]
tot = sum(buf[i] for i in range(len(NAMES)))
print(f"waves {waves}, cycles per wave {tot / waves:.0f}")
for i, n in enumerate(NAMES):
    print(f"{n:22s} {buf[i] / waves:9.0f} cyc/wave  {100 * buf[i] / tot:5.1f} %")
