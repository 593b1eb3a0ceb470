"""Time k_seg_head (labels only, the C5 launch shape: 256x256x32 voxels, d_full 768,
19 clusters) with HIP events; SDHIP_LIB selects the library (timing experiments)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from scenedino_amd import _lib  # noqa: E402
from scenedino_amd.seg_pack import PackedSegHead  # noqa: E402
from scenedino_amd.models.backbones.dino import MlpDimReduction  # noqa: E402
from scenedino_amd.downstream_head import SemanticHead  # noqa: E402

_lib.load()
torch.manual_seed(0)
dev = "cuda"
dr = MlpDimReduction(768, 64, 128).to(dev).eval()
sh = SemanticHead(19, 19, 768, 64).to(dev).eval()
pk = PackedSegHead(dr, sh.stego_head, sh.stego_cluster_head)
P = 256 * 256 * 32
x = torch.randn(P, 64, device=dev)
for _ in range(3):
    _lib.seg_query(x, pk.rec, want_labels=True)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
e0.record()
for _ in range(20):
    _lib.seg_query(x, pk.rec, want_labels=True)
e1.record()
torch.cuda.synchronize()
print(f"{os.environ.get('SDHIP_LIB', 'default')}: k_seg_head {e0.elapsed_time(e1) / 20 * 1e3:.1f} us")
