"""Diagnostic: the DPT's 192x640 output convolution (3x3, 256 -> 256, f32 out) on the
256 x 256 im2col tiles (shipped) vs the 8 x 32-pixel halo tiles of all 256 output channels
(SD_CONV_HALO256=1, the default since round 6): max |difference| and microseconds per call (HIP graph of 20 calls)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scenedino_amd import _lib  # noqa: E402

dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)


def rnd(*s, scale=1.0):
    return ((torch.rand(*s, device=dev, generator=g) * 2 - 1) * scale).to(torch.bfloat16)


def timeit(fn, n=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    gph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gph):
        for _ in range(n):
            fn()
    gph.replay()
    torch.cuda.synchronize()
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        gph.replay()
    e.record()
    torch.cuda.synchronize()
    return a.elapsed_time(e) * 1e3 / (5 * n)


_lib.load()
C, H, W = 256, 192, 640
w3 = rnd(C, 9 * C, scale=1 / math.sqrt(9 * C))
b = torch.randn(C, device=dev, generator=g) * 0.1
x = rnd(1, H, W, C)
outs = {}
for mode in ("0", "1", "0", "1"):
    os.environ["SD_CONV_HALO256"] = mode
    out = torch.empty(1, H, W, C, device=dev, dtype=torch.float32)
    us = timeit(lambda: _lib.conv3x3(x, w3, b, out=out, epi=_lib.SD_EPI_F32))
    outs[mode] = out.clone()
    print(f"halo256={mode}: {us:7.2f} us  {2 * H * W * C * 9 * C / us / 1e6:7.1f} TFLOP/s", flush=True)
d = (outs["0"] - outs["1"]).abs().max().item()
print(f"max |im2col - halo| = {d:.3e} (bit-equal: {torch.equal(outs['0'], outs['1'])})")
