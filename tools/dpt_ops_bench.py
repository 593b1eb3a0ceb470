#!/usr/bin/env python3
"""Diagnostic: the DPT head's large layers for a 192x640 frame one by one (256 channels:
the residual-unit 3x3 convolutions at 48x160 with pre-ReLU and residuals, the 3x3
convolutions at 96x320 and 192x640, the ConvTranspose2d(2, 2) at 96x320), microseconds per
call (HIP events around graph replays of 20 back-to-back calls, random operands).
SDHIP_LIB selects a variant build; SD_CONV_BIG=0 the k_gemm path."""
import json
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
    """Device time per call (us): n calls captured in one HIP graph, replayed 5 times."""
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
C = 256
w3 = rnd(C, 9 * C, scale=1 / math.sqrt(9 * C))
b = torch.zeros(C, device=dev)
res = {}
for name, (H, W, kw) in {
        "rcu48x160_relu": (48, 160, dict(relu_in=True)),
        "rcu48x160_relu_res": (48, 160, dict(relu_in=True, res=True)),
        "conv96x320": (96, 320, {}),
        "conv192x640_f32": (192, 640, dict(epi=_lib.SD_EPI_F32))}.items():
    x = rnd(1, H, W, C)
    if kw.pop("res", False):
        kw["res"], kw["res2"] = rnd(1, H, W, C), rnd(1, H, W, C)
    out = torch.empty(1, H, W, C, device=dev,
                      dtype=torch.float32 if kw.get("epi") == _lib.SD_EPI_F32 else torch.bfloat16)
    us = timeit(lambda: _lib.conv3x3(x, w3, b, out=out, **kw))
    res[name] = {"us": round(us, 2), "tflops": round(2 * H * W * C * 9 * C / us / 1e6, 1)}
x = rnd(1, 96, 320, C)
wt = rnd(4 * C, C, scale=1 / math.sqrt(C))
bt = torch.zeros(4 * C, device=dev)
out = torch.empty(1, 192, 640, C, device=dev, dtype=torch.bfloat16)
us = timeit(lambda: _lib.linear_nhwc(x, wt, bt, shuf=2, out=out))
res["convT96x320_shuf"] = {"us": round(us, 2), "GBps_out": round(out.numel() * 2 / us / 1e3, 1)}
print(json.dumps({"lib": os.environ.get("SDHIP_LIB") or "main",
                  "conv_big": os.environ.get("SD_CONV_BIG", "1"), "ops": res}))
