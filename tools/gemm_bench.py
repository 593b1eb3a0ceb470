#!/usr/bin/env python3
"""Diagnostic: sd_gemm on the encoder's GEMM shapes (ViT-B/8 and DINOv2-B/14 blocks, the DPT
output convolutions), microseconds per call (HIP events over 50 back-to-back calls, random
bf16 operands).  SD_GEMM_TILE=128|64|sk forces a tiling; SDHIP_LIB selects a variant."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scenedino_amd import _lib  # noqa: E402

dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)


def rnd(*s):
    return (torch.rand(*s, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)


def timeit(fn, n=50):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / n


res = {}
for name, T, C in (("vitb8", 1921, 768), ("dv2b14", 586, 768)):
    x = rnd(T, C)
    xf = torch.randn(T, C, device=dev, generator=g)
    for op, N, K, epi in (("qkv", 3 * C, C, _lib.SD_EPI_QKV), ("proj", C, C, _lib.SD_EPI_RESID),
                          ("fc1", 4 * C, C, _lib.SD_EPI_GELU), ("fc2", C, 4 * C, _lib.SD_EPI_RESID)):
        a = x if K == C else rnd(T, K)
        w = rnd(N, K)
        bias = torch.randn(N, device=dev, generator=g)
        if epi == _lib.SD_EPI_QKV:
            H = C // 64
            Tp = (T + 63) // 64 * 64
            q = torch.empty(1, H, T, 64, device=dev, dtype=torch.bfloat16)
            k = torch.zeros(1, H, Tp, 64, device=dev, dtype=torch.bfloat16)
            vt = torch.zeros(1, H, 64, Tp, device=dev, dtype=torch.bfloat16)
            fn = lambda: _lib.gemm(a, w, bias, epi, qkv=(q, k, vt), tokens=T, heads=H)
        elif epi == _lib.SD_EPI_RESID:
            fn = lambda: _lib.gemm(a, w, bias, epi, out=xf)
        else:
            o = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
            fn = lambda: _lib.gemm(a, w, bias, epi, out=o)
        us = timeit(fn)
        res[f"{name}.{op}"] = {"us": round(us, 2), "tflops": round(2 * T * N * K / us / 1e6, 1)}
for name, H, W in (("dpt_out192x640", 192, 640), ("dpt_head96x320", 96, 320)):
    x = rnd(1, H, W, 256)
    w = rnd(256, 9 * 256)
    bias = torch.randn(256, device=dev, generator=g)
    o = torch.empty(1, H, W, 256, device=dev)
    fn = lambda: _lib.conv3x3(x, w, bias, epi=_lib.SD_EPI_F32, out=o)
    us = timeit(fn, 20)
    res[name] = {"us": round(us, 2), "tflops": round(2 * H * W * 256 * 9 * 256 / us / 1e6, 1)}
print(json.dumps({"lib": os.environ.get("SDHIP_LIB", "default"), "tile": os.environ.get("SD_GEMM_TILE", "auto"),
                  "res": res}))
