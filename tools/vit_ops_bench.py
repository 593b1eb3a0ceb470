#!/usr/bin/env python3
"""Diagnostic: the ViT block's kernels at 481 tokens one by one (ViT-S/16: C 384, 6 heads;
DINOv2-B/14: C 768, 12 heads), microseconds per call (HIP events around graph replays of 20
back-to-back calls, random operands).  SDHIP_LIB selects a variant build."""
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


def timeit(fn, n=20):
    """Device time per call: n calls captured in one HIP graph, replayed 5 times (eager
    ctypes calls from Python are host-bound at ~8 us each)."""
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
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        gph.replay()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) * 1e3 / (5 * n), 2)


_lib.load()
res = {}
T = int(os.environ.get("TOKENS", "481"))
for name, C in (("vit-s16", 384), ("dinov2-b14", 768)):
    H = C // 64
    Tp = (T + 63) // 64 * 64
    x = torch.randn(T, C, device=dev, generator=g)
    xn = torch.empty(T, C, device=dev, dtype=torch.bfloat16)
    lw, lb = torch.rand(C, device=dev, generator=g) + 0.5, torch.randn(C, device=dev, generator=g) * 0.1
    q = torch.empty(1, H, T, 64, device=dev, dtype=torch.bfloat16)
    k = torch.zeros(1, H, Tp, 64, device=dev, dtype=torch.bfloat16)
    vt = torch.zeros(1, H, 64, Tp, device=dev, dtype=torch.bfloat16)
    ao = torch.empty(T, C, device=dev, dtype=torch.bfloat16)
    hid = torch.empty(T, 4 * C, device=dev, dtype=torch.bfloat16)
    wqkv, bqkv = rnd(3 * C, C), torch.randn(3 * C, device=dev, generator=g) * 0.1
    wp, bp = rnd(C, C), torch.randn(C, device=dev, generator=g) * 0.1
    w1, b1 = rnd(4 * C, C), torch.randn(4 * C, device=dev, generator=g) * 0.1
    w2, b2 = rnd(C, 4 * C), torch.randn(C, device=dev, generator=g) * 0.1
    gam = torch.rand(C, device=dev, generator=g)
    r = {}
    r["layernorm"] = timeit(lambda: _lib.layernorm(x, lw, lb, 1e-6, xn))
    r["ln_gemm_qkv"] = timeit(lambda: _lib.ln_gemm(x, lw, lb, 1e-6, wqkv, bqkv, _lib.SD_EPI_QKV,
                                                   qkv=(q, k, vt), tokens=T, heads=H))
    r["gemm_qkv"] = timeit(lambda: _lib.gemm(xn, wqkv, bqkv, _lib.SD_EPI_QKV, qkv=(q, k, vt),
                                             tokens=T, heads=H))
    r["attention"] = timeit(lambda: _lib.attention(q, k, vt, 0.125, ao))
    r["gemm_proj_resid"] = timeit(lambda: _lib.gemm(ao, wp, bp, _lib.SD_EPI_RESID, out=x, gamma=gam))
    r["ln_gemm_fc1"] = timeit(lambda: _lib.ln_gemm(x, lw, lb, 1e-6, w1, b1, _lib.SD_EPI_GELU, out=hid))
    r["gemm_fc1"] = timeit(lambda: _lib.gemm(xn, w1, b1, _lib.SD_EPI_GELU, out=hid))
    r["gemm_fc2_resid"] = timeit(lambda: _lib.gemm(hid, w2, b2, _lib.SD_EPI_RESID, out=x, gamma=gam))
    res[name] = r
print(json.dumps({"lib": os.environ.get("SDHIP_LIB", "default"), "tokens": T, "res": res}))
