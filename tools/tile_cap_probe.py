#!/usr/bin/env python3
"""Diagnostic: C2 frame time (offset and identity render poses) as a function of the tile
buffer size (sd_render_tile_cap), for the slope of the tile kernel's restaging cost.
SDHIP_TILE_RPW=2 runs K = 64 two rays per wave.  usage: tile_cap_probe.py [cap_kib ...]"""
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from scenedino_amd import _lib  # noqa: E402


def frame_ms(offset, n=20):
    dev = torch.device("cuda:0")
    net, renderer, wrapper, sampler, pose, Ks = bench.make_scene(0, dev, "bf16", offset)
    with torch.no_grad():
        for _ in range(5):
            bench.render_step(net, wrapper, sampler, pose, Ks)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            bench.render_step(net, wrapper, sampler, pose, Ks)
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


_lib.load()
caps = [int(a) for a in sys.argv[1:]] or [0]
for cap in caps:
    _lib.render_tile_cap(cap * 1024)
    print(f"cap {cap:3d} KiB: offset {frame_ms(True):.4f} ms  identity {frame_ms(False):.4f} ms", flush=True)
_lib.render_tile_cap(0)
