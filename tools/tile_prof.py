"""Diagnostic: per-phase cycle shares of k_render_tile from an ST_PROF=1 variant build
(tools/variants.sh 'prof=-DST_PROF=1'; run with SDHIP_LIB=.../libsdhip_prof.so)."""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from scenedino_amd import _lib  # noqa: E402

NAMES = ["ray_pass", "head", "itemA0", "ray_col", "barrier_X", "stage", "items", "epilogue",
         "vmcnt", "barrier_Y", " rp:z", " rp:geo", " rp:box",
         " it:rec+addr", " it:tr+blend", " it:code+relu", " it:sig..scan", " it:w", " it:hc"]


def main():
    offset = "--identity" not in sys.argv
    for a in sys.argv[1:]:
        if a.startswith("--k="):  # samples per ray (C1: 32)
            bench.K_SAMPLES = int(a[4:])
    dev = torch.device("cuda:0")
    net, renderer, wrapper, sampler, pose, Ks = bench.make_scene(0, dev, "bf16", offset)
    f = _lib.load().sd_tile_prof
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * 32)()
    with torch.no_grad():
        for _ in range(3):
            bench.render_step(net, wrapper, sampler, pose, Ks)
        torch.cuda.synchronize()
        f(buf, 1)
        n = 10
        for _ in range(n):
            bench.render_step(net, wrapper, sampler, pose, Ks)
        torch.cuda.synchronize()
        f(buf, 1)
    waves = buf[31]
    tot = sum(buf[i] for i in range(10))  # 10..12 subdivide ray_pass
    print(f"{'offset' if offset else 'identity'} K={bench.K_SAMPLES}: waves {waves}, cycles per wave {tot / max(waves, 1):.0f}")
    for i, nm in enumerate(NAMES):
        print(f"  {nm:10s} {buf[i] / max(waves, 1):10.0f} cyc/wave  {100 * buf[i] / max(tot, 1):5.1f}%")


main()
