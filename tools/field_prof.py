"""Diagnostic: per-phase cycle shares of k_field (the C5 voxel field query) from an
SD_FQ_PROF=1 variant build (tools/build_variant.py fqprof -DSD_FQ_PROF=1; run with
SDHIP_LIB=scenedino_amd/variants/fqprof.so)."""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from scenedino_amd import _lib, sscbench  # noqa: E402

NAMES = ["grid chunks (blend + layer 1 + tap waits)", "open next tile + its tap loads",
         "code chunks + sigma", "output layer + dino stores", "sigma / mask stores, loop",
         "next tile's points"]


def main():
    dev = torch.device("cuda:0")
    net, pts, dims = bench.c5_scene(dev, "bf16", 0)
    f = _lib.load().sd_field_prof
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * 8)()
    with torch.no_grad():
        for _ in range(2):
            net._grid_cache = None
            sscbench.query_voxels(net, pts, dims)
        torch.cuda.synchronize()
        f(buf, 1)
        n = 3
        for _ in range(n):
            net._grid_cache = None
            sscbench.query_voxels(net, pts, dims)
        torch.cuda.synchronize()
        f(buf, 0)
    tot = sum(buf[i] for i in range(len(NAMES)))
    waves = 2048 * n
    print(f"k_field phase split (s_memtime ticks per wave, {n} launches x 2048 waves)")
    for i, nm in enumerate(NAMES):
        print(f"  {nm:45s} {buf[i] / waves:12.0f}  {100.0 * buf[i] / tot:5.1f} %")


if __name__ == "__main__":
    main()
