"""Build libsdhip.so (all gfx950 HIP kernels + the C ABI) in-tree with hipcc.

Each translation unit compiles to its own object (in parallel, rebuilt only when the unit
or a shared header changed), then one link step writes the shared library."""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
SOURCES = ["csrc/sdhip_rays.hip", "csrc/sdhip_field.hip", "csrc/sdhip_proj.hip", "csrc/sdhip_tile.hip",
           "csrc/sdhip_seg.hip", "csrc/sdhip_ssc.hip", "csrc/sdhip_vit.hip", "csrc/sdhip_train.hip",
           "csrc/sdhip_down.hip", "csrc/sdhip_mlp.hip", "csrc/sdhip_conv.hip"]
HEADERS = ["csrc/sdhip_common.h", "csrc/sdhip_point.h", "csrc/sdhip_render.h", "../include/sdhip.h"]
OUT = os.path.join(HERE, "libsdhip.so")
OBJ_DIR = os.path.join(HERE, "_obj")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC",
         "-DSD_FASTPE=0", "-Wno-unused-result",
         # MFMA accumulators in arch VGPRs (no v_accvgpr copies before VALU epilogues);
         # no SLP packing of f32 math into v_pk_*_f32 (an issue-cost loss beside MFMAs)
         "-mllvm", "-amdgpu-mfma-vgpr-form=1", "-fno-slp-vectorize"]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, jobs: int = 8) -> str:
    srcs = [os.path.join(HERE, s) for s in SOURCES]
    hdrs = [os.path.join(HERE, h) for h in HEADERS]
    os.makedirs(OBJ_DIR, exist_ok=True)
    objs = [os.path.join(OBJ_DIR, os.path.basename(s) + ".o") for s in srcs]
    todo = [(s, o) for s, o in zip(srcs, objs) if force or _stale(o, [s] + hdrs)]

    def compile_one(so):
        s, o = so
        cmd = [hipcc()] + FLAGS + ["-c", "-o", o + ".tmp", s]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(o + ".tmp", o)

    if todo:
        with ThreadPoolExecutor(max_workers=max(1, min(jobs, len(todo)))) as ex:
            list(ex.map(compile_one, todo))
    if force or todo or _stale(OUT, objs):
        cmd = [hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT + ".tmp"] + objs
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
