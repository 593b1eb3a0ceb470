"""Build libsdhip.so (all gfx950 HIP kernels + the C ABI) in-tree with hipcc."""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SOURCES = ["csrc/sdhip_rays.hip", "csrc/sdhip_field.hip", "csrc/sdhip_proj.hip", "csrc/sdhip_tile.hip",
           "csrc/sdhip_seg.hip", "csrc/sdhip_vit.hip", "csrc/sdhip_train.hip"]
OUT = os.path.join(HERE, "libsdhip.so")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
         "-DSD_FASTPE=0", "-Wno-unused-result",
         # MFMA accumulators in arch VGPRs (no v_accvgpr copies before VALU epilogues);
         # no SLP packing of f32 math into v_pk_*_f32 (an issue-cost loss beside MFMAs)
         "-mllvm", "-amdgpu-mfma-vgpr-form=1", "-fno-slp-vectorize"]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def build(force: bool = False, verbose: bool = False) -> str:
    srcs = [os.path.join(HERE, s) for s in SOURCES]
    deps = srcs + [os.path.join(HERE, "csrc", "sdhip_common.h"), os.path.join(HERE, "csrc", "sdhip_point.h"),
            os.path.join(HERE, "csrc", "sdhip_render.h"),
                   os.path.join(HERE, "..", "include", "sdhip.h")]
    if not force and os.path.exists(OUT):
        t = os.path.getmtime(OUT)
        if all(os.path.getmtime(d) <= t for d in deps):
            return OUT
    cmd = [hipcc()] + FLAGS + ["-o", OUT + ".tmp"] + srcs
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
