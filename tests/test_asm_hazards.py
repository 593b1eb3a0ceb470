"""The inline-asm DPP statements of the render / ViT kernels are free of VALU-write ->
DPP-read hazards in the code the compiler actually emits (the compiler's hazard recognizer
does not look inside asm statements; round 5 found one in k_render_tile's hidden-sum
epilogue, where an f16 -> f32 conversion was scheduled directly in front of the DPP that
read it).  Compiles the device code of every source with inline-asm DPP (sdhip_render.h is
included by the render kernels) with the library's flags and scans it
(tools/dpp_hazard_scan.py).  CPU-only: hipcc cross-compiles gfx950."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.mark.parametrize("src", ["sdhip_tile.hip", "sdhip_proj.hip", "sdhip_vit.hip"])
def test_no_dpp_hazards_in_inline_asm(src, tmp_path):
    from scenedino_amd import build
    try:
        hipcc = build.hipcc()
    except RuntimeError:
        pytest.skip("hipcc not available")
    out = tmp_path / (src + ".s")
    flags = [f for f in build.FLAGS if f != "-fPIC"]
    subprocess.run([hipcc] + flags + ["--cuda-device-only", "-S", "-o", str(out),
                                      os.path.join(ROOT, "scenedino_amd", "csrc", src)],
                   check=True, capture_output=True)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "dpp_hazard_scan.py"), str(out)],
                       check=True, capture_output=True, text=True)
    assert r.stdout.strip().splitlines()[-1] == "hazards 0", r.stdout[-2000:]
