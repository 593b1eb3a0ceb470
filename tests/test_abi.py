"""CPU: the C-ABI library loads and exports every entry point include/sdhip.h declares
(no compute calls: there is no GPU here)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def declared_functions():
    src = open(os.path.join(ROOT, "include", "sdhip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sd_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    names = declared_functions()
    for n in ("sd_gen_rays", "sd_sample_z", "sd_render_fused", "sd_field_query", "sd_composite",
              "sd_pack_grid", "sd_pack_image", "sd_last_error", "sd_abi_version"):
        assert n in names


def test_library_exports_every_declared_symbol():
    from scenedino_amd import _lib
    lib = _lib.load()
    for name in declared_functions():
        assert hasattr(lib, name), f"libsdhip.so does not export {name}"
        assert name in _lib.SIGNATURES, f"{name} has no ctypes signature in _lib"


def test_abi_version_and_error_string():
    from scenedino_amd import _lib
    lib = _lib.load()
    assert lib.sd_abi_version() == _lib.ABI_VERSION
    assert isinstance(lib.sd_last_error(), bytes)


def test_invalid_arguments_return_error_without_gpu():
    """Argument validation happens before any HIP call, so it is testable on CPU."""
    from scenedino_amd import _lib
    lib = _lib.load()
    rc = lib.sd_gen_rays(None, None, None, 0, 0, 0, 3.0, 80.0, None, None)
    assert rc == -1 and b"invalid" in lib.sd_last_error()
    rc = lib.sd_render_fused(None, None, None)
    assert rc == -1


def test_struct_layouts_match_the_c_header(tmp_path):
    """ctypes mirrors of the ABI structs have the C compiler's sizes and offsets."""
    import subprocess
    from scenedino_amd import _lib
    structs = {"sd_mlp": _lib.SdMlp, "sd_render_args": _lib.SdRenderArgs,
               "sd_field_args": _lib.SdFieldArgs, "sd_head": _lib.SdHead,
               "sd_seg_head": _lib.SdSegHead, "sd_gemm_args": _lib.SdGemmArgs,
               "sd_ssc_args": _lib.SdSscArgs, "sd_patch_args": _lib.SdPatchArgs,
               "sd_salience_args": _lib.SdSalienceArgs,
               "sd_mlp_train_args": _lib.SdMlpTrainArgs, "sd_wgrad_args": _lib.SdWgradArgs,
               "sd_mlp_wgrad_args": _lib.SdMlpWgradArgs, "sd_frame_args": _lib.SdFrameArgs}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "sdhip.h"', "int main(void){"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {}
    for line in out:
        if line:
            c, f, v = line.split()
            got[(c, f)] = int(v)
    for cname, py in structs.items():
        assert ctypes.sizeof(py) == got[(cname, "size")], cname
        for fname, _ in py._fields_:
            assert getattr(py, fname).offset == got[(cname, fname)], (cname, fname)


def test_field_dtype_and_grid_dtype_rejection_without_gpu():
    """ABI 10: the bf16 mode's render / field kernels read f16 grids; the library
    states that through sd_field_dtype and rejects a grid_dtype that differs instead of
    reading bf16 bits as f16 (validation runs before any HIP call)."""
    from scenedino_amd import _lib
    lib = _lib.load()
    assert lib.sd_field_dtype(_lib.SD_F32) == _lib.SD_F32
    assert lib.sd_field_dtype(_lib.SD_BF16) == _lib.SD_F16
    assert lib.sd_field_dtype(_lib.SD_F16) == _lib.SD_F16
    assert lib.sd_field_dtype(7) == -1
    for mode in (_lib.SD_BF16, _lib.SD_F16):
        assert _lib.FIELD_DTYPE[mode] == lib.sd_field_dtype(mode)
    head = _lib.SdHead(w_pe=16, w_sig=16, w_out=16, b_dino=16, b_sigma=0.0, D=64,
                       dtype=_lib.SD_BF16)
    args = _lib.SdRenderArgs(grid_dtype=_lib.SD_BF16, work=16)
    rc = lib.sd_render_proj(ctypes.byref(args), ctypes.byref(head), None)
    assert rc == -1 and b"grid_dtype" in lib.sd_last_error()


def test_reserve_cus_setter_without_gpu():
    """sd_reserve_cus is a process-wide setter returning the previous value (no HIP call)."""
    from scenedino_amd import _lib
    prev = _lib.reserve_cus(16)
    try:
        assert _lib.reserve_cus(24) == 16
        assert _lib.reserve_cus(-3) == 24  # negative clamps to 0
        assert _lib.reserve_cus(0) == 0
    finally:
        _lib.reserve_cus(prev)
    lib = _lib.load()
    assert lib.sd_spin(0, 1.0, None) == -1 and b"sd_spin" in lib.sd_last_error()


def test_seg_record_layout_rejection_without_gpu():
    """ABI 11: sd_seg_head.frag_layout names the record's MFMA fragment maps; an unknown
    layout, or the fp8 norm (32x32 maps only) on a 16x16 record, is rejected before any HIP
    call.  The CPU packer writes the layout it built."""
    import torch
    from scenedino_amd import _lib
    from scenedino_amd.seg_pack import PackedSegHead
    lib = _lib.load()
    dr = torch.nn.Module()
    dr.linear_in, dr.linear_out = torch.nn.Linear(64, 128), torch.nn.Linear(128, 768)
    assert PackedSegHead(dr).rec.frag_layout == _lib.SD_SEG_FRAG16
    assert PackedSegHead(dr, mfma=32).rec.frag_layout == _lib.SD_SEG_FRAG32
    with pytest.raises(ValueError):
        PackedSegHead(dr, mfma=8)
    for layout, w2_f8, what in ((5, None, b"frag_layout"), (_lib.SD_SEG_FRAG16, 16, b"fp8")):
        rec = _lib.SdSegHead(w1=16, b1=16, w2=16, b2=16, wg=16, g2=16, d_in=64, d_latent=128,
                             d_full=768, frag_layout=layout, w2_f8=w2_f8)
        rc = lib.sd_seg_query(16, _lib.SD_BF16, 32, ctypes.byref(rec), None, 0.2, None, None,
                              16, None)
        assert rc == -1 and what in lib.sd_last_error()
