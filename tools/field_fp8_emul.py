"""Diagnostic: what an fp8 (OCP e4m3) projected grid P would do to the C5 voxel query
(fp8 for the field MLP's first layer).  P = W_in[:, :C] G + b_in is the
first layer's grid part (sd_project_grid); an fp8-P field kernel would gather e4m3 taps and
widen them to f16 for the blend (v_cvt_scalef32_pk_f16_fp8 is exact), so the f16 kernel run on
P rounded to e4m3 (per-tensor power-of-two scale s, values e4m3(P s) / s, exact in f16) gives
that kernel's outputs.  Reports sigma rel-L2 and the label / seg agreement of the C5 scene
against the unquantised run (sigma rel-L2 <= 5e-2, labels >= 99 %).
usage: field_fp8_emul.py [--scale=tensor|block32|none]"""
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from scenedino_amd import _lib, sscbench  # noqa: E402


def rel_l2(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def main():
    mode = "tensor"
    for a in sys.argv[1:]:
        if a.startswith("--scale="):
            mode = a[8:]
    dev = torch.device("cuda:0")
    net, pts, dims = bench.c5_scene(dev, "bf16")
    rec = net._seg_rec(True)
    xyz = pts.reshape(1, -1, 3)
    out = {}
    with torch.no_grad():
        for name in ("ref", "fp8"):
            net._grid_cache = None
            gc = net._grids()
            m = net._mlp()
            P = net._grid_proj(gc, m)  # (B, Hf, Wf, 128) f16, cached in gc
            if name == "fp8":
                Pf = P.float()
                if mode == "block32":
                    # MX-style: one power-of-two (E8M0) scale per 32 consecutive hidden
                    # channels of a grid pixel -- the K-block v_mfma_scale_f32_*_f8f6f4
                    # consumes (cbsz / blgp scale operands)
                    blk = Pf.reshape(*Pf.shape[:-1], Pf.shape[-1] // 32, 32)
                    amax = blk.abs().amax(-1, keepdim=True).clamp_min(1e-30)
                    s = torch.exp2(torch.floor(torch.log2(448.0 / amax)))
                    q = ((blk * s).to(torch.float8_e4m3fn).float() / s).reshape(Pf.shape)
                    sl = torch.log2(s)
                    desc = f"per-32-channel block scales 2^{int(sl.min())}..2^{int(sl.max())}"
                else:
                    s = 1.0
                    if mode == "tensor":
                        mx = float(Pf.abs().max())
                        s = 2.0 ** int(torch.floor(torch.log2(torch.tensor(448.0 / mx))))
                    q = (Pf * s).to(torch.float8_e4m3fn).float() / s
                    desc = f"scale 2^{int(torch.log2(torch.tensor(s)))}"
                P.copy_(q.to(P.dtype))
                print(f"P: max |P| {float(Pf.abs().max()):.3f}, {desc}, "
                      f"P rel-L2 after e4m3 {rel_l2(q, Pf):.3e}")
            sig, dino, _, _, _ = net.query(xyz, colors=False, dino_dtype=torch.bfloat16)
            Pn = sig.numel()
            lab, seg, _ = _lib.seg_query(dino.reshape(Pn, -1), rec.rec, sigma=sig.reshape(Pn),
                                         voxel_size=sscbench.VOXEL_SIZE, want_labels=True, want_seg=True)
            out[name] = (sig.reshape(-1).clone(), dino.reshape(Pn, -1).float().clone(), lab.clone(), seg.clone())
    # the same scene in the fp16 mode (dino output layer on f16 instead of bf16 MFMA): the
    # label agreement two accepted 16-bit modes reach on this random-weight scene
    net16, _, _ = bench.c5_scene(dev, "fp16")
    with torch.no_grad():
        sig, dino, _, _, _ = net16.query(xyz, colors=False, dino_dtype=torch.bfloat16)
        Pn = sig.numel()
        lab, seg, _ = _lib.seg_query(dino.reshape(Pn, -1), net16._seg_rec(True).rec, sigma=sig.reshape(Pn),
                                     voxel_size=sscbench.VOXEL_SIZE, want_labels=True, want_seg=True)
        out["fp16"] = (sig.reshape(-1), dino.reshape(Pn, -1).float(), lab, seg)
    s0, d0, l0, g0 = out["ref"]
    occ = g0 > 0
    for name, what in (("fp8", f"fp8 P ({mode} scale) vs f16 P, bf16 mode"),
                       ("fp16", "fp16 mode vs bf16 mode (both f16 P)")):
        s1, d1, l1, g1 = out[name]
        print(f"C5 scene ({s0.numel()} voxels), {what}:")
        print(f"  sigma rel-L2 {rel_l2(s1, s0):.3e}   dino rel-L2 {rel_l2(d1, d0):.3e}")
        print(f"  labels equal {float((l0 == l1).double().mean()):.4%}   seg equal {float((g0 == g1).double().mean()):.4%}"
              f"   seg equal on occupied ({int(occ.sum())}) {float((g0[occ] == g1[occ]).double().mean()):.4%}")


if __name__ == "__main__":
    main()
