"""Where the 16-bit render's depth error comes from (CPU emulation, diagnostic only).

Replays the projected-grid render (P = W_in[:, :C] G + b_in per pixel, bilinear
blend of P taps, + W_code . code, ReLU, sigma = W_sigma . relu(h) + b, softplus, the
reference's compositing) in fp32 on the CPU, rounding a chosen set of operands to bf16 or
fp16 exactly where the render kernels round them, and reports the maximum composited-depth
error against the reference's own renders (tests/golden: render_k32_cap0, render_k64_cap1,
and the 192x640x64 offset-pose frame, every 61st ray).

Operands: P (the projected grid), w (the bilinear tap weights, the blend MFMA's B operand),
code (the positional-code fragments), Wc (the code columns of W_in), X (relu(h), the sigma
MFMA's B operand), Ws (W_sigma, its A operand).

Usage: python tools/lowp_depth_emul.py  (about a minute on 8 CPU threads)
"""
import math
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import render_oracle as O  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")
I = lambda t: t  # noqa: E731
BF = lambda t: t.to(torch.bfloat16).float()  # noqa: E731
HF = lambda t: t.to(torch.float16).float()  # noqa: E731


def scene_small(name):
    d = np.load(os.path.join(GOLD, name + ".npz"))
    T = lambda k: torch.from_numpy(np.asarray(d[k]))  # noqa: E731
    w2c = torch.inverse(T("poses"))[:, 0]
    return dict(rays=T("rays")[0], u=T("u"), grid=T("grid"), W_in=T("W_in"), b_in=T("b_in"),
                W_out=T("W_out"), b_out=T("b_out"), w2c=w2c, Kf=T("Ks")[:, 0],
                cap=bool(d["hard_cap"]), ref=T("depth")[0])


def scene_full_offset():
    """make_golden.fx_render_full_offset's scene (seed 61, kaiming ResnetFC at seed 2,
    biases at seed 102), restricted to the fixture's subsampled rays."""
    from _fullscene import KITTI_K
    from scenedino_amd.models.prediction_heads import ResnetFC
    d = np.load(os.path.join(GOLD, "render_full_offset.npz"))
    g = torch.Generator().manual_seed(int(d["scene_seed"]))
    torch.rand(1, 1, 3, 192, 640, generator=g)
    grid = torch.randn(1, 256, 192, 640, generator=g)
    torch.manual_seed(2)
    head = ResnetFC(d_in=256 + 39, d_out=65, n_blocks=0, d_hidden=128)
    gb = torch.Generator().manual_seed(102)
    with torch.no_grad():
        head.lin_in.bias.copy_(0.1 * torch.randn(128, generator=gb))
        head.lin_out.bias.copy_(0.1 * torch.randn(65, generator=gb))
    Kn = torch.tensor(KITTI_K).view(1, 3, 3)
    rays = O.gen_rays(torch.as_tensor(d["render_pose"]).view(1, 4, 4), Kn, 192, 640)
    u = torch.rand(rays.shape[0], 64, generator=torch.Generator().manual_seed(int(d["u_seed"])))
    idx = torch.as_tensor(d["idx"])
    return dict(rays=rays[idx], u=u[idx], grid=grid, W_in=head.lin_in.weight.detach(),
                b_in=head.lin_in.bias.detach(), W_out=head.lin_out.weight.detach(),
                b_out=head.lin_out.bias.detach(), w2c=torch.eye(4).view(1, 4, 4), Kf=Kn,
                cap=False, ref=torch.as_tensor(d["depth"]))


def scene_offset_fixture(name):
    """make_golden.fx_render_full_offset_k32 / fx_render_c4_offset (configs[0] / configs[3]):
    the seed-61 scene, restricted to the fixture's rays (the head from the fixture if it
    holds one)."""
    from _fullscene import KITTI_K, scene_arrays
    d = np.load(os.path.join(GOLD, name + ".npz"))
    K = int(d["K"])
    D = int(d["D"]) if "D" in d else 64
    _, grid, (W_in, b_in, W_out, b_out) = scene_arrays(
        int(d["scene_seed"]), D=D, weights=d if "W_in" in d else None)
    Kn = torch.tensor(KITTI_K).view(1, 3, 3)
    rays = O.gen_rays(torch.as_tensor(d["render_pose"]).view(1, 4, 4), Kn, 192, 640)
    u = torch.rand(rays.shape[0], K, generator=torch.Generator().manual_seed(int(d["u_seed"])))
    idx = torch.as_tensor(d["idx"])
    return dict(rays=rays[idx], u=u[idx], grid=grid, W_in=W_in, b_in=b_in, W_out=W_out,
                b_out=b_out, w2c=torch.eye(4).view(1, 4, 4), Kf=Kn, cap=False,
                ref=torch.as_tensor(d["depth"]))


class Emu:
    def __init__(self, s):
        self.s = s
        rays, u, grid = s["rays"], s["u"], s["grid"]
        K = u.shape[1]
        C = grid.shape[1]
        self.z = O.sample_z(rays, K, u)
        pts = (rays[:, None, :3] + self.z.unsqueeze(2) * rays[:, None, 3:6]).reshape(1, -1, 3)
        xy, zz = O._project(pts, s["w2c"].unsqueeze(1), s["Kf"].unsqueeze(1))
        xy = xy.clamp(-2, 2)
        self.code = O.positional_code(xy[:, 0], zz[:, 0])[0]
        Hf, Wf = grid.shape[2:]
        x, y = xy[0, 0, :, 0], xy[0, 0, :, 1]
        ix = (((x + 1) * Wf - 1) / 2).clamp(0, Wf - 1)
        iy = (((y + 1) * Hf - 1) / 2).clamp(0, Hf - 1)
        x0, y0 = ix.floor().long(), iy.floor().long()
        x1, y1 = (x0 + 1).clamp(max=Wf - 1), (y0 + 1).clamp(max=Hf - 1)
        wx, wy = ix - x0, iy - y0
        self.ws = [(1 - wx) * (1 - wy), wx * (1 - wy), (1 - wx) * wy, wx * wy]
        # only the texels the samples touch are projected
        flat = torch.stack([y0 * Wf + x0, y0 * Wf + x1, y1 * Wf + x0, y1 * Wf + x1])
        uniq, inv = torch.unique(flat, return_inverse=True)
        self.G = grid[0].reshape(C, -1)[:, uniq]
        self.P = (s["W_in"][:, :C] @ self.G + s["b_in"].view(-1, 1)).t()  # (texels, 128)
        self._Pq = {}
        self.inv = inv
        self.K, self.C = K, C

    def depth(self, rP=I, rw=I, rcode=I, rWc=I, rX=I, rWs=I, rG=I):
        """rG: rounding of the projection's operands (grid G and W_in[:, :C], k_project's
        MFMA inputs) before P itself is rounded by rP."""
        s = self.s
        if rG is I:
            Pq = rP(self.P)
        else:
            if rG not in self._Pq:
                C = self.C
                self._Pq[rG] = (rG(s["W_in"][:, :C]).double() @ rG(self.G).double()
                                + s["b_in"].double().view(-1, 1)).float().t()
            Pq = rP(self._Pq[rG])
        h = sum(rw(w).unsqueeze(-1) * Pq[self.inv[q]] for q, w in enumerate(self.ws))
        h = h + rcode(self.code) @ rWc(s["W_in"][:, self.C:]).t()
        X = rX(torch.relu(h))
        sig = F.softplus(X @ rWs(s["W_out"][0]) + s["b_out"][0])
        R = self.z.shape[0]
        c = O.composite(self.z, sig.view(R, self.K), torch.zeros(R, self.K, 1),
                        torch.zeros(R, self.K, 3), s["cap"])
        return c["depth"]


SCHEMES = [
    ("all fp32 (emulator check)", {}),
    ("all bf16 (the bf16 kernels)", dict(rP=BF, rw=BF, rcode=BF, rWc=BF, rX=BF, rWs=BF)),
    ("bf16, sigma column exact (X, Ws in f32)", dict(rP=BF, rw=BF, rcode=BF, rWc=BF)),
    ("bf16, sigma column fp16", dict(rP=BF, rw=BF, rcode=BF, rWc=BF, rX=HF, rWs=HF)),
    ("bf16 but P, w fp16", dict(rP=HF, rw=HF, rcode=BF, rWc=BF, rX=BF, rWs=BF)),
    ("P, w, X, Ws fp16; code, Wc bf16", dict(rP=HF, rw=HF, rcode=BF, rWc=BF, rX=HF, rWs=HF)),
    ("all fp16 (the fp16 kernels)", dict(rP=HF, rw=HF, rcode=HF, rWc=HF, rX=HF, rWs=HF)),
    ("r5 bf16 mode A: G,Wg,P,w,X,Ws f16; code,Wc bf16",
     dict(rG=HF, rP=HF, rw=HF, rcode=BF, rWc=BF, rX=HF, rWs=HF)),
    ("r5 bf16 mode B: all f16 but the DINO head",
     dict(rG=HF, rP=HF, rw=HF, rcode=HF, rWc=HF, rX=HF, rWs=HF)),
    ("only P bf16", dict(rP=BF)),
    ("only w bf16", dict(rw=BF)),
    ("only code + Wc bf16", dict(rcode=BF, rWc=BF)),
    ("only X + Ws bf16", dict(rX=BF, rWs=BF)),
    ("only P f16", dict(rP=HF)),
    ("only w f16", dict(rw=HF)),
    ("only code + Wc f16", dict(rcode=HF, rWc=HF)),
    ("only X + Ws f16", dict(rX=HF, rWs=HF)),
    ("only G, Wg f16 (projection operands)", dict(rG=HF)),
    ("all f16 but X, Ws (sigma column hi+lo)", dict(rG=HF, rP=HF, rw=HF, rcode=HF, rWc=HF)),
    ("all f16 but P (P hi+lo)", dict(rG=HF, rw=HF, rcode=HF, rWc=HF, rX=HF, rWs=HF)),
]


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    scenes = [("render_k32_cap0", scene_small("render_k32_cap0")),
              ("render_k64_cap1", scene_small("render_k64_cap1")),
              ("render_full_offset", scene_full_offset())]
    if os.environ.get("EMUL_ONLY_C03") == "1":
        scenes = []
    scenes += [("full_offset_k32", scene_offset_fixture("render_full_offset_k32")),
               ("c4_offset_k128", scene_offset_fixture("render_c4_offset"))]
    emus = [(n, Emu(s), s["ref"]) for n, s in scenes]
    print("max |depth - reference| (m) of the emulated render; contract (SURVEY §8(c)): 1e-2 m")
    print(f"{'scheme':44s}" + "".join(f"{n:>22s}" for n, _, _ in emus))
    for name, kw in SCHEMES:
        errs = [float((e.depth(**kw) - ref).abs().max()) for _, e, ref in emus]
        print(f"{name:44s}" + "".join(f"{x:22.3e}" for x in errs))


if __name__ == "__main__":
    main()
