"""Differentiable (training) field path: autograd Functions over the sdhip_train.hip kernels.

The inference path (sd_render_proj / sd_render_fused) fuses everything into one kernel and
keeps no per-sample state; training (``train.py`` renders through the field and
back-propagates into the feature grid and the ResnetFC, base_trainer.py:223,251) runs

  FieldGather  (sd_field_gather / sd_field_gather_bwd)   a8-a10, a12, a15  -> X = [feat | code]
  ResnetFC     torch.nn.Linear (library GEMMs, autograd)  a13
  softplus     torch                                       a14
  Composite    (sd_composite / sd_composite_bwd)           a16

so that ``loss.backward()`` reaches ``grid_f_features`` (and through it whatever encoder
produced the grid) and the head parameters, as in the reference's
``BTSNet.forward`` -> ``NeRFRenderer.composite`` (bts.py:476-595, nerf.py:343-405).
No CPU fallback: every op here is a HIP kernel or a torch GPU op.
"""
from __future__ import annotations

import os

import torch

from . import _lib

# bench hook: an object with start(name) / stop(name) (HIP events on the launch stream)
kernel_timer = None


def _timed(name, fn):
    t = kernel_timer
    if t is not None:
        t.start(name)
    r = fn()
    if t is not None:
        t.stop(name)
    return r


class GridNHWC(torch.autograd.Function):
    """(B, C, Hf, Wf) f32 grid -> NHWC f32 for the gather.  A channels-last grid (the
    native encoder's output) is used in place and its gradient handed back channels-last:
    no copy either way.  An NCHW grid is transposed by sd_pack_grid, its gradient back by
    sd_unpack_grid."""

    @staticmethod
    def forward(ctx, grid):
        ctx.cl = _lib.channels_last(grid)
        if ctx.cl:
            return grid.float().permute(0, 2, 3, 1)
        return _lib.pack_grid(grid.float().contiguous(), _lib.SD_F32)

    @staticmethod
    def backward(ctx, g):
        if ctx.cl:
            return g.float().contiguous().permute(0, 3, 1, 2)
        return _lib.unpack_grid(g.float().contiguous())


class GatherAcc:
    """Grid-gradient accumulator shared by the FieldGather calls of one compositing pass
    (the renderer's chunks): every chunk's backward scatters into ONE zeroed NHWC buffer,
    handed to autograd by the first chunk of the backward pass (the others return no
    gradient), instead of one zeroed 4 x 126 MB buffer per chunk summed by autograd.
    Autograd runs the grid's node only after every chunk's backward, so the buffer is
    complete when it is read.  A backward pass is identified by autograd's graph-task id,
    not by counting chunks: chunks outside the loss's graph never run their backward, and
    a retained graph can be walked again; the buffer is released by a callback at the end
    of the pass."""

    def __init__(self):
        self.n = 0        # FieldGather calls recorded in the forward pass
        self.task = None  # graph task the buffer belongs to
        self.buf = None

    def take(self, shape, device):
        """(buffer, first) for the running backward pass."""
        task = torch._C._current_graph_task_id()
        if self.buf is None or self.task != task:
            # (zeroed here, serialised before the scatter: a fill of the 503 MB bench
            # buffer forked to a side stream during the forward slowed the kernels beside
            # it by more than its 63 us -- 0.75 vs 0.69 ms per step, profiles/r5_train)
            self.task, self.buf = task, torch.zeros(shape, device=device)
            torch.autograd.Variable._execution_engine.queue_callback(self._release)
            return self.buf, True
        return self.buf, False

    def _release(self):
        self.task, self.buf = None, None


class FieldGather(torch.autograd.Function):
    """X = [grid_sample(grid, project(xyz)) | positional_code(xyz) | 1], differentiable in
    the grid (bts.py:271-328).  grid_nhwc (B, Hf, Wf, C) f32; xyz (B, P, 3) (no gradient:
    the reference's sample points come from rays and depths without grad)."""

    @staticmethod
    def forward(ctx, grid_nhwc, xyz, cam_f, img, cam_c, colors, acc=None):
        # under torch.autocast the rows are written in the autocast dtype the MLP GEMMs
        # consume (no separate cast pass over the (N, C + 40) matrix)
        dt = (torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda")
              else torch.float32)
        x, invf, rgb, inv = _timed("gather", lambda: _lib.field_gather(
            xyz, grid_nhwc, cam_f, img, cam_c, colors, dtype=dt))
        ctx.save_for_backward(xyz, cam_f)
        ctx.grid_shape = tuple(grid_nhwc.shape)
        ctx.acc = acc if acc is not None else GatherAcc()
        ctx.acc.n += 1
        outs = [t for t in (invf, rgb, inv) if t is not None]
        ctx.mark_non_differentiable(*outs)
        return x, invf, rgb, inv

    @staticmethod
    def backward(ctx, gx, *_):
        xyz, cam_f = ctx.saved_tensors
        if not ctx.needs_input_grad[0] or gx is None:
            return None, None, None, None, None, None, None
        B, Hf, Wf, C = ctx.grid_shape
        buf, first = ctx.acc.take((B, Hf, Wf, C), xyz.device)
        gx = gx.float().contiguous()  # f32 rows for the scatter (see _lib.field_gather_bwd)
        _timed("gather_bwd", lambda: _lib.field_gather_bwd(xyz, gx, cam_f, Hf, Wf, C, dgrid=buf))
        return (buf if first else None), None, None, None, None, None, None


def _wgrad(a, b):
    """a^T b for tall a (N, m), b (N, n) with small m, n (weight gradients over N = 65 536
    points): as a batched GEMM over S slices of N + a sum, so the chip gets S times the
    workgroups of a single (m x n) output (a plain GEMM launches ~15 tiles here)."""
    N = a.shape[0]
    S = next((s for s in (32, 16, 8, 4, 2) if N % s == 0 and N // s >= 256), 1)
    if S == 1:
        return (a.t() @ b).float()
    part = torch.bmm(a.view(S, N // S, -1).transpose(1, 2), b.view(S, N // S, -1))
    return part.float().sum(0)


class FieldMLP(torch.autograd.Function):
    """ResnetFC with n_blocks = 0 (resnetfc.py:135-203): out = W_o relu(W_i x + b_i) + b_o
    on the gather rows x_aug = [x | 1] (N, d_in + 1).  The biases ride in the GEMMs:
    W2 = [[W_i, b_i], [0, 1]] (129 x (d_in+1)) gives h_aug = relu(x_aug W2^T) = [h | 1] and
    Wo = [W_o, b_o] gives out = h_aug Wo^T, so the backward is three GEMMs whose extra
    column / row are the bias gradients -- no column reductions (torch's are the slowest
    op of the step at 65 536-point chunks)."""

    @staticmethod
    def forward(ctx, x_aug, w_in, b_in, w_out, b_out):
        dh, d_in = w_in.shape
        if x_aug.shape[1] != d_in + 1:
            raise ValueError(f"FieldMLP: x_aug has {x_aug.shape[1]} columns, expected {d_in + 1}")
        # torch.autocast (the reference trains with_amp: nn.Linear in fp16): the GEMMs run
        # in the autocast dtype, parameter gradients come back in the parameters' dtype
        dt = (torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda")
              else w_in.dtype)
        W2 = torch.zeros(dh + 1, d_in + 1, device=w_in.device, dtype=dt)
        W2[:dh, :d_in] = w_in
        W2[:dh, d_in] = b_in
        W2[dh, d_in] = 1.0
        Wo = torch.cat((w_out, b_out[:, None]), 1).to(dt)
        xa = x_aug.to(dt)
        with torch.autocast("cuda", enabled=False):
            h = torch.relu(xa @ W2.t())
            out = h @ Wo.t()
        ctx.save_for_backward(xa, h, W2, Wo)
        ctx.dtypes = (x_aug.dtype, w_in.dtype)
        return out

    @staticmethod
    def backward(ctx, g):
        x_aug, h, W2, Wo = ctx.saved_tensors
        xdt, pdt = ctx.dtypes
        g = g.to(h.dtype).contiguous()
        dh_, d_in = W2.shape[0] - 1, W2.shape[1] - 1
        dWo = _wgrad(g, h).to(pdt)
        dh = (g @ Wo) * (h > 0)
        dW2 = _wgrad(dh, x_aug).to(pdt)
        dx = (dh @ W2).to(xdt) if ctx.needs_input_grad[0] else None  # xdt: the rows' dtype
        return (dx, dW2[:dh_, :d_in].contiguous(), dW2[:dh_, d_in].contiguous(),
                dWo[:, :dh_].contiguous(), dWo[:, dh_].contiguous())


def _packed_train(w_in, b_in, w_out, b_out, dtype, C):
    """Fragments of the current weights, packed on every call (one gather through a cached
    index, csrc/sdhip_mlp.hip's operand order).  Not cached by tensor version: torch's fused
    Adam (the bench's optimizer, capturable inside a HIP graph) updates parameters in place
    without bumping their version counter, so a version-keyed cache served the previous
    step's weights (found by tests/test_train_graph.py)."""
    from .mlp_pack import PackedTrainMLP
    return PackedTrainMLP(w_in, b_in, w_out, b_out, dtype, C)


class FieldMLPFused(torch.autograd.Function):
    """The training MLP under autocast as two fused kernels (csrc/sdhip_mlp.hip):
    forward sd_mlp_train_fwd (layer 1 + ReLU + layer 2 + softplus: returns sigma (N) and
    dino (N, D) f32), backward sd_mlp_train_bwd (dX for the gather's scatter, dH and dY
    rows) + the two weight-gradient GEMMs dW1 = dH^T X, dW_o = dY^T [H | 1] (biases from
    the ones columns).  x_aug (N, d_in + 1) f16 / bf16 rows of sd_field_gather."""

    @staticmethod
    def forward(ctx, x_aug, w_in, b_in, w_out, b_out, C):
        """C: the feature columns of x_aug (the grid's channels; the rest of d_in is the
        positional code)."""
        N, ldx = x_aug.shape
        dh, d_in = w_in.shape
        D = w_out.shape[0] - 1
        dt = _lib.SD_OF_TORCH[x_aug.dtype]
        if not 0 < C < d_in or ldx < d_in + 1:
            raise ValueError(f"FieldMLPFused: {C} feature columns do not fit rows of width "
                             f"{ldx} for a {d_in}-input layer")
        p = _packed_train(w_in, b_in, w_out, b_out, dt, C)
        x_aug = x_aug.contiguous()
        dev = x_aug.device
        h = torch.empty(N, 136, device=dev, dtype=x_aug.dtype)
        sigma = torch.empty(N, device=dev)
        dino = torch.empty(N, D, device=dev)
        a = _lib.SdMlpTrainArgs(x=x_aug.data_ptr(), N=N, ldx=ldx, kx=d_in + 1, dtype=dt, D=D, C=C,
                                w1f=p.w1f.data_ptr(), w2f=p.w2f.data_ptr(),
                                b_out=p.b_out.data_ptr(), h=h.data_ptr(), sigma=sigma.data_ptr(),
                                dino=dino.data_ptr())
        _timed("mlp", lambda: _lib.mlp_train_fwd(a, x_aug))
        ctx.save_for_backward(x_aug, h, sigma)
        ctx.p, ctx.meta = p, (N, ldx, d_in, D, C, dt, w_in.dtype)
        return sigma, dino

    @staticmethod
    def backward(ctx, g_sigma, g_dino):
        dx, *rest = FieldMLPFused.grads(ctx, g_sigma, g_dino, full_rows=True)
        return (dx if ctx.needs_input_grad[0] else None, *rest, None)

    @staticmethod
    def grads(ctx, g_sigma, g_dino, full_rows=False, dx16=False, scatter=None, no_dx=False):
        """(dX, dW_in, db_in, dW_out, db_out) of the saved forward; dX rows are the C
        feature columns, or (full_rows) as wide as x with zero code / ones columns; f32, or
        (dx16) in x's 16-bit dtype -- the dtype the reference's autocast Linear backward
        hands to grid_sample's backward.  ``scatter = (xyz (B, P, 3), cam_f, Hf, Wf, dgrid)``:
        the grid_sample backward fused into the kernel -- dX (in x's dtype) goes straight
        into the NHWC f32 grid gradient dgrid, and dX is returned as None.  ``no_dx``: no
        input gradient wanted -- the kernel skips the dX product and dX is None."""
        x_aug, h, sigma = ctx.saved_tensors
        p = ctx.p
        N, ldx, d_in, D, C, dt, pdt = ctx.meta
        dev = x_aug.device
        g_sigma = (g_sigma if g_sigma is not None else torch.zeros(N, device=dev)).float().contiguous()
        g_dino = (g_dino if g_dino is not None else torch.zeros(N, D, device=dev)).float().contiguous()
        dy = torch.empty(N, 72, device=dev, dtype=x_aug.dtype)
        dh = torch.empty(N, 128, device=dev, dtype=x_aug.dtype)
        a = _lib.SdMlpTrainArgs(x=x_aug.data_ptr(), N=N, ldx=ldx, kx=d_in + 1, dtype=dt, D=D, C=C,
                                h=h.data_ptr(), sigma=sigma.data_ptr(), d_sigma=g_sigma.data_ptr(),
                                d_dino=g_dino.data_ptr(), wtf=p.wtf.data_ptr(),
                                wxf=p.wxf.data_ptr(), dy=dy.data_ptr(), dh=dh.data_ptr())
        if scatter is not None:
            xyz, cam_f, Hf, Wf, dgrid = scatter
            xyz = xyz.contiguous()
            assert xyz.shape[0] * xyz.shape[1] == N and dgrid.dtype == torch.float32 and \
                dgrid.is_contiguous() and dgrid.shape == (xyz.shape[0], Hf, Wf, C)
            dx = None
            a.dx_dtype, a.lddx = dt, C
            a.xyz, a.cam_f, a.dgrid = xyz.data_ptr(), cam_f.data_ptr(), dgrid.data_ptr()
            a.P, a.Hf, a.Wf = xyz.shape[1], Hf, Wf
        elif no_dx:
            dx = None
        else:
            dx = torch.empty(N, ldx if full_rows else C, device=dev,
                             dtype=x_aug.dtype if dx16 else torch.float32)
            a.lddx, a.dx_dtype = dx.shape[1], dt if dx16 else _lib.SD_F32
            a.dx = dx.data_ptr()
        _timed("mlp_bwd", lambda: _lib.mlp_train_bwd(a, x_aug))
        # dW1 = dH^T X ([dW_in | db_in]) and dW_o = dY^T [H | 1] in one pass over the rows,
        # written in the parameter layout
        grads = _lib.mlp_train_wgrad(x_aug, dh, dy, h, d_in + 1, D)
        return (dx,) + tuple(t if t.dtype == pdt else t.to(pdt) for t in grads)


# 16-bit dX rows from the fused MLP backward into the gather's scatter (the autocast
# gradient dtype; halves the dX bytes): measured slower overall -- k_mlp_bwd 125 -> 103 us
# but k_field_gather_bwd 140 -> 223 us on 2-byte lane loads -- so f32 rows when unfused
DX16 = False
# the grid_sample backward fused into k_mlp_bwd (ml_scatter): no dX rows in HBM at all.
# SCENEDINO_AMD_FUSED_SCATTER=0 restores dX rows + k_field_gather_bwd (A/B diagnostics)
FUSED_SCATTER = os.environ.get("SCENEDINO_AMD_FUSED_SCATTER", "1") != "0"


class FieldGatherMLP(torch.autograd.Function):
    """FieldGather -> FieldMLPFused as ONE autograd node (training under autocast): the
    backward hands the MLP's f32 dX rows straight to the gather's scatter -- autograd would
    otherwise cast the gradient of the 16-bit rows to their dtype and back (two passes
    over N x (C + 40)).  learn_empty (bts.py:311-319): out-of-frustum rows take the empty
    feature; its gradient is the sum of their dX rows, which the scatter then skips."""

    @staticmethod
    def forward(ctx, grid_nhwc, xyz, cam_f, img, cam_c, colors, acc, empty, w_in, b_in, w_out,
                b_out):
        dt = torch.get_autocast_dtype("cuda")
        x, invf, rgb, inv = _timed("gather", lambda: _lib.field_gather(
            xyz, grid_nhwc, cam_f, img, cam_c, colors, dtype=dt))
        B, P, ldx = x.shape
        N = B * P
        x = x.view(N, ldx)
        C = grid_nhwc.shape[-1]
        if empty is not None:
            m = invf.reshape(N, 1)
            x[:, :C] = torch.where(m, empty.to(dt).view(1, C), x[:, :C])
        sigma, dino = FieldMLPFused.forward(ctx, x, w_in, b_in, w_out, b_out, C)
        ctx.xyz, ctx.cam_f, ctx.grid_shape = xyz, cam_f, tuple(grid_nhwc.shape)
        ctx.acc = acc if acc is not None else GatherAcc()
        ctx.acc.n += 1
        ctx.invf = invf if empty is not None else None
        ctx.empty_dtype = empty.dtype if empty is not None else None
        outs = [t for t in (invf, rgb, inv) if t is not None]
        ctx.mark_non_differentiable(*outs)
        return sigma.view(B, P), dino.view(B, P, -1), invf, rgb, inv

    @staticmethod
    def backward(ctx, g_sigma, g_dino, *_):
        N = ctx.meta[0]
        gs = g_sigma.reshape(N) if g_sigma is not None else None
        gd = g_dino.reshape(N, -1) if g_dino is not None else None
        B, Hf, Wf, C = ctx.grid_shape
        if FUSED_SCATTER and ctx.invf is None:  # (learn_empty rows need their dX: unfused)
            d_grid = None
            if ctx.needs_input_grad[0]:
                buf, first = ctx.acc.take((B, Hf, Wf, C), ctx.xyz.device)
                sc = (ctx.xyz, ctx.cam_f, Hf, Wf, buf)
                _, dw_in, db_in, dw_out, db_out = FieldMLPFused.grads(ctx, gs, gd, scatter=sc)
                d_grid = buf if first else None
            else:  # the grid needs no gradient: weight gradients only (no dX product)
                _, dw_in, db_in, dw_out, db_out = FieldMLPFused.grads(ctx, gs, gd, no_dx=True)
            return (d_grid, None, None, None, None, None, None, None, dw_in, db_in, dw_out,
                    db_out)
        dx, dw_in, db_in, dw_out, db_out = FieldMLPFused.grads(ctx, gs, gd, dx16=DX16)
        d_empty = None
        if ctx.invf is not None:
            m = ctx.invf.reshape(N, 1)
            d_empty = torch.where(m, dx[:, :C], torch.zeros((), device=dx.device)).sum(0)
            dx[:, :C] = torch.where(m, torch.zeros((), device=dx.device), dx[:, :C])
            d_empty = d_empty.to(ctx.empty_dtype)
        d_grid = None
        if ctx.needs_input_grad[0]:
            buf, first = ctx.acc.take((B, Hf, Wf, C), dx.device)
            xyz, cam_f = ctx.xyz, ctx.cam_f
            _timed("gather_bwd", lambda: _lib.field_gather_bwd(xyz, dx, cam_f, Hf, Wf, C,
                                                               dgrid=buf))
            d_grid = buf if first else None
        return (d_grid, None, None, None, None, None, None, d_empty, dw_in, db_in, dw_out,
                db_out)


class Composite(torch.autograd.Function):
    """Alpha compositing (nerf.py:376-405) with the sd_composite_bwd backward.
    z, sigma (R, K); feat (R, K, F) | None; rgb (R, K, Cc) | None.  Returns
    (weights, alphas, depth, feat_out, rgb_out).  z carries no gradient (the reference's
    depths are sampled without grad)."""

    @staticmethod
    def forward(ctx, z, sigma, feat, rgb, hard_alpha_cap):
        z = z.float().contiguous()
        sigma = sigma.float().contiguous()
        feat = feat.float().contiguous() if feat is not None else None
        rgb = rgb.float().contiguous() if rgb is not None else None
        w, a, d, fo, ro = _lib.composite(z, sigma, feat, rgb, hard_alpha_cap)
        ctx.save_for_backward(z, sigma, feat, rgb)
        ctx.hard = bool(hard_alpha_cap)
        return w, a, d, fo, ro

    @staticmethod
    def backward(ctx, g_w, g_a, g_d, g_f, g_r):
        z, sigma, feat, rgb = ctx.saved_tensors
        d_sigma, d_feat, d_rgb = _timed("composite_bwd", lambda: _lib.composite_bwd(
            z, sigma, feat, rgb, ctx.hard, g_d, g_f, g_r, g_w, g_a,
            need_feat=ctx.needs_input_grad[2], need_rgb=ctx.needs_input_grad[3]))
        return (None, d_sigma if ctx.needs_input_grad[1] else None, d_feat, d_rgb, None)


def composite(z, sigma, feat, rgb, hard_alpha_cap):
    """Differentiable when any input requires grad and grad mode is on; otherwise the plain
    sd_composite launch (no saved state)."""
    if torch.is_grad_enabled() and any(t is not None and t.requires_grad
                                       for t in (sigma, feat, rgb)):
        return Composite.apply(z, sigma, feat, rgb, hard_alpha_cap)
    return _lib.composite(z.float().contiguous(), sigma.float().contiguous(),
                          feat.float().contiguous() if feat is not None else None,
                          rgb.float().contiguous() if rgb is not None else None, hard_alpha_cap)


class SalienceDownsample(torch.autograd.Function):
    """PatchSalienceDownsampler.forward_patches (downsampler.py:82-98) on the device:
    sd_salience_fwd / sd_salience_bwd.  x (N, S, C) f32 -> out (N, C), salience (N, S),
    weight map (N, S); gradients reach x, the 1x1 conv (w, b) and patch_weight / bias."""

    @staticmethod
    def forward(ctx, x, w, b, pw, pb, normalize):
        N, S, C = x.shape
        wshape = w.shape
        x = x.float().contiguous()
        w = w.float().reshape(C).contiguous()
        pw_ = pw.float().reshape(S).contiguous()
        pb_ = pb.float().reshape(S).contiguous()
        out = torch.empty(N, C, device=x.device)
        sal = torch.empty(N, S, device=x.device)
        wmap = torch.empty(N, S, device=x.device)
        ynorm = torch.empty(N, device=x.device)
        bias = b.detach().float().reshape(-1).contiguous() if b is not None else None
        a = _lib.SdSalienceArgs(x=x.data_ptr(), w=w.data_ptr(),
                                b=bias.data_ptr() if bias is not None else None, pw=pw_.data_ptr(),
                                pb=pb_.data_ptr(), N=N, S=S, C=C, normalize=int(bool(normalize)),
                                out=out.data_ptr(), sal=sal.data_ptr(), wmap=wmap.data_ptr(),
                                ynorm=ynorm.data_ptr())
        _timed("salience", lambda: _lib.salience_fwd(a, x))
        ctx.save_for_backward(x, w, pw_, pb_, out, sal, wmap, ynorm)
        ctx.normalize, ctx.has_b = bool(normalize), b is not None
        ctx.pshape = (pw.shape, pb.shape, wshape)
        return out, sal, wmap

    @staticmethod
    def backward(ctx, g_out, g_sal, g_wmap):
        x, w, pw_, pb_, out, sal, wmap, ynorm = ctx.saved_tensors
        N, S, C = x.shape
        if g_out is None:
            g_out = torch.zeros_like(out)
        g_out = g_out.float().contiguous()
        g_sal = g_sal.float().contiguous() if g_sal is not None else None
        g_wmap = g_wmap.float().contiguous() if g_wmap is not None else None
        gx = torch.empty_like(x)
        gw = torch.empty(N, C, device=x.device)
        gpw = torch.empty(N, S, device=x.device)
        gpb = torch.empty(N, S, device=x.device)
        gb = torch.empty(N, device=x.device)
        a = _lib.SdSalienceArgs(
            x=x.data_ptr(), w=w.data_ptr(), b=None, pw=pw_.data_ptr(), pb=pb_.data_ptr(),
            N=N, S=S, C=C, normalize=int(ctx.normalize), out=out.data_ptr(), sal=sal.data_ptr(),
            wmap=wmap.data_ptr(), ynorm=ynorm.data_ptr(), g_out=g_out.data_ptr(),
            g_sal=g_sal.data_ptr() if g_sal is not None else None,
            g_wmap=g_wmap.data_ptr() if g_wmap is not None else None,
            gx=gx.data_ptr(), gw_part=gw.data_ptr(), gpw_part=gpw.data_ptr(),
            gpb_part=gpb.data_ptr(), gb_part=gb.data_ptr())
        _timed("salience_bwd", lambda: _lib.salience_bwd(a, x))
        return (gx, gw.sum(0).reshape(ctx.pshape[2]), gb.sum().reshape(1) if ctx.has_b else None,
                gpw.sum(0).reshape(ctx.pshape[0]), gpb.sum(0).reshape(ctx.pshape[1]), None)
