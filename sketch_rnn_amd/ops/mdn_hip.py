"""Fused MDN loss on the GPU (``csrc/mdn.hip``): one pass writes the
per-row loss terms and dL/dz; backward only rescales the pen / mixture
column groups by the incoming gradients."""
from __future__ import annotations

import ctypes as C
import math

import torch

from ..utils import native

# Row slabs of the head's [dW; db] reduction (csrc/mdn_head.hip mdn_head_dw):
# each workgroup's row loop is latency-bound, so more slabs = more loads in
# flight. Measured on MI355X (vae_large, same box, A/B twice): 16 slabs
# 26.72 / 26.65, 32 slabs 26.59 / 26.62, 64 slabs 26.62 / 26.62 ms/step.
HEAD_DW_SLABS = 32


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


class _MDNLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, target, M, mode, F, mask_pen, log_floor):
        lib = native.require_hip()
        z = z.contiguous().float()
        target = target.contiguous().float()
        N = z.shape[0]
        row_shape = torch.empty(N, device=z.device, dtype=torch.float32)
        row_pen = torch.empty(N, device=z.device, dtype=torch.float32)
        need = ctx.needs_input_grad[0]
        dz = torch.empty_like(z) if need else None
        rc = lib.lib.skr_mdn_loss(z.data_ptr(), z.stride(0), target.data_ptr(), target.stride(0), N, M, mode,
                                  float(F), int(mask_pen), float(log_floor), row_shape.data_ptr(),
                                  row_pen.data_ptr(), dz.data_ptr() if need else None, _stream())
        if rc != 0:
            raise RuntimeError("skr_mdn_loss failed (%d)" % rc)
        ctx.dz = dz
        shape = row_shape.mean()
        pen = row_pen.mean()
        return shape + pen, shape, pen

    @staticmethod
    def backward(ctx, g_total, g_shape, g_pen):
        dz = ctx.dz
        ctx.dz = None
        gs = g_total + g_shape
        gp = g_total + g_pen
        dz[:, :3] *= gp
        dz[:, 3:] *= gs
        return dz, None, None, None, None, None, None


def mdn_loss_hip(z, target, M, mode="magenta", stroke_importance=200.0, is_training=True, clamp=1e-20, eps=1e-6):
    if mode == "reference":
        return _MDNLoss.apply(z, target, M, 0, stroke_importance, 0, math.log(clamp))
    return _MDNLoss.apply(z, target, M, 1, 0.0, 0 if is_training else 1, math.log(eps))


# ---------------------------------------------------------------------------------
# fused head: projection + loss + dz in one kernel (csrc/mdn_head.hip)
# ---------------------------------------------------------------------------------
def head_fused_ok(x: torch.Tensor, W: torch.Tensor, M: int) -> bool:
    """The fused MDN head applies to bf16 HIP training on the GPU with M <= 24
    mixtures, a decoder width that is a multiple of 128 and at least one row
    (an empty batch takes the unfused path, whose reductions handle N = 0)."""
    from . import gemm, use_hip
    return (FUSED_HEAD and x.is_cuda and use_hip(x) and gemm.lp_dtype() == torch.bfloat16 and 1 <= M <= 24
            and x.numel() > 0
            and W.shape[0] % 128 == 0 and W.shape[1] == 3 + 6 * M)


FUSED_HEAD = True   # False: the head GEMM + MDN loss as separate ops (tests)


def _noutp(nout: int) -> int:
    return (nout + 31) // 32 * 32


class _MDNHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, W, b, target, seed, meta, X_lp):
        from ._hipapi import HeadDx, HeadDw, HeadFwd  # noqa: F401 (bound in native)
        from . import gemm
        M, mode, F, mask_pen, log_floor, keep, stream = meta
        ctx.set_materialize_grads(False)   # the shape / pen terms are usually unused: None grads
        lib = native.require_hip()
        Hd, NOUT = W.shape
        NOUTP = _noutp(NOUT)
        X2 = X.reshape(-1, Hd).contiguous().float()
        N = X2.shape[0]
        dev = X2.device
        XL = _lp_rows(X_lp, X, Hd) if keep >= 1.0 else None
        # [dW; db] on the long-K weight-gradient GEMM (csrc/wgrad_gemm.hip)
        # when the bf16 rows exist: dz then carries 256 columns per row (the
        # kernel's N tile; columns >= NOUTP are never read back)
        wg = XL is not None and gemm.WGRAD_HIP and Hd % 256 == 0 and NOUTP <= 256
        tgt = target.reshape(-1, 5).contiguous().float()
        Wt = torch.zeros(NOUTP, Hd, device=dev, dtype=torch.bfloat16)
        Wt[:NOUT] = W.t()
        bias = b.contiguous().float()
        nb = lib.lib.skr_mdn_head_nblocks(N)
        part = torch.empty(2 * nb, device=dev, dtype=torch.float32)
        out3 = torch.empty(3, device=dev, dtype=torch.float32)
        need = any(ctx.needs_input_grad[:3])
        dz = torch.empty(N, 256 if wg else NOUTP, device=dev, dtype=torch.bfloat16) if need else None
        from .recurrent import _seed_tensor
        sd = _seed_tensor(seed, dev)
        a = HeadFwd()
        if XL is not None:   # the decoder's bf16 h rows: half the bytes, the same bf16 operands
            a.X, a.ldx, a.N, a.Hd, a.x_bf16 = XL.data_ptr(), XL.stride(0), N, Hd, 1
        else:
            a.X, a.ldx, a.N, a.Hd, a.x_bf16 = X2.data_ptr(), X2.stride(0), N, Hd, 0
        a.ldz = dz.stride(0) if dz is not None else NOUTP
        a.Wt, a.bias, a.tgt, a.ldt = Wt.data_ptr(), bias.data_ptr(), tgt.data_ptr(), tgt.stride(0)
        a.M, a.NOUT, a.NOUTP, a.mode, a.mask_pen = M, NOUT, NOUTP, mode, mask_pen
        a.F, a.log_floor, a.inv_n = float(F), float(log_floor), 1.0 / max(N, 1)
        a.keep, a.seed, a.stream = float(keep), sd.data_ptr(), int(stream)
        a.dz, a.part = (dz.data_ptr() if dz is not None else None), part.data_ptr()
        rc = lib.lib.skr_mdn_head_fwd(C.byref(a), out3.data_ptr(), _stream())
        if rc != 0:
            raise RuntimeError("skr_mdn_head_fwd failed (%d)" % rc)
        ctx.save_for_backward(X2, W)
        ctx.dz, ctx.sd, ctx.meta, ctx.xshape, ctx.keep_alive = dz, sd, meta, X.shape, (Wt, tgt, bias, part)
        ctx.XL = XL if wg else None
        return out3[0], out3[1], out3[2]

    @staticmethod
    def backward(ctx, g_total, g_shape, g_pen):
        from ._hipapi import HeadDw, HeadDx
        from . import gemm
        X2, W = ctx.saved_tensors
        M, mode, F, mask_pen, log_floor, keep, stream = ctx.meta
        lib = native.require_hip()
        dz, sd, XL = ctx.dz, ctx.sd, ctx.XL
        ctx.dz = ctx.keep_alive = ctx.XL = None
        N, Hd = X2.shape
        NOUT = W.shape[1]
        NOUTP = _noutp(NOUT)
        dev = X2.device
        if g_pen is None and g_shape is None and g_total is not None:   # the training loss: one copy
            scale = g_total.float().reshape(1).expand(2).contiguous()
        else:
            z0 = torch.zeros((), device=dev)
            gt = g_total if g_total is not None else z0
            scale = torch.stack([gt + (g_pen if g_pen is not None else z0),
                                 gt + (g_shape if g_shape is not None else z0)]).float().contiguous()
        dX = dW = db = None
        if ctx.needs_input_grad[0]:
            Wb = torch.zeros(Hd, NOUTP, device=dev, dtype=torch.bfloat16)
            Wb[:, :NOUT] = W
            dX = torch.empty(N, Hd, device=dev, dtype=torch.float32)
            a = HeadDx()
            a.dz, a.N, a.NOUTP, a.Wb, a.Hd = dz.data_ptr(), N, NOUTP, Wb.data_ptr(), Hd
            a.scale, a.keep, a.seed, a.stream = scale.data_ptr(), float(keep), sd.data_ptr(), int(stream)
            a.dX, a.lddx, a.ldz = dX.data_ptr(), Hd, dz.stride(0)
            rc = lib.lib.skr_mdn_head_dx(C.byref(a), _stream())
            if rc != 0:
                raise RuntimeError("skr_mdn_head_dx failed (%d)" % rc)
            dX = dX.view(ctx.xshape)
        if (ctx.needs_input_grad[1] or ctx.needs_input_grad[2]) and XL is not None:
            # [dW | .] = X^T dz and db = colsum(dz) in one long-K GEMM pass, then
            # the per-column-group upstream scale (pen / mixture columns)
            full, cs = gemm.wgrad(XL, dz, colsum=True)
            svec = torch.cat([scale[0:1].expand(3), scale[1:2].expand(NOUT - 3)])
            dW = full[:, :NOUT] * svec
            db = cs[:NOUT] * svec
        elif ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            S = HEAD_DW_SLABS   # row slabs: workgroups = (Hd/64 + 1) * S, each a latency-bound row loop
            rows_per = (-(-N // S) + 31) // 32 * 32
            S = -(-N // rows_per)
            slab = torch.empty(S, Hd + 64, NOUTP, device=dev, dtype=torch.float32)
            dW = torch.empty(Hd, NOUT, device=dev, dtype=torch.float32)
            db = torch.empty(NOUT, device=dev, dtype=torch.float32)
            a = HeadDw()
            a.X, a.ldx, a.N, a.Hd = X2.data_ptr(), X2.stride(0), N, Hd
            a.dz, a.NOUTP = dz.data_ptr(), NOUTP
            a.scale, a.keep, a.seed, a.stream = scale.data_ptr(), float(keep), sd.data_ptr(), int(stream)
            a.slab, a.rows_per, a.ldz, a.x_bf16 = slab.data_ptr(), rows_per, dz.stride(0), 0
            rc = lib.lib.skr_mdn_head_dw(C.byref(a), S, NOUT, dW.data_ptr(), db.data_ptr(), _stream())
            if rc != 0:
                raise RuntimeError("skr_mdn_head_dw failed (%d)" % rc)
        return dX, dW, db, None, None, None, None


def _lp_rows(X_lp, X, Hd):
    """``X_lp`` (a bf16 copy of ``X`` the producer already holds, e.g. the
    decoder's saved bf16 h rows) as ``[N, Hd]`` rows the head kernels can
    read directly: unit column stride, 16-byte aligned rows; else None."""
    if (X_lp is None or X_lp.dtype != torch.bfloat16 or X_lp.shape[-1] != Hd or X_lp.numel() != X.numel()
            or not X_lp.is_cuda):
        return None
    try:
        XL = X_lp.view(-1, Hd)
    except RuntimeError:
        return None
    if XL.stride(1) != 1 or XL.stride(0) % 8 or XL.data_ptr() % 16:
        return None
    return XL


def mdn_head_loss_hip(x, W, b, target, M, mode="magenta", stroke_importance=200.0, is_training=True,
                      clamp=1e-20, eps=1e-6, drop_keep=1.0, drop_seed=0, drop_stream=0, x_lp=None):
    """``(total, shape, pen)`` of the MDN loss of ``z = drop(x) @ W + b`` with
    the projection, loss and dL/dz fused (``x [..., Hd]`` fp32). ``x_lp``:
    an optional bf16 copy of ``x`` (same shape; any strides with unit column
    stride), read instead of ``x`` when there is no dropout -- the kernels
    round ``x`` to bf16 anyway, so the result is the same."""
    if mode == "reference":
        meta = (M, 0, float(stroke_importance), 0, math.log(clamp), float(drop_keep), int(drop_stream))
    else:
        meta = (M, 1, 0.0, 0 if is_training else 1, math.log(eps), float(drop_keep), int(drop_stream))
    return _MDNHead.apply(x, W, b, target, drop_seed, meta, x_lp)
