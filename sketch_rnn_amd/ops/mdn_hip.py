"""Fused MDN loss on the GPU (``csrc/mdn.hip``): one pass writes the
per-row loss terms and dL/dz; backward only rescales the pen / mixture
column groups by the incoming gradients."""
from __future__ import annotations

import math

import torch

from ..utils import native


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
