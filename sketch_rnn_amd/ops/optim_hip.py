"""Fused clip + Adam over the flat parameter arena (``csrc/optim.hip``)."""
from __future__ import annotations

import torch

from ..utils import native

_CLIP = {None: 0, "none": 0, "global_norm": 1, "value": 2}


def flat_adam_step(opt) -> None:
    lib = native.require_hip()
    if not hasattr(opt, "_partial"):
        opt._partial = torch.zeros(2048, device=opt.flat.device, dtype=torch.float64)
    rc = lib.lib.skr_adam_step(opt.flat.data_ptr(), opt.grad.data_ptr(), opt.m.data_ptr(), opt.v.data_ptr(),
                               opt.scalars.data_ptr(), opt._partial.data_ptr(), opt.numel, float(opt.b1),
                               float(opt.b2), float(opt.eps), _CLIP[opt.clip_mode], float(opt.clip),
                               1 if opt.nonfinite == "skip" else 0, torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError("skr_adam_step failed (%d)" % rc)


def global_norm(flat_grad: torch.Tensor) -> torch.Tensor:
    lib = native.require_hip()
    partial = torch.zeros(2048, device=flat_grad.device, dtype=torch.float64)
    scal = torch.zeros(8, device=flat_grad.device, dtype=torch.float32)
    rc = lib.lib.skr_global_norm(flat_grad.data_ptr(), flat_grad.numel(), partial.data_ptr(), scal.data_ptr(),
                                 torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError("skr_global_norm failed (%d)" % rc)
    return scal[2]
