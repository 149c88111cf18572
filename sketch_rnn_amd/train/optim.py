"""Flat-arena Adam with gradient clipping (reference capability R13).

All trainable parameters live as views into ONE contiguous fp32 buffer and
their gradients as views into ONE contiguous fp32 gradient buffer
("arena"). That layout gives:

* a single fused HIP kernel for clip + Adam over every parameter
  (``csrc/optim.hip``) instead of one launch per tensor;
* a single (bucketed) RCCL all-reduce for data parallelism
  (:mod:`sketch_rnn_amd.parallel.dp`);
* graph-capture safety: no allocation in the step; ``lr`` and the Adam
  step count live in a device scalar block that the host updates before
  each replay.

Update rule is TF's ``AdamOptimizer`` (``model.py:183``): ``epsilon`` is
added to ``sqrt(v)`` and the bias corrections are folded into the step
size, ``lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t)``.

Clipping modes:
* ``"global_norm"`` -- ``tf.clip_by_global_norm`` (reference, ``model.py:182``);
* ``"value"`` -- per-element ``clip_by_value`` (sketch-rnn VAE).

Failure detection: the global gradient norm is computed every
step; ``nonfinite="skip"`` drops a step whose gradient norm is NaN/Inf on the
device (no parameter or moment update, ``t`` not advanced) and counts it in
``scalars[5]`` -- no host sync per step. ``"apply"`` keeps TF semantics.
Device scalars: ``[lr, t, grad_norm, clip_scale, skipped_now, skipped_total, grad_scale, -]``.

Data parallelism: the gradient buffer carries a small TAIL
after the arena (:attr:`FlatAdam.tail`, ``TAIL`` floats) that rides in the
last all-reduce bucket -- the step's loss scalars are packed there, so their
cross-rank sum needs no collective of its own -- and the 1/world average is
``grad_scale`` (``scalars[6]``), applied inside the norm and Adam kernels
instead of as a separate pass over the summed arena.
"""
from __future__ import annotations

import math
from typing import Iterable, List, Optional

import torch


class FlatAdam:
    TAIL = 64   # floats after the arena in grad_full (reduced with the last bucket)

    def __init__(self, params: Iterable[torch.nn.Parameter], lr: float = 1e-3, betas=(0.9, 0.999),
                 eps: float = 1e-8, clip_mode: Optional[str] = None, clip: float = 0.0,
                 align: int = 64, nonfinite: str = "skip"):
        self.params: List[torch.nn.Parameter] = [p for p in params if p.requires_grad]
        self.b1, self.b2 = betas
        self.eps = eps
        self.clip_mode = clip_mode
        self.clip = float(clip)
        if nonfinite not in ("skip", "apply"):
            raise ValueError(nonfinite)
        self.nonfinite = nonfinite
        dev = self.params[0].device
        # 256-byte aligned slots per tensor: vector loads never straddle tensors
        self.offsets, off = [], 0
        for p in self.params:
            self.offsets.append(off)
            off += (p.numel() + align - 1) // align * align
        self.numel = off
        self.offset_of = {id(p): o for p, o in zip(self.params, self.offsets)}
        self.flat = torch.zeros(off, device=dev, dtype=torch.float32)
        # gradients + the reduced tail (loss scalars); Adam reads only [:numel]
        self.grad_full = torch.zeros(off + self.TAIL, device=dev, dtype=torch.float32)
        self.grad = self.grad_full[:off]
        self.tail = self.grad_full[off:]
        self.m = torch.zeros(off, device=dev, dtype=torch.float32)
        self.v = torch.zeros(off, device=dev, dtype=torch.float32)
        for p, o in zip(self.params, self.offsets):
            n = p.numel()
            self.flat[o:o + n].copy_(p.detach().reshape(-1))
            p.data = self.flat[o:o + n].view_as(p)
            p.grad = self.grad[o:o + n].view_as(p)
            # the arena slot a backward kernel may write this gradient into
            # directly (ops.gemm.grad_slot): autograd then keeps that tensor as
            # p.grad and gather_grads has nothing to copy for it
            p._grad_slot = p.grad
        # device scalars: [lr, step, grad_norm, clip_scale, skipped_now, skipped_total, grad_scale, -]
        self.scalars = torch.zeros(8, device=dev, dtype=torch.float32)
        self.scalars[6] = 1.0
        self.set_lr(lr)
        self.step_count = 0

    # ---------------------------------------------------------------------------------
    def set_lr(self, lr: float) -> None:
        self.lr = float(lr)
        self.scalars[0].fill_(self.lr)

    def set_grad_scale(self, scale: float) -> None:
        """Factor applied to every gradient element before the norm, clip and
        Adam (data parallel: 1/world over a SUM all-reduce)."""
        self.grad_scale = float(scale)
        self.scalars[6].fill_(self.grad_scale)

    def zero_grad(self, set_to_none: bool = False) -> None:
        """``set_to_none``: unbind ``p.grad`` so autograd hands over the
        gradient tensors it produces instead of adding each into a zeroed
        arena view (one fill + one add launch per parameter); follow the
        backward with :meth:`gather_grads`."""
        if set_to_none:
            for p in self.params:
                p.grad = None
        else:
            self.grad.zero_()

    def gather_grads(self, params=None) -> None:
        """After ``zero_grad(set_to_none=True)`` + backward: copy the
        produced gradients into the arena with one multi-tensor copy, zero
        the slots of parameters that received none, and rebind ``p.grad`` to
        the arena views. Capture-safe (fixed pointer lists). ``params``: only
        these parameters (a backward split into phases gathers per phase)."""
        sel = None if params is None else {id(p) for p in params}
        dst, src = [], []
        for p, o in zip(self.params, self.offsets):
            if sel is not None and id(p) not in sel:
                continue
            view = self.grad[o:o + p.numel()].view_as(p)
            g = p.grad
            if g is None:
                view.zero_()
            elif g.data_ptr() != view.data_ptr():
                dst.append(view)
                src.append(g)
            p.grad = view
        if dst:
            torch._foreach_copy_(dst, src)

    def named_slices(self):
        for p, o in zip(self.params, self.offsets):
            yield p, o, p.numel()

    # ---------------------------------------------------------------------------------
    def step(self) -> None:
        """Clip + Adam. Capture-safe: the step count advances on device."""
        from .. import ops
        if ops.use_hip(self.flat):
            from ..ops import optim_hip
            optim_hip.flat_adam_step(self)
        else:
            self._step_torch()
        self.step_count += 1

    @torch.no_grad()
    def _step_torch(self) -> None:
        sc = self.scalars
        gs = torch.where(sc[6] > 0, sc[6], torch.ones_like(sc[6]))   # no host sync (graph capture)
        g = self.grad * gs
        norm = torch.sqrt((g.double() * g.double()).sum()).float()
        sc[2] = norm
        skip = (~torch.isfinite(norm)) & (self.nonfinite == "skip")
        sc[4] = skip.float()
        sc[5] += skip.float()
        sc[1] += (~skip).float()
        keep = (~skip).float()
        if self.clip_mode == "global_norm":
            scale = self.clip / torch.clamp(norm, min=self.clip)
            sc[3] = scale
            g = g * torch.where(skip, torch.zeros_like(scale), scale)
        else:
            sc[3] = 1.0
            if self.clip_mode == "value":
                g = g.clamp(-self.clip, self.clip)
            g = torch.where(skip, torch.zeros_like(g), g)
        t = torch.clamp(sc[1], min=1.0)
        lr_t = sc[0] * torch.sqrt(1.0 - self.b2 ** t) / (1.0 - self.b1 ** t) * keep
        b1 = 1.0 - (1.0 - self.b1) * keep
        b2 = 1.0 - (1.0 - self.b2) * keep
        self.m.mul_(b1).add_(g * (1.0 - b1))
        self.v.mul_(b2).add_(g * g * (1.0 - b2))
        self.flat.sub_(lr_t * self.m / (torch.sqrt(self.v) + self.eps))

    def skipped_steps(self) -> int:
        """Steps dropped for a non-finite gradient (one host sync)."""
        return int(self.scalars[5].item())

    # ---------------------------------------------------------------------------------
    def state_dict(self):
        return {"m": self.m, "v": self.v, "scalars": self.scalars, "step_count": self.step_count}

    def load_state_dict(self, sd):
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        gs = self.scalars[6].clone()
        self.scalars.copy_(sd["scalars"])
        self.scalars[6] = gs            # a property of this run's world size, not of the checkpoint
        self.step_count = int(sd["step_count"])
        self.lr = float(self.scalars[0])


def adam_reference_step(param, grad, m, v, t, lr, b1=0.9, b2=0.999, eps=1e-8):
    """TF Adam on plain tensors (fp64 oracle for the fused kernel tests)."""
    m = b1 * m + (1 - b1) * grad
    v = b2 * v + (1 - b2) * grad * grad
    lr_t = lr * math.sqrt(1 - b2 ** t) / (1 - b1 ** t)
    return param - lr_t * m / (torch.sqrt(v) + eps), m, v
