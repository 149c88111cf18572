"""Op dispatch: fused HIP kernels on the GPU, PyTorch oracle on the CPU.

Backend policy (``set_backend``):

* ``"auto"`` (default) -- tensors on a HIP device use the native kernels in
  ``libskrnn_hip.so``; if that library is missing on a GPU run this raises
  (no silent eager fallback); CPU tensors use the PyTorch oracle.
* ``"hip"`` -- force native (error on CPU tensors).
* ``"torch"`` -- force the PyTorch implementation everywhere (used by the
  numerics tests and by the eager comparator in ``bench.py --backend torch``).
"""
from __future__ import annotations

import torch

from .recurrent_torch import (gru_sequence_torch, hyper_sequence_torch, lstm_sequence_torch,
                              rnn_sequence_torch)

_BACKEND = "auto"
_COMPUTE_DTYPE = "fp32"   # operand precision of the recurrent / head GEMMs on the GPU


def set_compute_dtype(name: str) -> None:
    """``fp32`` | ``bf16``: operand precision of the GPU GEMMs. Accumulation,
    cell state and all pointwise math stay fp32. (No fp8: e4m3 recurrent
    GEMMs were built and measured equal to bf16 on every decode shape --
    README "fp8" -- and removed.)"""
    global _COMPUTE_DTYPE
    if name not in ("fp32", "bf16"):
        raise ValueError(name)
    _COMPUTE_DTYPE = name


def get_compute_dtype() -> str:
    return _COMPUTE_DTYPE


def set_backend(name: str) -> None:
    global _BACKEND
    if name not in ("auto", "hip", "torch"):
        raise ValueError(name)
    _BACKEND = name


def get_backend() -> str:
    return _BACKEND


def use_hip(t: torch.Tensor) -> bool:
    if _BACKEND == "torch":
        return False
    if not t.is_cuda:
        if _BACKEND == "hip":
            raise RuntimeError("backend 'hip' requested for a CPU tensor")
        return False
    from ..utils import native
    native.require_hip()  # raises loudly when the extension is missing
    return True


def lstm_sequence(xp, W_h, h0, c0, forget_bias: float = 1.0, reset=None, reset_h=None, reset_c=None,
                  drop_keep: float = 1.0, drop_seed: int = 0, drop_stream: int = 0, ln=None):
    if use_hip(xp):
        from .recurrent import lstm_sequence_hip
        return lstm_sequence_hip(xp, W_h, h0, c0, forget_bias, reset, reset_h, reset_c,
                                 drop_keep, drop_seed, drop_stream, ln)
    return lstm_sequence_torch(xp, W_h, h0, c0, forget_bias, reset, reset_h, reset_c,
                               drop_keep, drop_seed, drop_stream, ln)


def bilstm_sequence(xp_f, xp_b, W_f, W_b, h0, c0, drop_keep: float = 1.0, drop_seed: int = 0,
                    drop_stream: int = 0, ln_f=None, ln_b=None, forget_bias: float = 1.0):
    """Two independent recurrences of equal shape (the encoder's forward and
    backward directions). Returns the two output sequences. One dropout
    stream covers both as ``2B`` rows (forward rows first)."""
    if use_hip(xp_f):
        from .recurrent import bilstm_sequence_hip
        return bilstm_sequence_hip(xp_f, xp_b, W_f, W_b, h0, c0, drop_keep, drop_seed, (drop_stream, drop_stream),
                                   ln_f, ln_b, forget_bias)
    B = xp_f.shape[1]
    of, _ = lstm_sequence_torch(xp_f, W_f, h0, c0, forget_bias, drop_keep=drop_keep, drop_seed=drop_seed,
                                drop_stream=drop_stream, ln=ln_f, mask_rows=(2 * B, 0))
    ob, _ = lstm_sequence_torch(xp_b, W_b, h0, c0, forget_bias, drop_keep=drop_keep, drop_seed=drop_seed,
                                drop_stream=drop_stream, ln=ln_b, mask_rows=(2 * B, B))
    return of, ob


def bilstm_sequence_packed(xp, W_f, W_b, h0, c0, drop_keep: float = 1.0, drop_seed: int = 0,
                           drop_stream: int = 0, ln_f=None, ln_b=None, forget_bias: float = 1.0, lengths=None):
    """:func:`bilstm_sequence` with both directions' input projections packed
    as ``xp [T, 2B, 4H]`` (forward rows first), e.g. from
    :func:`.inproj.bilstm_input_proj`. ``lengths [B]`` (optional): outputs at
    ``t >= lengths[b]`` are never read by the caller, so a backend may skip
    those steps (their values are then unspecified; the oracle computes them)."""
    if use_hip(xp):
        from .recurrent import bilstm_sequence_packed_hip
        return bilstm_sequence_packed_hip(xp, W_f, W_b, h0, c0, drop_keep, drop_seed, (drop_stream, drop_stream),
                                          ln_f, ln_b, forget_bias, lengths)
    B = xp.shape[1] // 2
    return bilstm_sequence(xp[:, :B], xp[:, B:], W_f, W_b, h0, c0, drop_keep, drop_seed, drop_stream, ln_f, ln_b,
                           forget_bias)


def hyper_sequence(p, x, h0, c0, hh0, hc0, forget_bias: float = 1.0, drop_keep: float = 1.0,
                   drop_seed: int = 0, drop_stream: int = 0, hyp_drop_keep: float = 1.0, zc=None):
    """HyperLSTM over the input ``[x | zc broadcast over time]`` (``zc``
    optional: a per-sequence input whose projection is computed once)."""
    if use_hip(x):
        from .hyper import hyper_sequence_hip
        return hyper_sequence_hip(p, x, h0, c0, hh0, hc0, forget_bias, drop_keep, drop_seed,
                                  drop_stream, hyp_drop_keep, zc)
    if zc is not None:
        x = torch.cat([x, zc.unsqueeze(0).expand(x.shape[0], x.shape[1], zc.shape[-1])], -1)
    return hyper_sequence_torch(p, x, h0, c0, hh0, hc0, forget_bias, drop_keep, drop_seed,
                                drop_stream, hyp_drop_keep)


def gru_sequence(p, x, h0, reset=None, reset_h=None):
    """TF GRUCell recurrence over ``x [T, B, in]`` -> ``(H [T, B, H], h_T)``."""
    if use_hip(x):
        from .recurrent_gru import gru_sequence_hip
        return gru_sequence_hip(p, x, h0, reset, reset_h)
    return gru_sequence_torch(p, x, h0, reset, reset_h)


def rnn_sequence(p, x, h0, reset=None, reset_h=None):
    """tanh-RNN recurrence over ``x [T, B, in]`` -> ``(H [T, B, H], h_T)``."""
    if use_hip(x):
        from .recurrent_gru import rnn_sequence_hip
        return rnn_sequence_hip(p, x, h0, reset, reset_h)
    return rnn_sequence_torch(p, x, h0, reset, reset_h)


def mdn_loss(z, target, M: int, mode: str = "magenta", stroke_importance: float = 200.0,
             is_training: bool = True, clamp: float = 1e-20, eps: float = 1e-6):
    """``(total, shape_term, pen_term)`` means over rows (see models.mdn)."""
    if use_hip(z):
        from .mdn_hip import mdn_loss_hip
        return mdn_loss_hip(z, target, M, mode, stroke_importance, is_training, clamp, eps)
    from ..models.mdn import mdn_loss_torch
    return mdn_loss_torch(z, target, M, mode, stroke_importance, is_training, clamp, eps)


def mdn_head_loss(x, W, b, target, M: int, mode: str = "magenta", stroke_importance: float = 200.0,
                  is_training: bool = True, clamp: float = 1e-20, eps: float = 1e-6,
                  drop_keep: float = 1.0, drop_seed=0, drop_stream: int = 0, x_lp=None):
    """MDN loss of the head ``z = dropout(x) @ W + b`` (``x [..., Hd]``;
    ``x_lp``: an optional bf16 copy of ``x`` the fused head may read instead).

    bf16 HIP training: ONE kernel computes the projection on MFMA, the loss
    and dL/dz (csrc/mdn_head.hip; z never reaches HBM) and the backward runs
    hand-written MFMA kernels. Otherwise: dropout, ``gemm.linear`` and
    :func:`mdn_loss` (identical math, reference model.py:98-178)."""
    from .mdn_hip import head_fused_ok
    if head_fused_ok(x, W, M) and torch.is_grad_enabled():
        from .mdn_hip import mdn_head_loss_hip
        return mdn_head_loss_hip(x, W, b, target, M, mode, stroke_importance, is_training, clamp, eps,
                                 drop_keep, drop_seed, drop_stream, x_lp)
    from . import gemm
    from ..models.cells import dropout_mask
    x2 = x.reshape(-1, x.shape[-1])
    if drop_keep < 1.0:
        x2 = x2 * dropout_mask(drop_seed, drop_stream, 0, x2.shape, drop_keep, x2.device)
    z = gemm.linear(x2, W, b)
    return mdn_loss(z, target, M, mode, stroke_importance, is_training, clamp, eps)
