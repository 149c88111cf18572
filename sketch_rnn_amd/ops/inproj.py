"""Bidirectional-encoder input projection for narrow (stroke-5) inputs.

``xp[t, d*B + b] = x_d[t, b] @ W_d + bias_d`` for both directions in one
pass, in the ``[T, 2B, 4H]`` layout :func:`..recurrent.bilstm_sequence_packed_hip`
consumes, with the backward direction reading each sketch reversed within its
length (``x_1 = reverse_padded(x, lengths)``, models/vae.py). On the GPU this
is ``csrc/inproj.hip`` (forward: one write of xp; backward: dW and dbias from
one read of dxp) instead of two K=5 library GEMMs, two bias adds and a
concatenation in the forward and two column sums in the backward.
Reference behaviour being reproduced: Magenta's bidirectional encoder
(`sketch_rnn/model.py` encoder with `tf.nn.bidirectional_dynamic_rnn`); the
reference repo itself has no encoder.
"""
from __future__ import annotations

import torch

from ..utils import native


def _reverse_padded(x, lengths):
    T = x.shape[0]
    t = torch.arange(T, device=x.device).unsqueeze(1)
    src = lengths.unsqueeze(0) - 1 - t
    src = torch.where(src >= 0, src, t)
    return torch.gather(x, 0, src.unsqueeze(-1).expand_as(x))


def bilstm_input_proj_torch(x, lengths, W_f, W_b, b_f=None, b_b=None):
    T, B, IN = x.shape
    xr = _reverse_padded(x, lengths)
    xp_f = (x.reshape(T * B, IN) @ W_f).view(T, B, -1)
    xp_b = (xr.reshape(T * B, IN) @ W_b).view(T, B, -1)
    if b_f is not None:
        xp_f = xp_f + b_f
        xp_b = xp_b + b_b
    return torch.cat([xp_f, xp_b], 1)


class _BiInProj(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, lengths, W_f, W_b, b_f, b_b):
        lib = native.require_hip()
        T, B, IN = x.shape
        G = W_f.shape[1]
        x = x.contiguous().float()
        ln = lengths.to(device=x.device, dtype=torch.int64).contiguous()
        W = torch.stack([W_f, W_b]).float().contiguous()
        bias = torch.stack([b_f, b_b]).float().contiguous() if b_f is not None else None
        xp = torch.empty(T, 2 * B, G, device=x.device, dtype=torch.float32)
        rc = lib.lib.skr_inproj_fwd(x.data_ptr(), ln.data_ptr(), W.data_ptr(),
                                    None if bias is None else bias.data_ptr(), xp.data_ptr(), T, B, IN, G,
                                    torch.cuda.current_stream().cuda_stream)
        if rc != 0:
            raise RuntimeError("skr_inproj_fwd failed (%d)" % rc)
        ctx.save_for_backward(x, ln)
        ctx.has_bias = bias is not None
        return xp

    @staticmethod
    def backward(ctx, dxp):
        lib = native.require_hip()
        x, ln = ctx.saved_tensors
        T, B, IN = x.shape
        G = dxp.shape[-1]
        dxp = dxp.contiguous()
        RS = min(T, 64)
        part = torch.empty(RS, 2, IN + 1, G, device=x.device, dtype=torch.float32)
        rc = lib.lib.skr_inproj_bwd(x.data_ptr(), ln.data_ptr(), dxp.data_ptr(), part.data_ptr(), T, B, IN, G, RS,
                                    torch.cuda.current_stream().cuda_stream)
        if rc != 0:
            raise RuntimeError("skr_inproj_bwd failed (%d)" % rc)
        red = part.sum(0)                                   # [2, IN + 1, G]
        db = (red[0, IN], red[1, IN]) if ctx.has_bias else (None, None)
        return None, None, red[0, :IN], red[1, :IN], db[0], db[1]


def bilstm_input_proj(x, lengths, W_f, W_b, b_f=None, b_b=None):
    """``[T, 2B, G]`` input projections of both encoder directions."""
    if x.is_cuda and x.shape[-1] in (3, 5) and not x.requires_grad:
        from . import use_hip
        if use_hip(x):
            return _BiInProj.apply(x, lengths, W_f, W_b, b_f, b_b)
    return bilstm_input_proj_torch(x, lengths, W_f, W_b, b_f, b_b)
