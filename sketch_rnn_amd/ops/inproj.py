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
        rc = lib.lib.skr_inproj_bwd(x.data_ptr(), ln.data_ptr(), dxp.data_ptr(), 0, part.data_ptr(), T, B, IN, G, RS,
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


# ---- decoder: [stroke-5 | z] inputs with z broadcast over time ------------------------
def bproj_ok(x) -> bool:
    return x.is_cuda and x.shape[-1] in (3, 5)


def bproj_fwd(x, W, zw=None, bf16: bool = False):
    """``xp[t, b] = x[t, b] @ W + zw[b]`` (csrc/inproj.hip ``skr_bproj_fwd``);
    ``bf16``: xp stored as bf16."""
    lib = native.require_hip()
    T, B, IN = x.shape
    G = W.shape[1]
    x = x.contiguous().float()
    W = W.contiguous().float()
    zw = zw.contiguous().float() if zw is not None else None
    xp = torch.empty(T, B, G, device=x.device, dtype=torch.bfloat16 if bf16 else torch.float32)
    rc = lib.lib.skr_bproj_fwd(x.data_ptr(), W.data_ptr(), None if zw is None else zw.data_ptr(), xp.data_ptr(),
                               T, B, IN, G, int(bf16), torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError("skr_bproj_fwd failed (%d)" % rc)
    return xp


# bproj_reduce on the wide kernel (csrc/inproj.hip bproj_bwd_wide: 16-byte
# loads, the T steps split over 4 waves) where its alignment holds; False:
# the narrow kernel (the A/B arm).
BPROJ_WIDE = True
_WIDE_SET = [None]


def bproj_reduce(x, dxp, raw: bool = False):
    """One read of ``dxp [T, B, G]`` (fp32 or bf16, rows may be strided):
    ``S[b] = sum_t dxp[t, b]`` and ``P = sum_{t,b} x[t, b]^T dxp[t, b]`` ([IN, G]);
    ``raw``: P as the kernel's per-row partials ``[B, IN, G]`` (the caller
    sums them inside a grouped small-GEMM launch, :func:`gemm.ones_row`)."""
    lib = native.require_hip()
    T, B, IN = x.shape
    G = dxp.shape[-1]
    assert dxp.stride(-1) == 1 and dxp.stride(0) == B * dxp.stride(1)
    kind = 1 if dxp.dtype == torch.bfloat16 else 2
    if kind == 2 and dxp.dtype != torch.float32:
        dxp = dxp.float().contiguous()
    if _WIDE_SET[0] != BPROJ_WIDE:
        lib.lib.skr_bproj_set_wide(int(BPROJ_WIDE))
        _WIDE_SET[0] = BPROJ_WIDE
    S = torch.empty(B, G, device=x.device, dtype=torch.float32)
    P = torch.empty(B, IN, G, device=x.device, dtype=torch.float32)
    rc = lib.lib.skr_bproj_bwd(x.contiguous().data_ptr(), dxp.data_ptr(), kind, dxp.stride(1), S.data_ptr(),
                               P.data_ptr(), T, B, IN, G, torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError("skr_bproj_bwd failed (%d)" % rc)
    return (S, P) if raw else (S, P.sum(0))


# Backward reductions of the stroke projections (row sums of the per-row
# partials, the bias and z-side products) as ONE grouped small-GEMM launch;
# False: torch reduce / cat / library GEMMs (the A/B arm).
GROUPED_REDUCE = True


class _BProj(torch.autograd.Function):
    """The z part once per sequence (``csrc/small_gemm.hip``, bias folded in),
    the stroke part per (t, b) in ``skr_bproj_fwd``; backward: one read of
    dxp, then every reduction and z-side product in ONE grouped small-GEMM
    launch (no library GEMM, cat or reduce kernels on the step)."""

    @staticmethod
    def forward(ctx, x, zc, W, bias):
        from . import gemm
        IN = x.shape[-1]
        zw = None
        if zc is not None:
            zw = gemm.small_mm(zc, W[IN:], bias) if GROUPED_REDUCE else zc @ W[IN:]
        if bias is not None and not (zc is not None and GROUPED_REDUCE):
            zw = bias.expand(x.shape[1], -1) if zw is None else zw + bias
        ctx.save_for_backward(x, zc, W)
        ctx.has_bias = bias is not None
        return bproj_fwd(x, W[:IN], zw)

    @staticmethod
    def backward(ctx, dxp):
        from . import gemm
        x, zc, W = ctx.saved_tensors
        T, B, IN = x.shape
        G = W.shape[1]
        if not GROUPED_REDUCE:
            S, P = bproj_reduce(x, dxp.contiguous())
            dW = P if zc is None else torch.cat([P, zc.t() @ S], 0)
            dzc = S @ W[IN:].t() if zc is not None and ctx.needs_input_grad[1] else None
            return None, dzc, dW, S.sum(0) if ctx.has_bias else None
        S, P = bproj_reduce(x, dxp.contiguous(), raw=True)
        one = gemm.ones_row(B, x.device)
        dW = torch.empty_like(W)
        g = gemm.SmallGroup(x.device)
        g.mm(one, P.view(B, IN * G), out=dW[:IN].view(1, IN * G))   # sum over rows of the per-row partials
        dzc = db = None
        if zc is not None:
            g.mm(zc.t(), S, out=dW[IN:])
            if ctx.needs_input_grad[1]:
                dzc = g.mm(S, W[IN:].t())
        if ctx.has_bias:
            db = g.mm(one, S).view(G)
        g.run()
        return None, dzc, dW, db


def stroke_input_proj(x, zc, W, bias=None):
    """``[x | zc broadcast over T] @ W + bias`` -> ``[T, B, G]`` fp32 with the
    z part computed once per sequence (x: data, no gradient)."""
    from . import use_hip
    if bproj_ok(x) and not x.requires_grad and use_hip(x):
        return _BProj.apply(x, zc, W, bias)
    T, B, _ = x.shape
    xin = x if zc is None else torch.cat([x, zc.unsqueeze(0).expand(T, B, zc.shape[-1])], -1)
    from . import gemm
    xp = gemm.linear(xin, W)
    return xp + bias if bias is not None else xp
