"""Recurrent cell definitions: parameters + pure-PyTorch step functions.

The step functions here are the numerics *oracle* (fp32, autograd) for the
fused HIP recurrence in :mod:`sketch_rnn_amd.ops.recurrent`, and the CPU
execution path.

Cells (gate order ``i, j, f, o`` everywhere, ``j`` = candidate):

* ``lstm`` -- TF ``BasicLSTMCell`` semantics used by the reference
  (``model.py:18-23``): ``c' = c*sig(f + 1) + sig(i)*tanh(j)``,
  ``h' = tanh(c')*sig(o)``; optional recurrent dropout on ``tanh(j)``
  (sketch-rnn VAE ``LSTMCell``).
* ``gru`` / ``rnn`` -- TF ``GRUCell`` / ``BasicRNNCell`` (``model.py:14-25``;
  the reference's ``rnn`` path crashes on ``state_is_tuple``, fixed here).
* ``layer_norm`` -- LayerNorm-LSTM: LN over each gate block of the
  (bias-free) pre-activations with per-gate gamma/beta, LN on ``c'`` before
  the output tanh (epsilon 1e-3).
* ``hyper`` -- HyperLSTM: a LayerNorm-LSTM hyper cell reads ``[x, h]`` and
  emits per-gate scaling (and, on the recurrent path, shift) vectors for the
  main LSTM's ``W_xh x`` and ``W_hh h`` terms, followed by LN.

Recurrent dropout masks are produced by :func:`hash_uniform`, a stateless
counter hash that the HIP kernels evaluate bit-identically, so the fused
kernels and this oracle agree exactly even with dropout on.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

LN_EPS = 1e-3
_M32 = 0xFFFFFFFF


# ----------------------------------------------------------------------------
# stateless dropout hash (mirrors csrc/common.h: skr_hash32 / skr_uniform)
# ----------------------------------------------------------------------------
def _mix32(x: torch.Tensor) -> torch.Tensor:
    x = x & _M32
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    x = x ^ (x >> 16)
    return x


def hash_uniform(seed, stream: int, step: int, shape, device=None) -> torch.Tensor:
    """U[0,1) per element of ``shape`` from (seed, stream, step, flat index).

    ``seed`` may be a Python int or a 1-element int64 tensor (device-resident
    seeds keep the HIP-graph-captured step valid across replays)."""
    n = 1
    for s in shape:
        n *= s
    base = (stream * 0x85EBCA77 + step * 0xC2B2AE3D) & _M32
    if torch.is_tensor(seed):
        device = seed.device
        s64 = seed.reshape(()).to(torch.int64) & _M32
    else:
        s64 = torch.tensor(int(seed) & _M32, dtype=torch.int64, device=device)
    key = _mix32((s64 * 0x9E3779B1 + base) & _M32)
    idx = torch.arange(n, dtype=torch.int64, device=device)
    h = _mix32(idx ^ key)
    h = _mix32(h + key)
    return ((h >> 8).to(torch.float32) * (1.0 / 16777216.0)).view(*shape)


def hash_normal(seed, stream: int, step: int, shape, device=None) -> torch.Tensor:
    """N(0, 1) per element (Box-Muller over two hash_uniform streams): the
    VAE's reparameterisation noise, a pure function of (seed, stream, step)
    like the dropout masks -- independent of any process-global RNG state,
    so a step replays identically (HIP graphs, resume, two fresh runs)."""
    if torch.is_tensor(seed) and seed.is_cuda and seed.dtype == torch.int64:
        from ..utils import native
        lib = native.hip_lib()
        if lib is not None:   # one kernel (csrc/noise.hip) instead of ~40 int64 torch ops
            n = 1
            for s_ in shape:
                n *= s_
            out = torch.empty(*shape, device=seed.device, dtype=torch.float32)
            rc = lib.lib.skr_hash_normal(seed.data_ptr(), stream & _M32, step & _M32, out.data_ptr(), n,
                                         torch.cuda.current_stream(seed.device).cuda_stream)
            if rc != 0:
                raise RuntimeError("skr_hash_normal failed (%d)" % rc)
            return out
    u1 = 1.0 - hash_uniform(seed, stream, step, shape, device)        # (0, 1]
    u2 = hash_uniform(seed, stream + 0x3C6EF372, step, shape, device)
    return torch.sqrt(-2.0 * torch.log(u1)) * torch.cos((2.0 * math.pi) * u2)


def dropout_mask(seed: int, stream: int, step: int, shape, keep: float, device=None) -> torch.Tensor:
    """Inverted-dropout multiplier: ``1/keep`` where kept, else 0."""
    u = hash_uniform(seed, stream, step, shape, device)
    return (u < keep).to(torch.float32) * (1.0 / keep)


# ----------------------------------------------------------------------------
# initializers
# ----------------------------------------------------------------------------
def orthogonal_lstm_(w: torch.Tensor, scale: float = 1.0, gen: Optional[torch.Generator] = None):
    """Orthogonal init per ``H x H`` gate block of ``W_hh [H, 4H]``."""
    h = w.shape[0]
    blocks = []
    for _ in range(w.shape[1] // h):
        a = torch.randn(h, h, generator=gen, dtype=torch.float64)
        q, r = torch.linalg.qr(a)
        q = q * torch.sign(torch.diagonal(r)).unsqueeze(0)
        blocks.append(q)
    with torch.no_grad():
        w.copy_((torch.cat(blocks, 1) * scale).to(w.dtype))
    return w


def uniform_(w: torch.Tensor, gen=None):
    fan_in, fan_out = w.shape[0], w.shape[1]
    lim = math.sqrt(6.0 / (fan_in + fan_out))
    with torch.no_grad():
        w.copy_(torch.rand(w.shape, generator=gen) * 2 * lim - lim)
    return w


# ----------------------------------------------------------------------------
# step functions (oracle)
# ----------------------------------------------------------------------------
def lstm_pointwise(g: torch.Tensor, c: torch.Tensor, forget_bias: float = 1.0,
                   drop: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    i, j, f, o = g.chunk(4, dim=-1)
    gj = torch.tanh(j)
    if drop is not None:
        gj = gj * drop
    c_new = c * torch.sigmoid(f + forget_bias) + torch.sigmoid(i) * gj
    h_new = torch.tanh(c_new) * torch.sigmoid(o)
    return h_new, c_new


def layer_norm_all(g: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, nblocks: int = 4,
                   eps: float = LN_EPS) -> torch.Tensor:
    shp = g.shape
    gr = g.reshape(*shp[:-1], nblocks, shp[-1] // nblocks)
    mean = gr.mean(-1, keepdim=True)
    var = ((gr - mean) ** 2).mean(-1, keepdim=True)
    gr = (gr - mean) * torch.rsqrt(var + eps)
    return gr.reshape(shp) * gamma + beta


def layer_norm(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float = LN_EPS) -> torch.Tensor:
    mean = x.mean(-1, keepdim=True)
    xs = x - mean
    var = (xs * xs).mean(-1, keepdim=True)
    return gamma * xs * torch.rsqrt(var + eps) + beta


def ln_lstm_pointwise(g, c, ln_g, ln_b, lnc_g, lnc_b, forget_bias=1.0, drop=None):
    g = layer_norm_all(g, ln_g, ln_b)
    i, j, f, o = g.chunk(4, dim=-1)
    gj = torch.tanh(j)
    if drop is not None:
        gj = gj * drop
    c_new = c * torch.sigmoid(f + forget_bias) + torch.sigmoid(i) * gj
    h_new = torch.tanh(layer_norm(c_new, lnc_g, lnc_b)) * torch.sigmoid(o)
    return h_new, c_new


# ----------------------------------------------------------------------------
# parameter containers
# ----------------------------------------------------------------------------
class LSTMParams(nn.Module):
    """``W_x [in, 4H]``, ``W_h [H, 4H]``, ``bias [4H]`` (TF ``Linear``)."""

    def __init__(self, in_size: int, hidden: int, bias: bool = True, gen=None):
        super().__init__()
        self.in_size, self.hidden = in_size, hidden
        self.W_x = nn.Parameter(uniform_(torch.empty(in_size, 4 * hidden), gen))
        self.W_h = nn.Parameter(orthogonal_lstm_(torch.empty(hidden, 4 * hidden), 1.0, gen))
        self.bias = nn.Parameter(torch.zeros(4 * hidden)) if bias else None


class LNLSTMParams(nn.Module):
    def __init__(self, in_size: int, hidden: int, gen=None):
        super().__init__()
        self.in_size, self.hidden = in_size, hidden
        self.W_x = nn.Parameter(uniform_(torch.empty(in_size, 4 * hidden), gen))
        self.W_h = nn.Parameter(orthogonal_lstm_(torch.empty(hidden, 4 * hidden), 1.0, gen))
        self.ln_gamma = nn.Parameter(torch.ones(4 * hidden))
        self.ln_beta = nn.Parameter(torch.zeros(4 * hidden))
        self.lnc_gamma = nn.Parameter(torch.ones(hidden))
        self.lnc_beta = nn.Parameter(torch.zeros(hidden))


class GRUParams(nn.Module):
    """TF GRUCell: gates ``[r, u]`` (bias 1.0) and candidate."""

    def __init__(self, in_size: int, hidden: int, gen=None):
        super().__init__()
        self.in_size, self.hidden = in_size, hidden
        self.W_gx = nn.Parameter(uniform_(torch.empty(in_size, 2 * hidden), gen))
        self.W_gh = nn.Parameter(uniform_(torch.empty(hidden, 2 * hidden), gen))
        self.b_g = nn.Parameter(torch.ones(2 * hidden))
        self.W_cx = nn.Parameter(uniform_(torch.empty(in_size, hidden), gen))
        self.W_ch = nn.Parameter(uniform_(torch.empty(hidden, hidden), gen))
        self.b_c = nn.Parameter(torch.zeros(hidden))


class RNNParams(nn.Module):
    def __init__(self, in_size: int, hidden: int, gen=None):
        super().__init__()
        self.in_size, self.hidden = in_size, hidden
        self.W_x = nn.Parameter(uniform_(torch.empty(in_size, hidden), gen))
        self.W_h = nn.Parameter(uniform_(torch.empty(hidden, hidden), gen))
        self.bias = nn.Parameter(torch.zeros(hidden))


# order of the 12 hyper-norm embeddings in the packed [Hh, 12*E] projection:
# 8 scale embeddings (ix, jx, fx, ox, ih, jh, fh, oh) then 4 shift embeddings (ih, jh, fh, oh)
HYPER_SCALE_X, HYPER_SCALE_H, HYPER_SHIFT_H = slice(0, 4), slice(4, 8), slice(8, 12)


class HyperLSTMParams(nn.Module):
    """HyperLSTM: main LSTM ``H`` + LayerNorm-LSTM hyper cell ``Hh``.

    Packed hyper-norm projections (each a 2-layer linear map with no
    non-linearity, recurrent-batch-norm-style init):

    * ``W_z [Hh, 12E]``, ``b_z [12E]`` -- hyper output -> 12 embeddings
      (8 scale with bias 1.0 and zero weights; 4 shift, gaussian 0.01, no bias);
    * ``W_a [12, E, H]`` -- embedding -> per-unit vector (scale blocks init
      ``0.1 / E``, shift blocks init 0).
    """

    def __init__(self, in_size: int, hidden: int, hyper_units: int = 256, embed: int = 32,
                 use_layer_norm: bool = True, gen=None):
        super().__init__()
        self.in_size, self.hidden, self.hyper_units, self.embed = in_size, hidden, hyper_units, embed
        self.use_layer_norm = use_layer_norm
        H, Hh, E = hidden, hyper_units, embed
        self.W_x = nn.Parameter(uniform_(torch.empty(in_size, 4 * H), gen))
        self.W_h = nn.Parameter(orthogonal_lstm_(torch.empty(H, 4 * H), 1.0, gen))
        self.bias = nn.Parameter(torch.zeros(4 * H))
        # hyper cell: LN-LSTM over input [x, h]
        self.hyp_W_x = nn.Parameter(uniform_(torch.empty(in_size + H, 4 * Hh), gen))
        self.hyp_W_h = nn.Parameter(orthogonal_lstm_(torch.empty(Hh, 4 * Hh), 1.0, gen))
        self.hyp_ln_gamma = nn.Parameter(torch.ones(4 * Hh))
        self.hyp_ln_beta = nn.Parameter(torch.zeros(4 * Hh))
        self.hyp_lnc_gamma = nn.Parameter(torch.ones(Hh))
        self.hyp_lnc_beta = nn.Parameter(torch.zeros(Hh))
        wz = torch.zeros(Hh, 12 * E)
        wz[:, 8 * E:] = torch.randn(Hh, 4 * E, generator=gen) * 0.01
        self.W_z = nn.Parameter(wz)
        bz = torch.zeros(12 * E)
        bz[: 8 * E] = 1.0
        self.b_z = nn.Parameter(bz)
        wa = torch.zeros(12, E, H)
        wa[:8] = 0.1 / E
        self.W_a = nn.Parameter(wa)
        if use_layer_norm:
            self.ln_gamma = nn.Parameter(torch.ones(4 * H))
            self.ln_beta = nn.Parameter(torch.zeros(4 * H))
            self.lnc_gamma = nn.Parameter(torch.ones(H))
            self.lnc_beta = nn.Parameter(torch.zeros(H))


def hyper_lstm_step(p: HyperLSTMParams, x: torch.Tensor, xh: torch.Tensor, hyp_xh: torch.Tensor,
                    h, c, hh, hc, forget_bias=1.0, drop=None, hyp_drop=None):
    """One HyperLSTM step (oracle).

    ``xh = x @ W_x`` and ``hyp_xh = x @ hyp_W_x[:in]`` are precomputed.
    Returns ``(h', c', hh', hc')``.
    """
    H, E = p.hidden, p.embed
    # hyper cell (LN-LSTM on [x, h])
    hg = hyp_xh + h @ p.hyp_W_x[p.in_size:] + hh @ p.hyp_W_h
    hh_new, hc_new = ln_lstm_pointwise(hg, hc, p.hyp_ln_gamma, p.hyp_ln_beta, p.hyp_lnc_gamma,
                                       p.hyp_lnc_beta, forget_bias, hyp_drop)
    zs = hh_new @ p.W_z + p.b_z                                   # [B, 12E]
    vec = torch.einsum("bke,keh->bkh", zs.view(-1, 12, E), p.W_a)  # [B, 12, H]
    hhmat = h @ p.W_h                                             # [B, 4H]
    xg = xh.view(-1, 4, H) * vec[:, 0:4]
    rg = hhmat.view(-1, 4, H) * vec[:, 4:8] + vec[:, 8:12]
    g = (xg + rg).reshape(-1, 4 * H) + p.bias
    if p.use_layer_norm:
        h_new, c_new = ln_lstm_pointwise(g, c, p.ln_gamma, p.ln_beta, p.lnc_gamma, p.lnc_beta, forget_bias, drop)
    else:
        h_new, c_new = lstm_pointwise(g, c, forget_bias, drop)
    return h_new, c_new, hh_new, hc_new


def gru_step(p: GRUParams, x, h):
    ru = torch.sigmoid(x @ p.W_gx + h @ p.W_gh + p.b_g)
    r, u = ru.chunk(2, -1)
    cand = torch.tanh(x @ p.W_cx + (r * h) @ p.W_ch + p.b_c)
    return u * h + (1 - u) * cand


def rnn_step(p: RNNParams, x, h):
    return torch.tanh(x @ p.W_x + h @ p.W_h + p.bias)
