"""Pure-PyTorch recurrences (oracle / CPU backend).

Time-major everywhere: sequences are ``[T, B, ...]``. Input projections
(``x @ W_x + b``) are hoisted out of the recurrence by the callers, so each
step here only does the recurrent GEMM plus the cell's pointwise math --
the same decomposition the HIP backend (:mod:`.recurrent`) uses.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ..models import cells as C


def lstm_sequence_torch(xp: torch.Tensor, W_h: torch.Tensor, h0: torch.Tensor, c0: torch.Tensor,
                        forget_bias: float = 1.0, reset: Optional[torch.Tensor] = None,
                        reset_h: Optional[torch.Tensor] = None, reset_c: Optional[torch.Tensor] = None,
                        drop_keep: float = 1.0, drop_seed: int = 0, drop_stream: int = 0,
                        ln: Optional[Tuple[torch.Tensor, ...]] = None, mask_rows: Optional[Tuple[int, int]] = None):
    """LSTM / LayerNorm-LSTM recurrence.

    ``reset[t, b] != 0`` replaces the state carried out of step ``t`` with
    ``(reset_h, reset_c)`` -- the reference's end-of-character reset
    (``model.py:82-92``). Outputs are the un-reset cell outputs.
    ``ln = (ln_gamma, ln_beta, lnc_gamma, lnc_beta)`` selects LayerNorm-LSTM.
    ``mask_rows = (total, offset)``: this recurrence's rows are rows
    ``offset .. offset+B`` of a ``total``-row dropout mask (bidirectional
    encoder: both directions share one mask stream, as in the fused kernel).
    """
    T, B, G = xp.shape
    H = G // 4
    h, c = h0, c0
    outs = []
    total, off = mask_rows if mask_rows is not None else (B, 0)
    for t in range(T):
        g = xp[t] + h @ W_h
        drop = None
        if drop_keep < 1.0:
            drop = C.dropout_mask(drop_seed, drop_stream, t, (total, H), drop_keep, xp.device)[off:off + B]
        if ln is None:
            h_new, c_new = C.lstm_pointwise(g, c, forget_bias, drop)
        else:
            h_new, c_new = C.ln_lstm_pointwise(g, c, *ln, forget_bias=forget_bias, drop=drop)
        outs.append(h_new)
        if reset is not None:
            r = (reset[t] != 0).unsqueeze(-1)
            h = torch.where(r, reset_h, h_new)
            c = torch.where(r, reset_c, c_new)
        else:
            h, c = h_new, c_new
    return torch.stack(outs, 0), (h, c)


def hyper_sequence_torch(p: C.HyperLSTMParams, x: torch.Tensor, h0, c0, hh0, hc0, forget_bias: float = 1.0,
                         drop_keep: float = 1.0, drop_seed: int = 0, drop_stream: int = 0,
                         hyp_drop_keep: float = 1.0):
    """HyperLSTM over ``x [T, B, in]``; returns ``H [T, B, H]`` and final
    ``(h, c, hh, hc)``."""
    T, B, _ = x.shape
    H, Hh = p.hidden, p.hyper_units
    xh = x @ p.W_x                      # [T, B, 4H]
    hyp_xh = x @ p.hyp_W_x[: p.in_size]  # [T, B, 4Hh]
    h, c, hh, hc = h0, c0, hh0, hc0
    outs = []
    for t in range(T):
        drop = C.dropout_mask(drop_seed, drop_stream, t, (B, H), drop_keep, x.device) if drop_keep < 1 else None
        hdrop = C.dropout_mask(drop_seed, drop_stream + 1, t, (B, Hh), hyp_drop_keep, x.device) \
            if hyp_drop_keep < 1 else None
        h, c, hh, hc = C.hyper_lstm_step(p, x[t], xh[t], hyp_xh[t], h, c, hh, hc, forget_bias, drop, hdrop)
        outs.append(h)
    return torch.stack(outs, 0), (h, c, hh, hc)


def gru_sequence_torch(p: C.GRUParams, x: torch.Tensor, h0, reset=None, reset_h=None):
    h = h0
    outs = []
    for t in range(x.shape[0]):
        h_new = C.gru_step(p, x[t], h)
        outs.append(h_new)
        h = torch.where((reset[t] != 0).unsqueeze(-1), reset_h, h_new) if reset is not None else h_new
    return torch.stack(outs, 0), h


def rnn_sequence_torch(p: C.RNNParams, x: torch.Tensor, h0, reset=None, reset_h=None):
    h = h0
    outs = []
    for t in range(x.shape[0]):
        h_new = C.rnn_step(p, x[t], h)
        outs.append(h_new)
        h = torch.where((reset[t] != 0).unsqueeze(-1), reset_h, h_new) if reset is not None else h_new
    return torch.stack(outs, 0), h
