"""The reference model: unconditional decoder-only MDN-RNN.

Behaviour of ``model.py:7-184`` (reference capabilities R7-R12):

* ``num_layers`` stacked cells of ``rnn_size`` (``lstm`` | ``gru`` | ``rnn``);
* dropout (``keep_prob``) on the top-layer output in training only
  (``DropoutWrapper(output_keep_prob)`` around the whole stack);
* after consuming an input whose ``eoc`` flag is set, every layer's carried
  state is reset to the *batch-initial* state (``model.py:82-92``) -- for
  any number of layers (the reference hard-codes two);
* ``xw_plus_b`` output projection to ``3 + 6M`` MDN parameters;
* reference-mode MDN loss (:mod:`.mdn`).

Execution is layer-by-layer: each layer's input projection is one hoisted
GEMM over all ``T*B`` rows and only the recurrent part runs step by step
(``ops.lstm_sequence``: fused HIP recurrence on the GPU).
Inference mode (``infer=True``) is the single-step decoder used by the
sampler (``model.py:9-11``).
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.nn as nn

from .. import ops
from ..ops import gemm, inproj, persist
from ..config import RefConfig
from . import cells as C


def _stroke_proj(xt: torch.Tensor, W: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
    """Layer-0 input projection ``x @ W_x + b`` of the stroke-5 input ([T, B, 5]
    -> [T, B, 4H] fp32): csrc/inproj.hip on the HIP backend (one write of xp;
    dW / dbias from one read of dxp), an fp32 addmm elsewhere."""
    if ops.use_hip(xt) and inproj.bproj_ok(xt) and not xt.requires_grad:
        return inproj.stroke_input_proj(xt, None, W, bias)
    T, B, _ = xt.shape
    return torch.addmm(bias, xt.reshape(T * B, -1), W).view(T, B, -1)


class SketchRNN(nn.Module):
    def __init__(self, cfg: RefConfig, seed: Optional[int] = None):
        super().__init__()
        self.cfg = cfg
        gen = torch.Generator().manual_seed(cfg.seed if seed is None else seed)
        H = cfg.rnn_size
        layers = []
        for l in range(cfg.num_layers):
            in_size = 5 if l == 0 else H
            if cfg.model == "lstm":
                layers.append(C.LSTMParams(in_size, H, gen=gen))
            elif cfg.model == "gru":
                layers.append(C.GRUParams(in_size, H, gen=gen))
            elif cfg.model == "rnn":
                layers.append(C.RNNParams(in_size, H, gen=gen))
            else:
                raise ValueError("model type not supported: %s" % cfg.model)
        self.layers = nn.ModuleList(layers)
        self.output_w = nn.Parameter(C.uniform_(torch.empty(H, cfg.n_out), gen))
        self.output_b = nn.Parameter(torch.zeros(cfg.n_out))

    # -- state --------------------------------------------------------------------
    def zero_state(self, batch_size: int, device=None) -> List:
        H = self.cfg.rnn_size
        z = lambda: torch.zeros(batch_size, H, device=device)
        return [(z(), z()) if self.cfg.model == "lstm" else z() for _ in self.layers]

    @staticmethod
    def detach_state(state):
        return [tuple(s.detach() for s in st) if isinstance(st, tuple) else st.detach() for st in state]

    # -- forward --------------------------------------------------------------------
    def forward(self, x: torch.Tensor, state: Optional[List] = None, train: bool = True,
                drop_seed: int = 0, reset_on_eoc: bool = True):
        """``x [B, T, 5]`` (reference layout). Returns ``(z [T*B, NOUT], final_state)``
        with rows in time-major order."""
        out, final = self.features(x, state, reset_on_eoc)
        return self._head(out, train, drop_seed), final

    def features(self, x: torch.Tensor, state: Optional[List] = None, reset_on_eoc: bool = True):
        """Top-layer outputs ``[T*B, H]`` (time-major rows, before the output
        dropout) and the final state."""
        cfg = self.cfg
        B, T, _ = x.shape
        if state is None:
            state = self.zero_state(B, x.device)
        xt = x.transpose(0, 1).contiguous()            # [T, B, 5]
        reset = (xt[:, :, 3] > 0).to(torch.float32) if reset_on_eoc else None
        inp = xt
        final = []
        L = len(self.layers)
        if cfg.model == "lstm" and L <= 2 and ops.use_hip(x) and persist.persist_ok(cfg.rnn_size, 1, L, B=B):
            # the whole stack as ONE persistent launch (csrc/lstm_persist.hip):
            # layer 1's input projection runs inside the recurrence, so the
            # two layers advance as a wavefront
            p0 = self.layers[0]
            xp0 = _stroke_proj(xt, p0.W_x, p0.bias)
            out, final = persist.lstm_stack(
                xp0, [p.W_h for p in self.layers], [s[0] for s in state], [s[1] for s in state],
                W_in1=self.layers[1].W_x if L == 2 else None, b1=self.layers[1].bias if L == 2 else None,
                reset=reset)
            return out.reshape(T * B, -1), final
        for l, p in enumerate(self.layers):
            if cfg.model == "lstm":
                h0, c0 = state[l]
                if l == 0:   # K = 5: a trivial fp32 product
                    xp = _stroke_proj(inp, p.W_x, p.bias)
                else:        # hoisted layer-l input projection in the compute precision (bf16 MFMA)
                    xp = gemm.linear(inp.reshape(T * B, -1), p.W_x, p.bias).view(T, B, -1)
                out, (hT, cT) = ops.lstm_sequence(xp, p.W_h, h0, c0, forget_bias=1.0, reset=reset,
                                                  reset_h=h0, reset_c=c0)
                final.append((hT, cT))
            elif cfg.model == "gru":
                out, hT = ops.gru_sequence(p, inp, state[l], reset=reset, reset_h=state[l])
                final.append(hT)
            else:
                out, hT = ops.rnn_sequence(p, inp, state[l], reset=reset, reset_h=state[l])
                final.append(hT)
            inp = out
        return inp.reshape(T * B, -1), final

    def _head(self, out: torch.Tensor, train: bool, drop_seed) -> torch.Tensor:
        cfg = self.cfg
        if train and cfg.keep_prob < 1.0:
            out = out * C.dropout_mask(drop_seed, 7, 0, out.shape, cfg.keep_prob, out.device)
        # head through ops.gemm.linear (as the VAE head, vae.py:177): bf16 operands
        # in bf16 mode and the bias gradient as one column-sum kernel (torch's
        # dim-0 sum was 0.31 ms/step, profiles/r1_ref_config_kernel_summary.txt)
        return gemm.linear(out, self.output_w, self.output_b)

    def loss(self, x: torch.Tensor, y: torch.Tensor, state=None, train: bool = True, drop_seed: int = 0):
        """Reference cost: ``(cost, cost_shape, cost_pen, final_state)``."""
        out, final = self.features(x, state)
        tgt = y.transpose(0, 1).reshape(-1, 5)
        # output dropout (model.py:29-30) + head (model.py:98-99) + loss (model.py:124-178):
        # one fused kernel on the GPU (ops.mdn_head_loss)
        keep = self.cfg.keep_prob if (train and self.cfg.keep_prob < 1.0) else 1.0
        cost, shape, pen = ops.mdn_head_loss(out, self.output_w, self.output_b, tgt, self.cfg.num_mixture,
                                             mode="reference", stroke_importance=self.cfg.stroke_importance_factor,
                                             clamp=self.cfg.loss_clamp, drop_keep=keep, drop_seed=drop_seed,
                                             drop_stream=7)
        return cost, shape, pen, final

    # -- single step (sampling) --------------------------------------------------------
    @torch.no_grad()
    def step(self, x: torch.Tensor, state: List) -> Tuple[torch.Tensor, List]:
        """One decoder step at ``B`` rows: ``x [B, 5]`` -> ``z [B, NOUT]``.

        Applies the reference's T=1 eoc semantics: if the fed input has
        ``eoc`` set, the returned carried state is the fed-in state
        (``model.py:91`` with ``initial_state`` = the fed state)."""
        z, final = self.forward(x.unsqueeze(1), state, train=False)
        return z, final
