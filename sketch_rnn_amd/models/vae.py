"""seq2seq VAE: bidirectional-LSTM encoder, latent z, RNN decoder, MDN head.

Public API (sketch-rnn VAE semantics, see BASELINE.json north star):

* :class:`SketchVAE(cfg)` -- ``cfg.dec_model`` in ``lstm | layer_norm | hyper``,
  ``cfg.enc_model`` in ``lstm | layer_norm``; ``cfg.conditional`` toggles the
  encoder / latent; ``cfg.num_classes > 0`` adds a class embedding to z.
* ``model.encode(strokes, lengths)`` -> ``(mu, presig)``
* ``model.loss(strokes, lengths, labels, kl_weight)`` -> dict with
  ``cost = r_cost + kl_weight * max(KL, kl_tolerance)``, ``r_cost``, ``kl_cost``
* ``model.initial_state(z)`` / ``model.decode_step(x, z, state)`` for sampling.

Data layout: magenta stroke-5 ``[B, Nmax + 1, 5]`` with the S0 token at
``t = 0``; the decoder is teacher-forced on ``strokes[:, :Nmax]`` and
predicts ``strokes[:, 1:]``; the encoder reads ``strokes[:, 1:]`` with true
lengths (forward direction gathers ``h[len - 1]``, backward direction runs
on the per-row reversed prefix).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn as nn

from .. import ops
from ..config import VAEConfig
from ..ops import gemm
from . import cells as C
from ..ops.inproj import bilstm_input_proj, stroke_input_proj

# dropout hash streams
_S_ENC_FW, _S_ENC_BW, _S_DEC, _S_IN, _S_OUT, _S_EPS = 11, 13, 17, 23, 29, 31
# False: the latent layer as separate torch ops (the oracle form; tests)
LATENT_FUSED = True


def _gaussian(shape, std, gen):
    return torch.randn(shape, generator=gen) * std


def reverse_padded(x: torch.Tensor, lengths: torch.Tensor) -> torch.Tensor:
    """Reverse each row's first ``len`` steps of a time-major ``[T, B, D]``."""
    T = x.shape[0]
    t = torch.arange(T, device=x.device).unsqueeze(1)
    src = lengths.unsqueeze(0) - 1 - t
    src = torch.where(src >= 0, src, t)  # beyond the length: keep (never read)
    return torch.gather(x, 0, src.unsqueeze(-1).expand_as(x))


class Encoder(nn.Module):
    def __init__(self, cfg: VAEConfig, gen):
        super().__init__()
        self.cfg = cfg
        Cls = C.LNLSTMParams if cfg.enc_model == "layer_norm" else C.LSTMParams
        self.fw = Cls(5, cfg.enc_rnn_size, gen=gen)
        self.bw = Cls(5, cfg.enc_rnn_size, gen=gen)
        self.mu_w = nn.Parameter(_gaussian((2 * cfg.enc_rnn_size, cfg.z_size), 0.001, gen))
        self.mu_b = nn.Parameter(torch.zeros(cfg.z_size))
        self.sig_w = nn.Parameter(_gaussian((2 * cfg.enc_rnn_size, cfg.z_size), 0.001, gen))
        self.sig_b = nn.Parameter(torch.zeros(cfg.z_size))

    def forward(self, x: torch.Tensor, lengths: torch.Tensor, train: bool, seed: int):
        """``x [T, B, 5]`` time-major -> ``(mu, presig)``."""
        last_h = self.last_hidden(x, lengths, train, seed)
        return last_h @ self.mu_w + self.mu_b, last_h @ self.sig_w + self.sig_b

    def last_hidden(self, x: torch.Tensor, lengths: torch.Tensor, train: bool, seed: int) -> torch.Tensor:
        """``[h_fw[len-1] | h_bw[len-1]]`` ([B, 2H]): the encoder summary the
        latent heads read."""
        cfg = self.cfg
        T, B, _ = x.shape
        H = cfg.enc_rnn_size
        keep = cfg.recurrent_dropout_prob if (train and cfg.use_recurrent_dropout) else 1.0
        ln = isinstance(self.fw, C.LNLSTMParams)
        from ..ops import persist
        if not ln and persist.bilstm_last_ok(x, H, B):
            # one autograd node: input projection + persistent biLSTM writing
            # only h[len - 1] of each row (ops/persist.py _PersistBiEncoder)
            return persist.bilstm_last_h(x, lengths, self.fw.W_x, self.bw.W_x, self.fw.bias, self.bw.bias,
                                         self.fw.W_h, self.bw.W_h, drop_keep=keep, drop_seed=seed,
                                         drop_stream=_S_ENC_FW)
        zeros = x.new_zeros(B, H)
        lns = [(p.ln_gamma, p.ln_beta, p.lnc_gamma, p.lnc_beta) if ln else None for p in (self.fw, self.bw)]
        # both directions' projections in one [T, 2B, 4H] tensor (the backward
        # direction reads each sketch reversed within its length)
        xp = bilstm_input_proj(x, lengths, self.fw.W_x, self.bw.W_x, None if ln else self.fw.bias,
                               None if ln else self.bw.bias)
        # only h[len - 1] of each row is read: the persistent kernel may stop
        # each row block after its longest row (TF dynamic_rnn sequence_length)
        outs = ops.bilstm_sequence_packed(xp, self.fw.W_h, self.bw.W_h, zeros, zeros, drop_keep=keep,
                                          drop_seed=seed, drop_stream=_S_ENC_FW, ln_f=lns[0], ln_b=lns[1],
                                          lengths=lengths)
        idx = (lengths - 1).clamp(min=0).view(1, B, 1).expand(1, B, H)
        return torch.cat([torch.gather(o, 0, idx).squeeze(0) for o in outs], -1)


class SketchVAE(nn.Module):
    def __init__(self, cfg: VAEConfig, seed: Optional[int] = None):
        super().__init__()
        self.cfg = cfg
        gen = torch.Generator().manual_seed(cfg.seed if seed is None else seed)
        H = cfg.dec_rnn_size
        self.encoder = Encoder(cfg, gen) if cfg.conditional else None
        self.class_emb = None
        if cfg.num_classes > 0:
            self.class_emb = nn.Parameter(_gaussian((cfg.num_classes, cfg.z_size), 0.01, gen))
        z_in = cfg.z_size * (2 if (cfg.num_classes > 0 and cfg.class_embed == "concat") else 1)
        self.z_in = z_in if cfg.conditional or cfg.num_classes > 0 else 0
        in_size = 5 + self.z_in
        if cfg.dec_model == "lstm":
            self.dec = C.LSTMParams(in_size, H, gen=gen)
        elif cfg.dec_model == "layer_norm":
            self.dec = C.LNLSTMParams(in_size, H, gen=gen)
        elif cfg.dec_model == "hyper":
            self.dec = C.HyperLSTMParams(in_size, H, cfg.hyper_num_units, cfg.hyper_embedding_size,
                                         use_layer_norm=cfg.hyper_use_layer_norm, gen=gen)
        else:
            raise ValueError(cfg.dec_model)
        self.state_size = 2 * (H + (cfg.hyper_num_units if cfg.dec_model == "hyper" else 0))
        if self.z_in:
            self.init_w = nn.Parameter(_gaussian((self.z_in, self.state_size), 0.001, gen))
            self.init_b = nn.Parameter(torch.zeros(self.state_size))
        self.output_w = nn.Parameter(C.uniform_(torch.empty(H, cfg.n_out), gen))
        self.output_b = nn.Parameter(torch.zeros(cfg.n_out))

    # -- latent ---------------------------------------------------------------------
    def encode(self, strokes: torch.Tensor, lengths: torch.Tensor, train: bool = False, seed: int = 0):
        x = strokes[:, 1:].transpose(0, 1)
        return self.encoder(x, lengths, train, seed)

    def condition(self, z: Optional[torch.Tensor], labels: Optional[torch.Tensor], B: int, device):
        parts = []
        if z is not None:
            parts.append(z)
        if self.class_emb is not None and labels is not None:
            e = self.class_emb[labels]
            if self.cfg.class_embed == "concat" or z is None:
                parts.append(e)
            else:
                parts[0] = parts[0] + e
        if not parts:
            return None
        return torch.cat(parts, -1) if len(parts) > 1 else parts[0]

    def initial_state(self, zc: Optional[torch.Tensor], B: int, device):
        """Split ``tanh(zc @ W + b)`` into the decoder's state tensors."""
        H, Hh = self.cfg.dec_rnn_size, self.cfg.hyper_num_units
        if zc is None:
            s = torch.zeros(B, self.state_size, device=device)
        else:
            s = torch.tanh(zc @ self.init_w + self.init_b)
        m = self.cfg.dec_model
        if m == "lstm":          # LSTMCell state = [c, h]
            c, h = s.split(H, -1)
            return (h, c)
        if m == "layer_norm":    # LayerNormLSTMCell state = [h, c]
            h, c = s.split(H, -1)
            return (h, c)
        h, hh, c, hc = s.split([H, Hh, H, Hh], -1)  # HyperLSTM state = [h, hh, c, hc]
        return (h, c, hh, hc)

    # -- decoder ---------------------------------------------------------------------
    def decode(self, x: torch.Tensor, zc: Optional[torch.Tensor], state, train: bool, seed: int,
               out_dropout: bool = True):
        """``x [T, B, 5]`` time-major -> ``(outputs [T, B, H], final_state)``.
        ``out_dropout=False``: the caller applies the output dropout itself
        (the fused MDN head masks its input in-kernel)."""
        cfg = self.cfg
        T, B, _ = x.shape
        if train and cfg.use_input_dropout:   # the mask covers z too: no per-sequence factoring
            if zc is not None:
                x = torch.cat([x, zc.unsqueeze(0).expand(T, B, zc.shape[-1])], -1)
                zc = None
            x = x * C.dropout_mask(seed, _S_IN, 0, x.shape, cfg.input_dropout_prob, x.device)
        # otherwise z stays separate: its projection is computed once per sequence
        keep = cfg.recurrent_dropout_prob if (train and cfg.use_recurrent_dropout) else 1.0
        p = self.dec
        if cfg.dec_model == "hyper":
            h0, c0, hh0, hc0 = state
            hkeep = cfg.recurrent_dropout_prob if (train and cfg.hyper_use_recurrent_dropout) else 1.0
            out, final = ops.hyper_sequence(p, x, h0, c0, hh0, hc0, drop_keep=keep, drop_seed=seed,
                                            drop_stream=_S_DEC, hyp_drop_keep=hkeep, zc=zc)
        else:
            h0, c0 = state
            ln = (p.ln_gamma, p.ln_beta, p.lnc_gamma, p.lnc_beta) if cfg.dec_model == "layer_norm" else None
            xp = stroke_input_proj(x, zc, p.W_x, None if ln else p.bias)
            out, final = ops.lstm_sequence(xp, p.W_h, h0, c0, drop_keep=keep, drop_seed=seed,
                                           drop_stream=_S_DEC, ln=ln)
        if train and cfg.use_output_dropout and out_dropout:
            out = out * C.dropout_mask(seed, _S_OUT, 0, out.shape, cfg.output_dropout_prob, out.device)
        return out, final

    def head(self, out: torch.Tensor) -> torch.Tensor:
        return gemm.linear(out.reshape(-1, out.shape[-1]), self.output_w, self.output_b)

    # -- training objective -------------------------------------------------------------
    def loss(self, strokes: torch.Tensor, lengths: torch.Tensor, labels: Optional[torch.Tensor] = None,
             kl_weight: float = 1.0, train: bool = True, seed: int = 0,
             eps: Optional[torch.Tensor] = None, split_encoder: bool = False) -> Dict[str, torch.Tensor]:
        """``split_encoder``: cut the autograd graph at the encoder outputs;
        ``cost.backward()`` then stops there and the result carries
        ``"_enc": (enc, cut)`` so the caller runs the encoder's backward as a
        separate phase (``torch.autograd.backward(enc, [t.grad for t in cut])``).
        The cut point depends on the latent path:

        * fused latent layer (``ops/latent.py``, the GPU default): the cut is
          at the encoder summary ``last_h`` -- ``enc = (last_h,)``,
          ``cut = (last_h_detached,)``. The latent heads (``mu_w``, ``mu_b``,
          ``sig_w``, ``sig_b``) sit after the cut, so their gradients are
          produced in phase A even though the parameters belong to the
          encoder (the trainer's late arena part);
        * torch latent layer: the cut is at ``(mu, presig)``."""
        cfg = self.cfg
        B = strokes.shape[0]
        Nmax = strokes.shape[1] - 1
        dev = strokes.device
        # time-major stroke batch, transposed ONCE: the encoder input sT[1:],
        # the decoder input sT[:Nmax] and the targets are contiguous views
        # of it (each consumer copied its own transposed slice before)
        sT = strokes.transpose(0, 1).contiguous()
        z = None
        kl = strokes.new_zeros(())
        from ..ops import latent as L
        H, Hh = cfg.dec_rnn_size, cfg.hyper_num_units
        widths = {"hyper": (H, Hh, H, Hh), "lstm": (H, H), "layer_norm": (H, H)}[cfg.dec_model]
        # (eligibility from a parameter: no fp32 copy of the stroke batch per call)
        if cfg.conditional and self.class_emb is None and L.latent_ok(self.encoder.mu_w, len(widths)) and \
                LATENT_FUSED:
            # encoder summary -> (mu, presig, z, KL, decoder state) as one node (ops/latent.py)
            last_h = self.encoder.last_hidden(sT[1:], lengths, train, seed)
            if split_encoder:
                enc = (last_h,)
                last_h = last_h.detach().requires_grad_()
                enc_cut = (enc, (last_h,))
            from ..ops.recurrent import _seed_tensor
            mu, presig, z, kl, *segs = L.latent(last_h, self.encoder.mu_w, self.encoder.mu_b, self.encoder.sig_w,
                                                self.encoder.sig_b, self.init_w, self.init_b,
                                                _seed_tensor(seed, dev), widths, cfg.kl_tolerance, _S_EPS, eps=eps)
            # segment order = the state layout of initial_state: hyper [h, hh, c, hc] -> (h, c, hh, hc);
            # LSTMCell [c, h] -> (h, c); LayerNormLSTMCell [h, c]
            state = {"hyper": lambda q: (q[0], q[2], q[1], q[3]), "lstm": lambda q: (q[1], q[0]),
                     "layer_norm": lambda q: (q[0], q[1])}[cfg.dec_model](segs)
            zc = z
        elif cfg.conditional:
            mu, presig = self.encoder(sT[1:], lengths, train, seed)
            if split_encoder:
                enc = (mu, presig)
                mu, presig = mu.detach().requires_grad_(), presig.detach().requires_grad_()
                enc_cut = (enc, (mu, presig))
            sigma = torch.exp(presig / 2.0)
            if eps is None:
                eps = C.hash_normal(seed, _S_EPS, 0, (B, cfg.z_size), dev)
            z = mu + sigma * eps
            kl_raw = -0.5 * torch.mean(1 + presig - mu * mu - torch.exp(presig))
            kl = torch.clamp(kl_raw, min=cfg.kl_tolerance)
            zc = self.condition(z, labels, B, dev)
            state = self.initial_state(zc, B, dev)
        else:
            zc = self.condition(z, labels, B, dev)
            state = self.initial_state(zc, B, dev)
        x_in = sT[:Nmax]
        out, _ = self.decode(x_in, zc, state, train, seed, out_dropout=False)
        target = sT[1:].reshape(-1, 5)
        # head + loss (fused on the GPU: projection, MDN loss and dL/dz in one kernel)
        keep = cfg.output_dropout_prob if (train and cfg.use_output_dropout) else 1.0
        r_cost, shape, pen = ops.mdn_head_loss(out.reshape(-1, out.shape[-1]), self.output_w, self.output_b, target,
                                               cfg.num_mixture, mode="magenta", is_training=cfg.is_training,
                                               drop_keep=keep, drop_seed=seed, drop_stream=_S_OUT,
                                               x_lp=getattr(out, "_skr_lp", None))
        cost = r_cost + kl * kl_weight
        out = {"cost": cost, "r_cost": r_cost, "kl_cost": kl, "shape_cost": shape, "pen_cost": pen}
        if split_encoder and cfg.conditional:
            out["_enc"] = enc_cut
        return out

    # -- sampling helpers --------------------------------------------------------------------
    @torch.no_grad()
    def decode_step(self, x: torch.Tensor, zc: Optional[torch.Tensor], state):
        """One decoder step: ``x [B, 5]`` -> ``(z_head [B, NOUT], new_state)``."""
        out, final = self.decode(x.unsqueeze(0), zc, state, train=False, seed=0)
        return self.head(out), final
