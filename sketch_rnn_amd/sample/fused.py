"""Fused whole-sketch decoder for the reference model (``csrc/decode_ref.hip``).

The reference samples one stroke per ``sess.run`` (``model.py:187-264``:
two host transfers per stroke, ~486 strokes/s here). :class:`GraphDecoder`
removes the host from the loop but still replays a chain of kernels per
stroke (step GEMMs, cells, head, sampler). :class:`FusedRefDecoder` runs
the whole decode -- both LSTM layers, the MDN head and the sampler, every
step -- as ONE kernel launch per batch: weights stay in LDS, the cell state
in registers, and strokes travel between the workgroups through in-launch
hand-offs.

Semantics are those of ``GraphDecoder`` in reference mode (identical hash
random numbers, the reference's pen-temperature bug unless
``fix_pen_temperature``, per-step eoc state hold, end-of-sketch padding of
finished rows), with bf16 MFMA operands and fp32 state. Eligible models:
``lstm`` cells, ``rnn_size`` 256, 1 or 2 layers, at most 32 mixtures
(:func:`fused_decode_ok`); anything else keeps using ``GraphDecoder``.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import torch

from ..utils import native

_H = 256
_FLAG_STRIDE = 64
_XLD = 8


def fused_decode_ok(model) -> bool:
    cfg = model.cfg
    return (getattr(cfg, "kind", "") == "reference" and cfg.model == "lstm" and cfg.rnn_size == _H
            and cfg.num_layers in (1, 2) and 1 <= cfg.num_mixture <= 32)


class NotCoResident(RuntimeError):
    """The launch's workgroups cannot all be resident at once on this device
    (``skr_decode_ref`` returned -8); callers fall back to ``GraphDecoder``."""


def _chunk_rows(L: int, mtw: int, cus: int = 256) -> int:
    """Rows one launch can take: every workgroup must be co-resident (one
    ~100 KB-LDS workgroup per CU, ``cus`` CUs -- 256 on MI355X; L*16 + 1
    workgroups per row block)."""
    return (cus // (L * (_H // 16) + 1)) * 16 * mtw


class FusedRefDecoder:
    """B sketches of N strokes from a reference :class:`SketchRNN` in one launch
    per chunk of rows. ``run()`` returns ``(strokes [B, N, 5], lengths [B])``
    like :meth:`GraphDecoder.run` (offsets multiplied by ``data_scale``)."""

    def __init__(self, model, batch: int, steps: int, temperature: float = 1.0, greedy: bool = False,
                 fix_pen_temperature: bool = False):
        if not fused_decode_ok(model):
            raise ValueError("FusedRefDecoder: needs a reference lstm model with rnn_size 256, 1-2 layers, M <= 32")
        self.lib = native.require_hip()
        self.model = model
        self.B, self.N = int(batch), int(steps)
        self.temp, self.greedy, self.fix_pen = float(temperature), bool(greedy), bool(fix_pen_temperature)
        cfg = model.cfg
        self.L, self.M = cfg.num_layers, cfg.num_mixture
        self.nout = 3 + 6 * self.M
        self.noutp = -(-self.nout // 16) * 16
        self.dev = next(model.parameters()).device
        self.mtw = 1 if self.B <= 16 else 2
        cus = torch.cuda.get_device_properties(self.dev).multi_processor_count if self.dev.type == "cuda" else 256
        self.rows = _chunk_rows(self.L, self.mtw, cus)
        if self.rows <= 0:
            raise NotCoResident("FusedRefDecoder: %d CUs cannot hold one row block (%d workgroups)"
                                % (cus, self.L * (_H // 16) + 1))
        self.seed = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self._w = None
        self._sig = None

    # -- weights (bf16 operands, refreshed when the parameters change) -------------------
    @torch.no_grad()
    def _weights(self):
        sig = tuple(p._version for p in self.model.parameters()) + tuple(p.data_ptr() for p in self.model.parameters())
        if self._w is not None and sig == self._sig:
            return self._w
        m, bf = self.model, torch.bfloat16
        p0 = m.layers[0]
        w = {
            "WT0": p0.W_h.detach().t().to(bf).contiguous(),                      # [4H, H]
            "Wx0": p0.W_x.detach().float().contiguous(),                         # [5, 4H]
            "b0": p0.bias.detach().float().contiguous(),
            "bo": m.output_b.detach().float().contiguous(),
        }
        if self.L == 2:
            p1 = m.layers[1]
            w["WT1"] = torch.cat([p1.W_x.detach(), p1.W_h.detach()], 0).t().to(bf).contiguous()   # [4H, 2H]
            w["b1"] = p1.bias.detach().float().contiguous()
        WoT = torch.zeros(self.noutp, _H, dtype=bf, device=self.dev)
        WoT[: self.nout] = m.output_w.detach().t().to(bf)
        w["WoT"] = WoT
        self._w, self._sig = w, sig
        return w

    def _launch(self, r0: int, Bc: int, xin: torch.Tensor, forced: bool, zout: Optional[torch.Tensor]):
        from ..ops._hipapi import DecArgs
        from ..ops.recurrent import cluster_error_flag
        w = self._weights()
        N, L, dev, bf, f32 = self.N, self.L, self.dev, torch.bfloat16, torch.float32
        RB = 16 * self.mtw
        nrb = -(-Bc // RB)
        a = DecArgs()
        a.N, a.B, a.L, a.H, a.mtw, a.nrb = N, Bc, L, _H, self.mtw, nrb
        a.M, a.nout, a.noutp, a.mode = self.M, self.nout, self.noutp, 0
        a.greedy, a.fix_pen, a.forced, a.row0 = int(self.greedy), int(self.fix_pen), int(forced), int(r0)
        a.temp, a.forget_bias = self.temp, 1.0
        keep = []
        for l in range(L):
            ly = a.ly[l]
            z = torch.zeros(Bc, _H, dtype=f32, device=dev)          # reference sampling starts from the zero state
            hbuf = torch.empty(N + 1, Bc, _H, dtype=bf, device=dev)
            hbuf[0].zero_()
            hup = torch.empty(N, Bc, _H, dtype=bf, device=dev)
            ly.WT = w["WT0" if l == 0 else "WT1"].data_ptr()
            ly.bias = w["b0" if l == 0 else "b1"].data_ptr()
            ly.h0, ly.c0, ly.hbuf, ly.hup = z.data_ptr(), z.data_ptr(), hbuf.data_ptr(), hup.data_ptr()
            ly.hT = ly.cT = None
            keep += [z, hbuf, hup]
        out = torch.empty(Bc, N, 5, dtype=f32, device=dev)
        done = torch.zeros(Bc, dtype=torch.int32, device=dev)
        flags = torch.empty(nrb * _FLAG_STRIDE, dtype=torch.int32, device=dev)   # zeroed by the launcher
        a.Wx0, a.WoT, a.bo = w["Wx0"].data_ptr(), w["WoT"].data_ptr(), w["bo"].data_ptr()
        a.xin, a.out, a.done = xin.data_ptr(), out.data_ptr(), done.data_ptr()
        a.zout = zout.data_ptr() if zout is not None else None
        a.seed, a.flags, a.err = self.seed.data_ptr(), flags.data_ptr(), cluster_error_flag(dev).data_ptr()
        rc = self.lib.lib.skr_decode_ref(ctypes.byref(a), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        if rc == -8:
            raise NotCoResident("skr_decode_ref: workgroups cannot be co-resident on this device (code -8)")
        if rc != 0:
            raise RuntimeError("skr_decode_ref: launch failed (code %d)" % rc)
        keep += [flags, done]
        return out, keep

    @torch.no_grad()
    def run(self, seed: int = 0, return_z: bool = False):
        """Returns ``(strokes, lengths)`` (plus the head outputs ``z [N, B, 3+6M]``
        with ``return_z``)."""
        from ..ops.recurrent import check_cluster_errors
        self.seed.fill_(int(seed))
        outs, zs, keep = [], [], []
        for r0 in range(0, self.B, self.rows):
            Bc = min(self.rows, self.B - r0)
            xin = torch.zeros(self.N + 1, Bc, _XLD, device=self.dev)        # x(0) = 0 (model.py:200)
            zout = torch.empty(self.N, Bc, self.nout, device=self.dev) if return_z else None
            o, k = self._launch(r0, Bc, xin, False, zout)
            outs.append(o)
            zs.append(zout)
            keep += k + [xin]
        strokes = torch.cat(outs, 0)
        check_cluster_errors(self.dev)
        hits = strokes[:, :, 3] > 0
        lengths = torch.where(hits.any(1), hits.float().argmax(1) + 1,
                              torch.full_like(hits[:, 0], self.N, dtype=torch.long))
        strokes[:, :, 0:2] *= self.model.cfg.data_scale
        if return_z:
            return strokes, lengths, torch.cat(zs, 1)
        return strokes, lengths

    @torch.no_grad()
    def forced(self, xs: torch.Tensor) -> torch.Tensor:
        """Teacher-forced decode: ``xs [N, B, 5]`` fed inputs -> head outputs
        ``z [N, B, 3+6M]`` (the kernel's numerics against the step oracle)."""
        from ..ops.recurrent import check_cluster_errors
        N, B = xs.shape[0], xs.shape[1]
        assert N == self.N and B == self.B
        zs, keep = [], []
        for r0 in range(0, B, self.rows):
            Bc = min(self.rows, B - r0)
            xin = torch.zeros(N + 1, Bc, _XLD, device=self.dev)
            xin[:N, :, :5] = xs[:, r0:r0 + Bc].to(self.dev, torch.float32)
            zout = torch.empty(N, Bc, self.nout, device=self.dev)
            _, k = self._launch(r0, Bc, xin, True, zout)
            zs.append(zout)
            keep += k + [xin]
        z = torch.cat(zs, 1)
        check_cluster_errors(self.dev)
        return z
