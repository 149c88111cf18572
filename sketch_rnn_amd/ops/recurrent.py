"""Native recurrences on the GPU: per-step library GEMM + fused HIP cell kernel.

Step ``t`` of a layer is two launches: ``R = h_{t-1} @ W_h`` (hipBLASLt,
bf16/fp32 operands, fp32 out) and one fused cell kernel
(``csrc/lstm_cell.hip``) that adds the hoisted input projection, applies
LayerNorm / hyper modulation / gates / dropout / eoc reset and writes the
next GEMM's operand directly. The backward runs the mirror image in reverse
and leaves all weight gradients to single large GEMMs over the whole
sequence after the scan. Launched from Python but designed to be captured
whole into a HIP graph (no allocation depends on data, no host sync).

Autograd boundaries are whole sequences (one ``Function`` per layer), so
no per-step autograd nodes exist.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from ..utils import native
from . import gemm
from ._hipapi import LstmBwdArgs, LstmFwdArgs

_NULL = None


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError("%s: launch failed (code %d)" % (what, rc))


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _seed_tensor(seed, device) -> torch.Tensor:
    if torch.is_tensor(seed):
        return seed.to(device=device, dtype=torch.int64).reshape(1)
    return torch.tensor([int(seed)], dtype=torch.int64, device=device)


def _lp_kind(t: torch.Tensor) -> int:
    return 1 if t.dtype == torch.bfloat16 else 2


class _Saved:
    """Plain holder for the big per-sequence buffers (kept off autograd)."""


# =====================================================================================
# LSTM / LayerNorm-LSTM sequence
# =====================================================================================
class _LSTMSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xp, W_h, h0, c0, reset_h, reset_c, ln_g, ln_b, lnc_g, lnc_b, reset, seed, meta):
        forget_bias, keep, stream = meta
        lib = native.require_hip()
        T, B, G = xp.shape
        H = G // 4
        dev = xp.device
        f32 = torch.float32
        ln = ln_g is not None
        xp = xp.contiguous()
        Wl = gemm.lp(W_h).contiguous()
        ldt = Wl.dtype
        A = torch.empty(T + 1, B, H, device=dev, dtype=ldt)   # GEMM operands: carried h
        A[0].copy_(h0)
        CC = torch.empty(T + 1, B, H, device=dev, dtype=f32)  # carried c
        CC[0].copy_(c0)
        Hout = torch.empty(T, B, H, device=dev, dtype=f32)
        Cout = torch.empty(T, B, H, device=dev, dtype=f32)
        ACT = torch.empty(T, B, 4 * H, device=dev, dtype=f32)
        XHAT = torch.empty(T, B, 4 * H, device=dev, dtype=f32) if ln else None
        RSTD = torch.empty(T, B, 5, device=dev, dtype=f32) if ln else None
        CHAT = torch.empty(T, B, H, device=dev, dtype=f32) if ln else None
        HC = torch.empty(2, B, H, device=dev, dtype=f32)
        R = torch.empty(B, 4 * H, device=dev, dtype=f32)
        rst = reset.contiguous().to(f32) if reset is not None else None
        rh = reset_h.contiguous() if reset_h is not None else None
        rc = reset_c.contiguous() if reset_c is not None else None
        sd = _seed_tensor(seed, dev)
        a = LstmFwdArgs()
        a.B, a.H = B, H
        a.ld_xp, a.ld_R = 4 * H, 4 * H
        a.vec, a.vec_gs, a.bias = None, 0, None
        a.ln_g, a.ln_b, a.lnc_g, a.lnc_b = _ptr(ln_g), _ptr(ln_b), _ptr(lnc_g), _ptr(lnc_b)
        a.init_h, a.init_c = _ptr(rh), _ptr(rc)
        a.forget_bias, a.keep = float(forget_bias), float(keep)
        a.seed, a.stream = sd.data_ptr(), int(stream)
        a.ld_lp, a.lp_kind = H, _lp_kind(A)
        a.R = R.data_ptr()
        st = _stream()
        for t in range(T):
            gemm.mm(A[t], Wl, out=R)
            a.xp = xp[t].data_ptr()
            a.c_prev = CC[t].data_ptr()
            a.reset = _ptr(rst[t]) if rst is not None else None
            a.step = t
            a.h_out, a.c_out, a.act = Hout[t].data_ptr(), Cout[t].data_ptr(), ACT[t].data_ptr()
            if ln:
                a.xhat, a.rstd, a.chat = XHAT[t].data_ptr(), RSTD[t].data_ptr(), CHAT[t].data_ptr()
            a.h_carry = HC[t % 2].data_ptr()
            a.h_lp = A[t + 1].data_ptr()
            a.c_carry = CC[t + 1].data_ptr()
            _check(lib.lib.skr_lstm_fwd_step(ctypes.byref(a), int(ln), 0, st), "lstm_fwd_step")
        hT = HC[(T - 1) % 2].clone() if T > 0 else h0.clone()
        cT = CC[T].clone()
        s = _Saved()
        s.Wl, s.A, s.CC, s.Cout, s.ACT, s.XHAT, s.RSTD, s.CHAT = Wl, A, CC, Cout, ACT, XHAT, RSTD, CHAT
        s.reset, s.seed, s.meta = rst, sd, meta
        s.ln_g, s.lnc_g, s.lnc_b = ln_g, lnc_g, lnc_b
        s.has_reset_state = reset_h is not None
        ctx.s = s
        ctx.dims = (T, B, H)
        return Hout, hT, cT

    @staticmethod
    def backward(ctx, dHout, dhT, dcT):
        s = ctx.s
        T, B, H = ctx.dims
        forget_bias, keep, stream = s.meta
        lib = native.require_hip()
        dev = s.A.device
        f32 = torch.float32
        ln = s.ln_g is not None
        dG = torch.empty(T, B, 4 * H, device=dev, dtype=f32)
        lp_on = s.Wl.dtype == torch.bfloat16
        dG_lp = torch.empty(T, B, 4 * H, device=dev, dtype=torch.bfloat16) if lp_on else None
        dh_rec = dhT.contiguous().clone() if dhT is not None else torch.zeros(B, H, device=dev, dtype=f32)
        dc_rec = dcT.contiguous().clone() if dcT is not None else torch.zeros(B, H, device=dev, dtype=f32)
        dHout = dHout.contiguous() if dHout is not None else None
        dinit_h = torch.zeros(B, H, device=dev, dtype=f32) if s.reset is not None else None
        dinit_c = torch.zeros(B, H, device=dev, dtype=f32) if s.reset is not None else None
        DLNY = torch.empty(T, B, 4 * H, device=dev, dtype=f32) if ln else None
        DLNCY = torch.empty(T, B, H, device=dev, dtype=f32) if ln else None
        WT = s.Wl.t()
        a = LstmBwdArgs()
        a.B, a.H = B, H
        a.ld_dh_rec = H
        a.dh_rec, a.dc_rec = dh_rec.data_ptr(), dc_rec.data_ptr()
        a.ln_g, a.lnc_g, a.lnc_b = _ptr(s.ln_g), _ptr(s.lnc_g), _ptr(s.lnc_b)
        a.keep, a.seed, a.stream = float(keep), s.seed.data_ptr(), int(stream)
        a.ld_dG, a.ld_dG_lp, a.dG_lp_kind = 4 * H, 4 * H, 1 if lp_on else 0
        a.dinit_h, a.dinit_c = _ptr(dinit_h), _ptr(dinit_c)
        st = _stream()
        for t in range(T - 1, -1, -1):
            a.dh_out = dHout[t].data_ptr() if dHout is not None else None
            a.act, a.c_new, a.c_prev = s.ACT[t].data_ptr(), s.Cout[t].data_ptr(), s.CC[t].data_ptr()
            if ln:
                a.xhat, a.rstd, a.chat = s.XHAT[t].data_ptr(), s.RSTD[t].data_ptr(), s.CHAT[t].data_ptr()
                a.dlny, a.dlncy = DLNY[t].data_ptr(), DLNCY[t].data_ptr()
            a.reset = _ptr(s.reset[t]) if s.reset is not None else None
            a.step = t
            a.dG = dG[t].data_ptr()
            a.dG_lp = dG_lp[t].data_ptr() if lp_on else None
            _check(lib.lib.skr_lstm_bwd_step(ctypes.byref(a), int(ln), 0, st), "lstm_bwd_step")
            gemm.mm(dG_lp[t] if lp_on else dG[t], WT, out=dh_rec)
        dGm = (dG_lp if lp_on else dG).view(T * B, 4 * H)
        dW = gemm.mm(s.A[:T].reshape(T * B, H).t(), dGm)
        g_ln = [None] * 4
        if ln:
            xh = s.XHAT.view(T * B, 4 * H)
            dl = DLNY.view(T * B, 4 * H)
            g_ln = [(dl * xh).sum(0), dl.sum(0),
                    (DLNCY.view(T * B, H) * s.CHAT.view(T * B, H)).sum(0), DLNCY.view(T * B, H).sum(0)]
        dh0, dc0 = dh_rec, dc_rec
        ctx.s = None
        return (dG, dW, dh0, dc0, dinit_h, dinit_c, g_ln[0], g_ln[1], g_ln[2], g_ln[3], None, None, None)


def lstm_sequence_hip(xp, W_h, h0, c0, forget_bias=1.0, reset=None, reset_h=None, reset_c=None,
                      drop_keep=1.0, drop_seed=0, drop_stream=0, ln=None):
    if ln is None:
        ln = (None, None, None, None)
    if reset is not None and reset_h is None:
        raise ValueError("reset requires reset_h / reset_c")
    Hout, hT, cT = _LSTMSeq.apply(xp, W_h, h0, c0, reset_h, reset_c, *ln, reset, drop_seed,
                                  (float(forget_bias), float(drop_keep), int(drop_stream)))
    return Hout, (hT, cT)


# =====================================================================================
# HyperLSTM sequence
# =====================================================================================
class _HyperSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, h0, c0, hh0, hc0, seed, W_x, W_h, bias, hW_x, hW_h, hln_g, hln_b, hlnc_g, hlnc_b,
                W_z, b_z, W_a, ln_g, ln_b, lnc_g, lnc_b, meta):
        forget_bias, keep, hkeep, stream, E = meta
        lib = native.require_hip()
        T, B, IN = x.shape
        H, Hh = W_h.shape[0], hW_h.shape[0]
        G, Gh = 4 * H, 4 * Hh
        K, N = H + Hh, G + Gh
        dev = x.device
        f32 = torch.float32
        x2 = x.reshape(T * B, IN).contiguous()
        xl = gemm.lp(x2)
        XH = gemm.mm(xl, gemm.lp(W_x)).view(T, B, G)
        XHY = gemm.mm(xl, gemm.lp(hW_x[:IN])).view(T, B, Gh)
        dt = gemm.lp_dtype()
        Wcat = torch.zeros(K, N, device=dev, dtype=dt)
        Wcat[:H, :G].copy_(W_h)
        Wcat[:H, G:].copy_(hW_x[IN:])
        Wcat[H:, G:].copy_(hW_h)
        A = torch.empty(T + 1, B, K, device=dev, dtype=dt)
        A[0, :, :H].copy_(h0)
        A[0, :, H:].copy_(hh0)
        RC = torch.empty(T, B, N, device=dev, dtype=f32)
        CC = torch.empty(T + 1, B, H, device=dev, dtype=f32)
        CC[0].copy_(c0)
        HCC = torch.empty(T + 1, B, Hh, device=dev, dtype=f32)
        HCC[0].copy_(hc0)
        Hout = torch.empty(T, B, H, device=dev, dtype=f32)
        Cout = torch.empty(T, B, H, device=dev, dtype=f32)
        ACT = torch.empty(T, B, G, device=dev, dtype=f32)
        XHAT = torch.empty(T, B, G, device=dev, dtype=f32)
        RSTD = torch.empty(T, B, 5, device=dev, dtype=f32)
        CHAT = torch.empty(T, B, H, device=dev, dtype=f32)
        HH = torch.empty(T, B, Hh, device=dev, dtype=f32)
        HCout = torch.empty(T, B, Hh, device=dev, dtype=f32)
        HACT = torch.empty(T, B, Gh, device=dev, dtype=f32)
        HXHAT = torch.empty(T, B, Gh, device=dev, dtype=f32)
        HRSTD = torch.empty(T, B, 5, device=dev, dtype=f32)
        HCHAT = torch.empty(T, B, Hh, device=dev, dtype=f32)
        ZS = torch.empty(T, B, 12 * E, device=dev, dtype=f32)
        VEC = torch.empty(T, 12, B, H, device=dev, dtype=f32)
        HC = torch.empty(2, B, H, device=dev, dtype=f32)
        HHC = torch.empty(2, B, Hh, device=dev, dtype=f32)
        sd = _seed_tensor(seed, dev)
        # hyper cell args (LN-LSTM, no modulation)
        ah = LstmFwdArgs()
        ah.B, ah.H = B, Hh
        ah.ld_xp, ah.ld_R = Gh, N
        ah.ln_g, ah.ln_b, ah.lnc_g, ah.lnc_b = hln_g.data_ptr(), hln_b.data_ptr(), hlnc_g.data_ptr(), hlnc_b.data_ptr()
        ah.forget_bias, ah.keep = float(forget_bias), float(hkeep)
        ah.seed, ah.stream = sd.data_ptr(), int(stream) + 1
        ah.ld_lp, ah.lp_kind = K, _lp_kind(A)
        # main cell args (LN + modulation)
        am = LstmFwdArgs()
        am.B, am.H = B, H
        am.ld_xp, am.ld_R = G, N
        am.vec_gs, am.bias = B * H, bias.data_ptr()
        am.ln_g, am.ln_b, am.lnc_g, am.lnc_b = ln_g.data_ptr(), ln_b.data_ptr(), lnc_g.data_ptr(), lnc_b.data_ptr()
        am.forget_bias, am.keep = float(forget_bias), float(keep)
        am.seed, am.stream = sd.data_ptr(), int(stream)
        am.ld_lp, am.lp_kind = K, _lp_kind(A)
        Wz = W_z.contiguous()
        Wa = W_a.contiguous()
        st = _stream()
        for t in range(T):
            gemm.mm(A[t], Wcat, out=RC[t])
            ah.xp, ah.R = XHY[t].data_ptr(), RC[t, :, G:].data_ptr()
            ah.c_prev, ah.step = HCC[t].data_ptr(), t
            ah.h_out, ah.c_out, ah.act = HH[t].data_ptr(), HCout[t].data_ptr(), HACT[t].data_ptr()
            ah.xhat, ah.rstd, ah.chat = HXHAT[t].data_ptr(), HRSTD[t].data_ptr(), HCHAT[t].data_ptr()
            ah.h_carry, ah.h_lp, ah.c_carry = HHC[t % 2].data_ptr(), A[t + 1, :, H:].data_ptr(), HCC[t + 1].data_ptr()
            _check(lib.lib.skr_lstm_fwd_step(ctypes.byref(ah), 1, 0, st), "hyper_fwd_step")
            torch.addmm(b_z, HH[t], Wz, out=ZS[t])
            torch.bmm(ZS[t].view(B, 12, E).transpose(0, 1), Wa, out=VEC[t])
            am.xp, am.R, am.vec = XH[t].data_ptr(), RC[t, :, :G].data_ptr(), VEC[t].data_ptr()
            am.c_prev, am.step = CC[t].data_ptr(), t
            am.h_out, am.c_out, am.act = Hout[t].data_ptr(), Cout[t].data_ptr(), ACT[t].data_ptr()
            am.xhat, am.rstd, am.chat = XHAT[t].data_ptr(), RSTD[t].data_ptr(), CHAT[t].data_ptr()
            am.h_carry, am.h_lp, am.c_carry = HC[t % 2].data_ptr(), A[t + 1, :, :H].data_ptr(), CC[t + 1].data_ptr()
            _check(lib.lib.skr_lstm_fwd_step(ctypes.byref(am), 1, 1, st), "hyper_main_fwd_step")
        hT = HC[(T - 1) % 2].clone()
        hhT = HHC[(T - 1) % 2].clone()
        s = _Saved()
        for k, v in dict(xl=xl, XH=XH, Wcat=Wcat, A=A, RC=RC, CC=CC, HCC=HCC, Cout=Cout, ACT=ACT, XHAT=XHAT,
                         RSTD=RSTD, CHAT=CHAT, HH=HH, HCout=HCout, HACT=HACT, HXHAT=HXHAT, HRSTD=HRSTD,
                         HCHAT=HCHAT, ZS=ZS, VEC=VEC, seed=sd, meta=meta, W_x=W_x, hW_x=hW_x, Wz=Wz, Wa=Wa,
                         ln_g=ln_g, lnc_g=lnc_g, lnc_b=lnc_b, hln_g=hln_g, hlnc_g=hlnc_g, hlnc_b=hlnc_b).items():
            setattr(s, k, v)
        ctx.s = s
        ctx.dims = (T, B, IN, H, Hh, E)
        return Hout, hT, CC[T].clone(), hhT, HCC[T].clone()

    @staticmethod
    def backward(ctx, dHout, dhT, dcT, dhhT, dhcT):
        s = ctx.s
        T, B, IN, H, Hh, E = ctx.dims
        forget_bias, keep, hkeep, stream, _ = s.meta
        lib = native.require_hip()
        dev = s.A.device
        f32 = torch.float32
        G, Gh = 4 * H, 4 * Hh
        K, N = H + Hh, G + Gh
        lp_on = s.Wcat.dtype == torch.bfloat16
        dRC = torch.empty(T, B, N, device=dev, dtype=f32)
        dRC_lp = torch.empty(T, B, N, device=dev, dtype=torch.bfloat16) if lp_on else None
        dXH = torch.empty(T, B, G, device=dev, dtype=f32)
        DLNY = torch.empty(T, B, G, device=dev, dtype=f32)
        DLNCY = torch.empty(T, B, H, device=dev, dtype=f32)
        HDLNY = torch.empty(T, B, Gh, device=dev, dtype=f32)
        HDLNCY = torch.empty(T, B, Hh, device=dev, dtype=f32)
        dZS = torch.empty(T, B, 12 * E, device=dev, dtype=f32)
        dvec = torch.empty(12, B, H, device=dev, dtype=f32)
        dzs12 = torch.empty(12, B, E, device=dev, dtype=f32)
        dWa = torch.zeros(12, E, H, device=dev, dtype=f32)
        dbias = torch.zeros(4, H, device=dev, dtype=f32)
        dhh_z = torch.empty(B, Hh, device=dev, dtype=f32)
        dA = torch.zeros(B, K, device=dev, dtype=f32)
        if dhT is not None:
            dA[:, :H].copy_(dhT)
        if dhhT is not None:
            dA[:, H:].copy_(dhhT)
        dc_rec = dcT.contiguous().clone() if dcT is not None else torch.zeros(B, H, device=dev, dtype=f32)
        dhc_rec = dhcT.contiguous().clone() if dhcT is not None else torch.zeros(B, Hh, device=dev, dtype=f32)
        dHout = dHout.contiguous() if dHout is not None else None
        WcT = s.Wcat.t()
        WzT = s.Wz.t()
        WaT = s.Wa.transpose(1, 2)
        am = LstmBwdArgs()
        am.B, am.H = B, H
        am.dh_rec, am.ld_dh_rec, am.dc_rec = dA.data_ptr(), K, dc_rec.data_ptr()
        am.ln_g, am.lnc_g, am.lnc_b = s.ln_g.data_ptr(), s.lnc_g.data_ptr(), s.lnc_b.data_ptr()
        am.ld_xp, am.ld_R, am.vec_gs = G, N, B * H
        am.keep, am.seed, am.stream = float(keep), s.seed.data_ptr(), int(stream)
        am.ld_dG, am.ld_dG_lp, am.dG_lp_kind = N, N, 1 if lp_on else 0
        am.ld_dxp, am.dvec = G, dvec.data_ptr()
        ah = LstmBwdArgs()
        ah.B, ah.H = B, Hh
        ah.dh_out = dhh_z.data_ptr()
        ah.dh_rec, ah.ld_dh_rec, ah.dc_rec = dA[:, H:].data_ptr(), K, dhc_rec.data_ptr()
        ah.ln_g, ah.lnc_g, ah.lnc_b = s.hln_g.data_ptr(), s.hlnc_g.data_ptr(), s.hlnc_b.data_ptr()
        ah.keep, ah.seed, ah.stream = float(hkeep), s.seed.data_ptr(), int(stream) + 1
        ah.ld_dG, ah.ld_dG_lp, ah.dG_lp_kind = N, N, 1 if lp_on else 0
        st = _stream()
        for t in range(T - 1, -1, -1):
            am.dh_out = dHout[t].data_ptr() if dHout is not None else None
            am.act, am.c_new, am.c_prev = s.ACT[t].data_ptr(), s.Cout[t].data_ptr(), s.CC[t].data_ptr()
            am.xhat, am.rstd, am.chat = s.XHAT[t].data_ptr(), s.RSTD[t].data_ptr(), s.CHAT[t].data_ptr()
            am.xp, am.R, am.vec = s.XH[t].data_ptr(), s.RC[t, :, :G].data_ptr(), s.VEC[t].data_ptr()
            am.step = t
            am.dG = dRC[t, :, :G].data_ptr()
            am.dG_lp = dRC_lp[t, :, :G].data_ptr() if lp_on else None
            am.dxp = dXH[t].data_ptr()
            am.dlny, am.dlncy = DLNY[t].data_ptr(), DLNCY[t].data_ptr()
            _check(lib.lib.skr_lstm_bwd_step(ctypes.byref(am), 1, 1, st), "hyper_main_bwd_step")
            # hyper-norm projections: vec = zs @ W_a (per block)
            torch.bmm(dvec, WaT, out=dzs12)
            dWa.baddbmm_(s.ZS[t].view(B, 12, E).permute(1, 2, 0), dvec)
            dbias.add_(dvec[8:12].sum(1))
            dZS[t].view(B, 12, E).copy_(dzs12.transpose(0, 1))
            torch.mm(dZS[t], WzT, out=dhh_z)
            ah.act, ah.c_new, ah.c_prev = s.HACT[t].data_ptr(), s.HCout[t].data_ptr(), s.HCC[t].data_ptr()
            ah.xhat, ah.rstd, ah.chat = s.HXHAT[t].data_ptr(), s.HRSTD[t].data_ptr(), s.HCHAT[t].data_ptr()
            ah.step = t
            ah.dG = dRC[t, :, G:].data_ptr()
            ah.dG_lp = dRC_lp[t, :, G:].data_ptr() if lp_on else None
            ah.dlny, ah.dlncy = HDLNY[t].data_ptr(), HDLNCY[t].data_ptr()
            _check(lib.lib.skr_lstm_bwd_step(ctypes.byref(ah), 1, 0, st), "hyper_bwd_step")
            gemm.mm(dRC_lp[t] if lp_on else dRC[t], WcT, out=dA)
        TB = T * B
        dRCm = (dRC_lp if lp_on else dRC).view(TB, N)
        dWcat = gemm.mm(s.A[:T].reshape(TB, K).t(), dRCm)
        dW_h = dWcat[:H, :G]
        dhW_x = torch.empty_like(s.hW_x)
        dhW_x[IN:] = dWcat[:H, G:]
        dhW_h = dWcat[H:, G:]
        dXHY = dRC[:, :, G:].reshape(TB, Gh)
        dXHm = dXH.view(TB, G)
        dXHl, dXHYl = gemm.lp(dXHm), gemm.lp(dXHY)
        dW_x = gemm.mm(s.xl.t(), dXHl)
        dhW_x[:IN] = gemm.mm(s.xl.t(), dXHYl)
        dx = gemm.mm(dXHl, gemm.lp(s.W_x).t())
        dx += gemm.mm(dXHYl, gemm.lp(s.hW_x[:IN]).t())
        dZSm = dZS.view(TB, 12 * E)
        dW_z = s.HH.view(TB, Hh).t() @ dZSm
        db_z = dZSm.sum(0)
        xh, dl = s.XHAT.view(TB, G), DLNY.view(TB, G)
        g_ln = ((dl * xh).sum(0), dl.sum(0), (DLNCY.view(TB, H) * s.CHAT.view(TB, H)).sum(0),
                DLNCY.view(TB, H).sum(0))
        hxh, hdl = s.HXHAT.view(TB, Gh), HDLNY.view(TB, Gh)
        g_hln = ((hdl * hxh).sum(0), hdl.sum(0), (HDLNCY.view(TB, Hh) * s.HCHAT.view(TB, Hh)).sum(0),
                 HDLNCY.view(TB, Hh).sum(0))
        dh0, dhh0 = dA[:, :H].contiguous(), dA[:, H:].contiguous()
        ctx.s = None
        return (dx.view(T, B, IN), dh0, dc_rec, dhh0, dhc_rec, None, dW_x, dW_h, dbias.view(G), dhW_x, dhW_h,
                g_hln[0], g_hln[1], g_hln[2], g_hln[3], dW_z, db_z, dWa, g_ln[0], g_ln[1], g_ln[2], g_ln[3], None)


def hyper_sequence_hip(p, x, h0, c0, hh0, hc0, forget_bias=1.0, drop_keep=1.0, drop_seed=0, drop_stream=0,
                       hyp_drop_keep=1.0):
    if not p.use_layer_norm:
        raise NotImplementedError("HIP HyperLSTM path requires use_layer_norm=True")
    outs = _HyperSeq.apply(x, h0, c0, hh0, hc0, drop_seed, p.W_x, p.W_h, p.bias, p.hyp_W_x, p.hyp_W_h,
                           p.hyp_ln_gamma, p.hyp_ln_beta, p.hyp_lnc_gamma, p.hyp_lnc_beta, p.W_z, p.b_z, p.W_a,
                           p.ln_gamma, p.ln_beta, p.lnc_gamma, p.lnc_beta,
                           (float(forget_bias), float(drop_keep), float(hyp_drop_keep), int(drop_stream), p.embed))
    Hout, hT, cT, hhT, hcT = outs
    return Hout, (hT, cT, hhT, hcT)
