"""GRU and vanilla-RNN recurrences on the GPU (reference ``--model gru`` /
``--model rnn``, model.py:16-23): per step, skinny split-K MFMA GEMMs
(``csrc/skinny_gemm.hip``) plus the fused elementwise kernels of
``csrc/gru_cell.hip``. Stroke-5 (layer-0) input projections and their
weight / bias gradients run on ``csrc/inproj.hip`` (fp32, one pass each
way); recurrent weight gradients on ``csrc/wgrad_gemm.hip`` (bf16,
256-multiple shapes; :func:`.gemm.wgrad`). Same eoc reset semantics as the LSTM path
(carry replaced by ``reset_h`` after a step whose input has eoc set, and the
carried gradient of that step routed to ``reset_h``).
"""
from __future__ import annotations

import ctypes

import torch

from ..utils import native
from . import gemm, inproj
from ._hipapi import GruBwdArgs, GruFwdArgs
from .recurrent import _check


def _stroke_input(x: torch.Tensor, ctx) -> bool:
    """Layer-0 stroke input (3 or 5 features, no gradient wanted): the input
    projection and its weight gradients run on csrc/inproj.hip in fp32."""
    return inproj.bproj_ok(x) and not ctx.needs_input_grad[0]


def _kind(t: torch.Tensor) -> int:
    return 1 if t.dtype == torch.bfloat16 else 2


class _GRUSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, h0, reset, reset_h, W_gx, W_gh, b_g, W_cx, W_ch, b_c):
        lib = native.require_hip()
        T, B, IN = x.shape
        H = W_gh.shape[0]
        dev, f32 = x.device, torch.float32
        TB = T * B
        stroke = _stroke_input(x, ctx)
        if stroke:   # [x @ W_gx + b_g | x @ W_cx + b_c] in one fp32 pass (csrc/inproj.hip)
            xl = x.contiguous().float()
            XP = inproj.bproj_fwd(xl, torch.cat([W_gx, W_cx], 1),
                                  torch.cat([b_g, b_c]).expand(B, 3 * H))
            XG, XC, ld_x = XP[..., :2 * H], XP[..., 2 * H:], 3 * H
        else:
            xl = gemm.lp(x.reshape(TB, IN).contiguous())
            XG = (gemm.mm(xl, gemm.lp(W_gx)) + b_g).view(T, B, 2 * H)
            XC = (gemm.mm(xl, gemm.lp(W_cx)) + b_c).view(T, B, H)
            ld_x = 0
        dt = gemm.lp_dtype()
        Wg, Wc = gemm.lp(W_gh).contiguous(), gemm.lp(W_ch).contiguous()   # B^T of the backward products
        WgT, WcT = Wg.t().contiguous(), Wc.t().contiguous()               # B^T of h @ W_gh, (r*h) @ W_ch
        S_g = gemm.plan_splits(B, 2 * H, H, 1, dt)
        S_c = gemm.plan_splits(B, H, H, 1, dt)
        HL = torch.empty(T + 1, B, H, device=dev, dtype=dt)
        HL[0].copy_(h0)
        HP = torch.empty(T + 1, B, H, device=dev, dtype=f32)
        HP[0].copy_(h0)
        RG = torch.empty(max(S_g, 1), B, 2 * H, device=dev, dtype=f32)
        RC = torch.empty(max(S_c, 1), B, H, device=dev, dtype=f32)
        RU = torch.empty(T, B, 2 * H, device=dev, dtype=f32)
        RH = torch.empty(T, B, H, device=dev, dtype=dt)
        CAND = torch.empty(T, B, H, device=dev, dtype=f32)
        HOUT = torch.empty(T, B, H, device=dev, dtype=f32)
        rst = reset.contiguous().to(f32) if reset is not None else None
        rh = reset_h.contiguous() if reset_h is not None else None
        a = GruFwdArgs()
        a.B, a.H = B, H
        a.ld_xg, a.ld_xc = (ld_x, ld_x) if stroke else (2 * H, H)
        a.Rg, a.ld_Rg, a.Rg_nslab, a.Rg_slab = RG.data_ptr(), 2 * H, max(S_g, 1), B * 2 * H
        a.Rc, a.ld_Rc, a.Rc_nslab, a.Rc_slab = RC.data_ptr(), H, max(S_c, 1), B * H
        a.init_h = rh.data_ptr() if rh is not None else None
        a.ld_rh, a.rh_kind, a.ld_lp, a.lp_kind = H, _kind(RH), H, _kind(HL)
        st = torch.cuda.current_stream().cuda_stream
        for t in range(T):
            gemm.rec_gemm(HL[t], WgT, RG, S_g)
            a.xg, a.h_prev, a.ru, a.rh_lp = XG[t].data_ptr(), HP[t].data_ptr(), RU[t].data_ptr(), RH[t].data_ptr()
            a.reset = rst[t].data_ptr() if rst is not None else None
            _check(lib.lib.skr_gru_fwd(ctypes.byref(a), 0, st), "gru_fwd_gates")
            gemm.rec_gemm(RH[t], WcT, RC, S_c)
            a.xc, a.cand, a.h_out = XC[t].data_ptr(), CAND[t].data_ptr(), HOUT[t].data_ptr()
            a.h_carry, a.h_lp = HP[t + 1].data_ptr(), HL[t + 1].data_ptr()
            _check(lib.lib.skr_gru_fwd(ctypes.byref(a), 1, st), "gru_fwd_out")
        ctx.save_for_backward(xl, W_gx, W_cx, Wg, Wc, HL, HP, RU, RH, CAND, rst)
        ctx.has_reset, ctx.stroke = rst is not None, stroke
        return HOUT, HP[T].clone()

    @staticmethod
    def backward(ctx, dHout, dhT):
        xl, W_gx, W_cx, Wg, Wc, HL, HP, RU, RH, CAND, rst = ctx.saved_tensors
        lib = native.require_hip()
        T, B, H = CAND.shape
        TB = T * B
        dev, f32 = CAND.device, torch.float32
        lp_on = Wg.dtype == torch.bfloat16
        ldt = Wg.dtype
        DPC = torch.empty(T, B, H, device=dev, dtype=f32)
        DPG = torch.empty(T, B, 2 * H, device=dev, dtype=f32)
        DPC_lp = torch.empty(T, B, H, device=dev, dtype=ldt) if lp_on else DPC
        DPG_lp = torch.empty(T, B, 2 * H, device=dev, dtype=ldt) if lp_on else DPG
        S_dc = gemm.plan_splits(B, H, H, 1, ldt)
        S_dg = gemm.plan_splits(B, H, 2 * H, 1, ldt)
        DRH = torch.empty(max(S_dc, 1), B, H, device=dev, dtype=f32)
        DHG = torch.zeros(max(S_dg, 1), B, H, device=dev, dtype=f32)
        DE = torch.zeros(2, B, H, device=dev, dtype=f32)
        if dhT is not None:
            DE[0].copy_(dhT)
        DHT = torch.empty(B, H, device=dev, dtype=f32)
        dinit = torch.zeros(B, H, device=dev, dtype=f32) if ctx.has_reset else None
        dHout = dHout.contiguous() if dHout is not None else None
        a = GruBwdArgs()
        a.B, a.H = B, H
        a.dhg, a.ld_dhg, a.dhg_nslab, a.dhg_slab = DHG.data_ptr(), H, max(S_dg, 1), B * H
        a.drh, a.ld_drh, a.drh_nslab, a.drh_slab = DRH.data_ptr(), H, max(S_dc, 1), B * H
        a.dinit_h = dinit.data_ptr() if dinit is not None else None
        a.dh_tot, a.dpc_kind, a.dpg_kind = DHT.data_ptr(), (1 if lp_on else 0), (1 if lp_on else 0)
        st = torch.cuda.current_stream().cuda_stream
        cur = 0
        for t in range(T - 1, -1, -1):
            a.dh_out = dHout[t].data_ptr() if dHout is not None else None
            a.dh_elem, a.dh_elem_out = DE[cur].data_ptr(), DE[1 - cur].data_ptr()
            a.ru, a.cand, a.h_prev = RU[t].data_ptr(), CAND[t].data_ptr(), HP[t].data_ptr()
            a.reset = rst[t].data_ptr() if rst is not None else None
            a.dpc, a.dpc_lp = DPC[t].data_ptr(), (DPC_lp[t].data_ptr() if lp_on else None)
            a.dpg, a.dpg_lp = DPG[t].data_ptr(), (DPG_lp[t].data_ptr() if lp_on else None)
            _check(lib.lib.skr_gru_bwd(ctypes.byref(a), 0, st), "gru_bwd_out")
            gemm.rec_gemm(DPC_lp[t], Wc, DRH, S_dc)
            _check(lib.lib.skr_gru_bwd(ctypes.byref(a), 1, st), "gru_bwd_gates")
            gemm.rec_gemm(DPG_lp[t], Wg, DHG, S_dg)
            cur = 1 - cur
        dh0 = DE[cur] + DHG.sum(0)
        dpg2, dpc2 = DPG_lp.view(TB, 2 * H), DPC_lp.view(TB, H)
        dW_gh = gemm.wgrad(HL[:T].reshape(TB, H), dpg2)
        dW_ch = gemm.wgrad(RH.reshape(TB, H), dpc2)
        if ctx.stroke:   # dW_x, dbias from one read of the fp32 gate gradients each
            db_g, dW_gx = inproj.bproj_reduce(xl, DPG)
            db_c, dW_cx = inproj.bproj_reduce(xl, DPC)
            db_g, db_c = db_g.sum(0), db_c.sum(0)
        else:
            dW_gx = gemm.wgrad(xl, dpg2)
            dW_cx = gemm.wgrad(xl, dpc2)
            db_g, db_c = DPG.view(TB, 2 * H).sum(0), DPC.view(TB, H).sum(0)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = (gemm.mm(dpg2, gemm.lp(W_gx).t()) + gemm.mm(dpc2, gemm.lp(W_cx).t())).view(T, B, -1)
        return (dx, dh0, None, dinit, dW_gx, dW_gh, db_g, dW_cx, dW_ch, db_c)


class _RNNSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, h0, reset, reset_h, W_x, W_h, bias):
        lib = native.require_hip()
        T, B, IN = x.shape
        H = W_h.shape[0]
        dev, f32 = x.device, torch.float32
        TB = T * B
        stroke = _stroke_input(x, ctx)
        if stroke:
            xl = x.contiguous().float()
            XP = inproj.bproj_fwd(xl, W_x, bias.expand(B, H))
        else:
            xl = gemm.lp(x.reshape(TB, IN).contiguous())
            XP = (gemm.mm(xl, gemm.lp(W_x)) + bias).view(T, B, H)
        dt = gemm.lp_dtype()
        Wl = gemm.lp(W_h).contiguous()
        WlT = Wl.t().contiguous()
        S = gemm.plan_splits(B, H, H, 1, dt)
        HL = torch.empty(T + 1, B, H, device=dev, dtype=dt)
        HL[0].copy_(h0)
        HP = torch.empty(T + 1, B, H, device=dev, dtype=f32)
        HP[0].copy_(h0)
        R = torch.empty(max(S, 1), B, H, device=dev, dtype=f32)
        HN = torch.empty(T, B, H, device=dev, dtype=f32)
        HOUT = torch.empty(T, B, H, device=dev, dtype=f32)
        rst = reset.contiguous().to(f32) if reset is not None else None
        rh = reset_h.contiguous() if reset_h is not None else None
        a = GruFwdArgs()
        a.B, a.H = B, H
        a.ld_xg = H
        a.Rg, a.ld_Rg, a.Rg_nslab, a.Rg_slab = R.data_ptr(), H, max(S, 1), B * H
        a.init_h = rh.data_ptr() if rh is not None else None
        a.ld_lp, a.lp_kind = H, _kind(HL)
        st = torch.cuda.current_stream().cuda_stream
        for t in range(T):
            gemm.rec_gemm(HL[t], WlT, R, S)
            a.xg, a.cand, a.h_out = XP[t].data_ptr(), HN[t].data_ptr(), HOUT[t].data_ptr()
            a.h_carry, a.h_lp = HP[t + 1].data_ptr(), HL[t + 1].data_ptr()
            a.reset = rst[t].data_ptr() if rst is not None else None
            _check(lib.lib.skr_gru_fwd(ctypes.byref(a), 2, st), "rnn_fwd")
        ctx.save_for_backward(xl, W_x, Wl, HL, HN, rst)
        ctx.has_reset, ctx.stroke = rst is not None, stroke
        return HOUT, HP[T].clone()

    @staticmethod
    def backward(ctx, dHout, dhT):
        xl, W_x, Wl, HL, HN, rst = ctx.saved_tensors
        lib = native.require_hip()
        T, B, H = HN.shape
        TB = T * B
        dev, f32 = HN.device, torch.float32
        lp_on = Wl.dtype == torch.bfloat16
        DP = torch.empty(T, B, H, device=dev, dtype=f32)
        DP_lp = torch.empty(T, B, H, device=dev, dtype=Wl.dtype) if lp_on else DP
        S = gemm.plan_splits(B, H, H, 1, Wl.dtype)
        DHG = torch.zeros(max(S, 1), B, H, device=dev, dtype=f32)
        if dhT is not None:
            DHG[0].copy_(dhT)
        dinit = torch.zeros(B, H, device=dev, dtype=f32) if ctx.has_reset else None
        dHout = dHout.contiguous() if dHout is not None else None
        a = GruBwdArgs()
        a.B, a.H = B, H
        a.dhg, a.ld_dhg, a.dhg_nslab, a.dhg_slab = DHG.data_ptr(), H, max(S, 1), B * H
        a.dinit_h = dinit.data_ptr() if dinit is not None else None
        a.dpc_kind = 1 if lp_on else 0
        st = torch.cuda.current_stream().cuda_stream
        for t in range(T - 1, -1, -1):
            a.dh_out = dHout[t].data_ptr() if dHout is not None else None
            a.cand = HN[t].data_ptr()
            a.reset = rst[t].data_ptr() if rst is not None else None
            a.dpc, a.dpc_lp = DP[t].data_ptr(), (DP_lp[t].data_ptr() if lp_on else None)
            _check(lib.lib.skr_gru_bwd(ctypes.byref(a), 2, st), "rnn_bwd")
            gemm.rec_gemm(DP_lp[t], Wl, DHG, S)
        dh0 = DHG.sum(0)
        dp2 = DP_lp.view(TB, H)
        dW_h = gemm.wgrad(HL[:T].reshape(TB, H), dp2)
        if ctx.stroke:
            dbias, dW_x = inproj.bproj_reduce(xl, DP)
            dbias = dbias.sum(0)
        else:
            dW_x = gemm.wgrad(xl, dp2)
            dbias = DP.view(TB, H).sum(0)
        dx = gemm.mm(dp2, gemm.lp(W_x).t()).view(T, B, -1) if ctx.needs_input_grad[0] else None
        return (dx, dh0, None, dinit, dW_x, dW_h, dbias)


def gru_sequence_hip(p, x, h0, reset=None, reset_h=None):
    return _GRUSeq.apply(x, h0, reset, reset_h, p.W_gx, p.W_gh, p.b_g, p.W_cx, p.W_ch, p.b_c)


def rnn_sequence_hip(p, x, h0, reset=None, reset_h=None):
    return _RNNSeq.apply(x, h0, reset, reset_h, p.W_x, p.W_h, p.bias)
