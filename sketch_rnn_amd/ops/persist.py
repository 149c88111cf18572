"""Persistent LSTM sequences on the GPU (``csrc/lstm_persist.hip``).

One kernel launch runs a whole sequence -- forward, and one more the whole
reverse-time backward -- for

* a stack of up to two plain-LSTM layers (the reference decoder-only model,
  ``model.py:14-30``: the layer-1 input projection ``h0_t @ W_x1`` is
  computed inside the recurrence, so the two layers run as a wavefront:
  layer 1 step t overlaps layer 0 step t+1), or
* two independent recurrences of one layer (the VAE's bidirectional
  encoder),

with bf16 MFMA operands and fp32 cell state, the reference's eoc state reset
and the stateless recurrent-dropout hash. Weight gradients are formed after
the scan as single long-K products over every saved step (``gemm.wgrad``).

Plain LSTM layers only: a LayerNorm-LSTM variant (both LayerNorms' row
statistics exchanged in-launch) measured slower than the per-step clustered
cells on vae_layernorm (11.50 vs 10.34 ms/step: each of the two exchanges
per step is a ~6 us payload-drain + flag hop) and was removed in round 5.

Dispatch: :func:`persist_ok` is the eligibility test (bf16 compute dtype,
H in {256, 512}); ``SKR_PERSIST=0`` disables the path (the per-step fused
kernels of :mod:`.recurrent` run instead).
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence, Tuple

import torch

from ..utils import native
from . import gemm
from ._hipapi import PBwdArgs, PFwdArgs

PERSIST_ENABLED = os.environ.get("SKR_PERSIST", "1") != "0"
# debug: fill every handed-off buffer with NaN before the launch, so a read
# that overtakes its hand-off shows up as a NaN instead of a stale value
POISON = os.environ.get("SKR_PERSIST_POISON", "0") == "1"
_ROWS = 32          # rows per workgroup row block (MTW = 2 sixteen-row tiles) ...
_ROWS_WIDE = 64     # ... or 64 (MTW = 4) when the 32-row grid exceeds one workgroup per CU


def _cu_count() -> int:
    if not torch.cuda.is_available():
        return 256
    return torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count


def block_rows(H: int, nd: int, L: int, B: int) -> int:
    """Rows per row block (32, or 64 when the 32-row grid of L * nd *
    ceil(B / 32) row blocks x H / 16 workgroups exceeds one workgroup per
    CU); 0 when neither fits."""
    for rows in (_ROWS, _ROWS_WIDE):
        if L * nd * (-(-B // rows)) * (H // 16) <= _cu_count():
            return rows
    return 0


def persist_ok(H: int, nd: int = 1, L: int = 1, ln: bool = False, B: Optional[int] = None) -> bool:
    """Eligibility of the persistent kernels. ``B``: rows per direction; the
    grid (L * nd * ceil(B / rows) row blocks x H / 16 workgroups, rows 32 or
    64: :func:`block_rows`) must fit one workgroup per CU, since every
    workgroup spin-waits on its peers (the launcher refuses a larger grid:
    -8). Callers fall back to the per-step kernels otherwise."""
    if not PERSIST_ENABLED or ln or gemm.lp_dtype() != torch.bfloat16:
        return False
    if L == 2:
        shape_ok = nd == 1 and H == 256
    else:
        shape_ok = L == 1 and nd in (1, 2) and H in (256, 512)
    if not shape_ok:
        return False
    if B is not None and block_rows(H, nd, L, B) == 0:
        return False
    return True


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError("%s: launch failed (code %d)" % (what, rc))


class _Saved:
    pass


def _fwd_launch(xp0, W_in1, b1, W_h0, W_h1, h0a, c0a, h0b, c0b, reset, seed, meta, tlen=None, last=False):
    """The forward launch of :class:`_PersistLSTM` (also used by
    :class:`_PersistBiEncoder`). ``last``: instead of the top layer's whole
    output sequence, write only h at each row's last valid step
    (``tlen[b] - 1``) -- ``[nd*B, H]``. Returns ``(top, finals, saved, dims)``."""
    L, nd, keep, stream, fb = meta
    from .recurrent import _seed_tensor, cluster_error_flag
    lib = native.require_hip()
    T, NB, G = xp0.shape
    H, B = G // 4, NB // nd
    dev, bf, f32 = xp0.device, torch.bfloat16, torch.float32
    nrb = -(-B // (block_rows(H, nd, L, B) or _ROWS))
    xp0 = xp0.contiguous()
    Wh = [W_h0] + ([W_h1] if L == 2 else [])
    h0s = [h0a.contiguous()] + ([h0b.contiguous()] if L == 2 else [])
    c0s = [c0a.contiguous()] + ([c0b.contiguous()] if L == 2 else [])
    # bf16 operands in both layouts, one pass per weight (csrc/convert.hip)
    Wl0, WT0 = gemm.cast_transpose(W_h0.reshape(-1, H, G))                 # [nd, H, 4H] (backward B^T), [nd, 4H, H]
    Wl, WT = [Wl0], [WT0]
    Wu = None
    if L == 2:
        WT1 = torch.empty(G, 2 * H, dtype=bf, device=dev)                  # [4H, 2H]: [W_in | W_h] per column
        Wu, _ = gemm.cast_transpose(W_in1, trans=WT1[:, :H])               # [H, 4H]
        Wl1, _ = gemm.cast_transpose(W_h1, trans=WT1[:, H:])
        Wl.append(Wl1.reshape(1, H, G))
        WT.append(WT1)
    rst = reset.contiguous().to(f32) if reset is not None else None
    sd = _seed_tensor(seed, dev)
    b1c = b1.contiguous().to(f32) if L == 2 else None
    a = PFwdArgs()
    a.T, a.B, a.nd, a.L, a.H, a.nrb = T, B, nd, L, H, nrb
    a.reset, a.forget_bias, a.seed = _ptr(rst), float(fb), sd.data_ptr()
    # zeroed by the launcher: the h hand-off epochs
    flags = torch.empty(L * nd * nrb * 64, dtype=torch.int32, device=dev)
    a.flags, a.err = flags.data_ptr(), cluster_error_flag(dev).data_ptr()
    tl = tlen.to(device=dev, dtype=torch.int32).contiguous() if tlen is not None else None
    assert not last or (tl is not None and L == 1)
    a.tlen = _ptr(tl)
    s = _Saved()
    s.hlp, s.hup, s.c_out, s.c_carry, s.act = [], [], [], [], []
    outs = []
    for l in range(L):
        ly = a.ly[l]
        # carried h, direction-major [nd, T+1, B, H] (the kernel's layout:
        # each direction is one contiguous [T*B, H] operand of its dW GEMM)
        hlp = torch.empty(nd, T + 1, B, H, dtype=bf, device=dev)
        if POISON:
            hlp.fill_(float("nan"))
        hlp[:, 0].copy_(h0s[l].view(nd, B, H))
        hup = torch.empty(T, NB, H, dtype=bf, device=dev) if (l < L - 1 and rst is not None) else None
        h_out = torch.empty(T, NB, H, dtype=f32, device=dev) if (l == L - 1 and not last) else None
        h_last = torch.empty(B, nd * H, dtype=f32, device=dev) if last else None   # [h_fw | h_bw] rows
        c_out = torch.empty(T, NB, H, dtype=f32, device=dev)
        c_carry = torch.empty(T + 1, NB, H, dtype=f32, device=dev) if rst is not None else None
        act = torch.empty(T, NB, G, dtype=f32, device=dev)
        hT = torch.empty(NB, H, dtype=f32, device=dev)
        cT = torch.empty(NB, H, dtype=f32, device=dev)
        ly.WT, ly.w_gs, ly.kin = WT[l].data_ptr(), (G * H if (l == 0 and nd > 1) else 0), (0 if l == 0 else H)
        if l == 0:
            ly.xp, ly.xp_ts, ly.xp_ld = xp0.data_ptr(), NB * G, G
        else:
            ly.xp, ly.xp_ts, ly.xp_ld = b1c.data_ptr(), 0, 0
        ly.c0 = c0s[l].data_ptr()
        ly.init_h, ly.init_c = (h0s[l].data_ptr(), c0s[l].data_ptr()) if rst is not None else (None, None)
        ly.hlp, ly.hup, ly.h_out, ly.c_out = hlp.data_ptr(), _ptr(hup), _ptr(h_out), c_out.data_ptr()
        ly.c_carry, ly.act, ly.hT, ly.cT = _ptr(c_carry), _ptr(act), hT.data_ptr(), cT.data_ptr()
        ly.keep, ly.stream = float(keep), int(stream) + l
        ly.h_last = _ptr(h_last)
        s.hlp.append(hlp)
        s.hup.append(hup)
        s.c_out.append(c_out)
        s.c_carry.append(c_carry)
        s.act.append(act)
        if l == L - 1:
            top = h_last if last else h_out
        outs += [hT, cT]
    _check(lib.lib.skr_lstm_persist_fwd(ctypes.byref(a), torch.cuda.current_stream().cuda_stream),
           "lstm_persist_fwd")
    s.Wl, s.Wu, s.c0s, s.rst, s.seed, s.meta = Wl, Wu, c0s, rst, sd, meta
    s.shapes = [W.shape for W in Wh]
    s.keep_flags = flags
    s.tlen = tl
    s.last = last
    return top, outs, s, (T, B, H, nrb)


def _bwd_launch(s, dims, dtop, dfinal, fp32_dg=True):
    """The backward launch + weight gradients. ``fp32_dg=False``: the gate
    gradient is written only in bf16 (the caller reads ``dg_lp``). Returns
    ``(dg, dg_lp, dWh, dWin1, db1, dh0, dc0)`` (lists per layer)."""
    T, B, H, nrb = dims
    L, nd, keep, stream, fb = s.meta
    from .recurrent import cluster_error_flag
    lib = native.require_hip()
    NB, G = nd * B, 4 * H
    dev, bf, f32 = s.hlp[0].device, torch.bfloat16, torch.float32
    b = PBwdArgs()
    b.T, b.B, b.nd, b.L, b.H, b.nrb = T, B, nd, L, H, nrb
    b.reset, b.seed = _ptr(s.rst), s.seed.data_ptr()
    flags = torch.empty(L * nd * nrb * 64, dtype=torch.int32, device=dev)
    b.flags, b.err = flags.data_ptr(), cluster_error_flag(dev).data_ptr()
    b.tlen = _ptr(s.tlen)
    dtop = dtop.contiguous() if dtop is not None else None
    dg_lp, dg, dh0, dc0, dih, dic, keep_alive = [], [], [], [], [], [], []
    for l in range(L):
        ly = b.ly[l]
        ly.Wr, ly.wr_gs = s.Wl[l].data_ptr(), (H * G if nd > 1 else 0)
        ly.Wu = s.Wu.data_ptr() if (L == 2 and l == 0) else None
        top = l == L - 1
        ly.dh_out = _ptr(dtop) if (top and not s.last) else None
        ly.dh_last = _ptr(dtop) if (top and s.last) else None
        dhT, dcT = dfinal[2 * l], dfinal[2 * l + 1]
        dhT = dhT.contiguous() if dhT is not None else None
        dcT = dcT.contiguous() if dcT is not None else None
        keep_alive += [dhT, dcT]
        ly.dhT, ly.dcT = _ptr(dhT), _ptr(dcT)
        ly.act, ly.c_out, ly.c_carry, ly.c0 = (_ptr(s.act[l]), s.c_out[l].data_ptr(), _ptr(s.c_carry[l]),
                                               s.c0s[l].data_ptr())
        gl = torch.empty(nd, T, B, G, dtype=bf, device=dev)       # direction-major, like hlp
        if POISON:
            gl.fill_(float("nan"))
        gf = torch.empty(T, NB, G, dtype=f32, device=dev) if (fp32_dg or l < L - 1) else None
        h0g = torch.empty(NB, H, dtype=f32, device=dev)
        c0g = torch.empty(NB, H, dtype=f32, device=dev)
        ihg = torch.empty(NB, H, dtype=f32, device=dev) if s.rst is not None else None
        icg = torch.empty(NB, H, dtype=f32, device=dev) if s.rst is not None else None
        ly.dg_lp, ly.dg, ly.dh0, ly.dc0 = gl.data_ptr(), _ptr(gf), h0g.data_ptr(), c0g.data_ptr()
        ly.dinit_h, ly.dinit_c = _ptr(ihg), _ptr(icg)
        ly.keep, ly.stream = float(keep), int(stream) + l
        dg_lp.append(gl)
        dg.append(gf)
        dh0.append(h0g)
        dc0.append(c0g)
        dih.append(ihg)
        dic.append(icg)
    _check(lib.lib.skr_lstm_persist_bwd(ctypes.byref(b), torch.cuda.current_stream().cuda_stream),
           "lstm_persist_bwd")
    # weight gradients: one long-K product per matrix over all T*B rows
    dWh = []
    for l in range(L):
        A = s.hlp[l][:, :T]                                        # [nd, T, B, H] (a view: no copy)
        if nd == 1:
            dW = gemm.wgrad(A.reshape(T * NB, H), dg_lp[l].view(T * NB, G))
        else:
            dW = gemm.wgrad(A.reshape(nd, T * B, H), dg_lp[l].view(nd, T * B, G))
        dWh.append(dW.reshape(s.shapes[l]))
    dWin1 = db1 = None
    if L == 2:
        src = s.hup[0] if s.hup[0] is not None else s.hlp[0][0, 1:]
        dWin1, db1 = gemm.wgrad(src.reshape(T * NB, H), dg_lp[1].view(T * NB, G), colsum=True)
    # the eoc-reset targets are the initial states themselves
    dh0t = [dh0[l] + dih[l] if dih[l] is not None else dh0[l] for l in range(L)]
    dc0t = [dc0[l] + dic[l] if dic[l] is not None else dc0[l] for l in range(L)]
    return dg, dg_lp, dWh, dWin1, db1, dh0t, dc0t


class _PersistLSTM(torch.autograd.Function):
    """Inputs: ``xp0 [T, nd*B, 4H]`` (layer-0 input projection + bias),
    ``W_in1 [H, 4H]`` / ``b1 [4H]`` (layer 1's input weights, L = 2),
    ``W_h0 [nd, H, 4H]`` (or ``[H, 4H]``), ``W_h1``, initial states
    ``[nd*B, H]`` per layer (also the eoc-reset targets), ``reset [T, nd*B]``.
    Outputs: the top layer's ``h [T, nd*B, H]`` and every layer's final
    carried ``(h, c)``."""

    @staticmethod
    def forward(ctx, xp0, W_in1, b1, W_h0, W_h1, h0a, c0a, h0b, c0b, reset, seed, meta, tlen=None):
        top, outs, s, dims = _fwd_launch(xp0, W_in1, b1, W_h0, W_h1, h0a, c0a, h0b, c0b, reset, seed, meta, tlen)
        ctx.s, ctx.dims = s, dims
        return (top, *outs)

    @staticmethod
    def backward(ctx, dtop, *dfinal):
        L = ctx.s.meta[0]
        dg, _, dWh, dWin1, db1, dh0t, dc0t = _bwd_launch(ctx.s, ctx.dims, dtop, dfinal)
        ctx.s = None
        return (dg[0], dWin1, db1, dWh[0], dWh[1] if L == 2 else None,
                dh0t[0], dc0t[0], dh0t[1] if L == 2 else None, dc0t[1] if L == 2 else None,
                None, None, None, None)


class _PersistBiEncoder(torch.autograd.Function):
    """The VAE encoder as one autograd node: the input projection of both
    directions (csrc/inproj.hip), the persistent bidirectional LSTM, and
    only ``h[len - 1]`` of every row written ([2B, H], forward rows first).
    Backward: the persistent kernel adds ``dh_last`` at each row's last step
    (no [T, 2B, H] output or gradient tensor exists; ``h_last`` is written
    as ``[B, 2H] = [h_fw | h_bw]``, the layout the latent layer reads), writes the gate
    gradient in bf16 only, and the input-projection gradients are read from
    it directly (no fp32 [T, 2B, 4H] copy)."""

    @staticmethod
    def forward(ctx, x, lengths, W_xf, W_xb, b_f, b_b, W_hf, W_hb, seed, meta):
        keep, stream, fb = meta
        from .inproj import bilstm_input_proj
        with torch.no_grad():
            xp = bilstm_input_proj(x, lengths, W_xf, W_xb, b_f, b_b)      # [T, 2B, 4H] fp32
        T, NB, G = xp.shape
        H = G // 4
        h0 = torch.zeros(NB, H, device=xp.device, dtype=torch.float32)
        W = torch.stack([W_hf, W_hb], 0)
        top, _, s, dims = _fwd_launch(xp, None, None, W, None, h0, h0, None, None, None, seed,
                                      (1, 2, keep, stream, fb), lengths, last=True)
        ctx.s, ctx.dims = s, dims
        ctx.x = x.contiguous().float()
        ctx.ln = lengths.to(device=x.device, dtype=torch.int64).contiguous()
        ctx.has_bias = b_f is not None
        return top

    @staticmethod
    def backward(ctx, dlast):
        _, dg_lp, dWh, _, _, _, _ = _bwd_launch(ctx.s, ctx.dims, dlast, (None, None), fp32_dg=False)
        lib = native.require_hip()
        x, ln = ctx.x, ctx.ln
        T, B, IN = x.shape
        G = dg_lp[0].shape[-1]
        RS = min(T, 64)
        part = torch.empty(RS, 2, IN + 1, G, device=x.device, dtype=torch.float32)
        rc = lib.lib.skr_inproj_bwd(x.data_ptr(), ln.data_ptr(), dg_lp[0].data_ptr(), 1, part.data_ptr(), T, B, IN,
                                    G, RS, torch.cuda.current_stream().cuda_stream)
        if rc != 0:
            raise RuntimeError("skr_inproj_bwd failed (%d)" % rc)
        red = part.sum(0)                                   # [2, IN + 1, G]
        db = (red[0, IN], red[1, IN]) if ctx.has_bias else (None, None)
        ctx.s = None
        return None, None, red[0, :IN], red[1, :IN], db[0], db[1], dWh[0][0], dWh[0][1], None, None


def bilstm_last_h(x, lengths, W_xf, W_xb, b_f, b_b, W_hf, W_hb, drop_keep=1.0, drop_seed=0, drop_stream=0,
                  forget_bias=1.0) -> torch.Tensor:
    """``[h_fw[len-1] | h_bw[len-1]]`` ([B, 2H]) of the bidirectional encoder
    over stroke inputs ``x [T, B, 3|5]`` (the backward direction reads each
    sketch reversed within its length). Eligibility: :func:`bilstm_last_ok`."""
    return _PersistBiEncoder.apply(x, lengths, W_xf, W_xb, b_f, b_b, W_hf, W_hb, drop_seed,
                                   (float(drop_keep), int(drop_stream), float(forget_bias)))


def bilstm_last_ok(x, H: int, B: int) -> bool:
    from . import use_hip
    from .recurrent import PERSIST_LENGTHS
    return (BI_ENCODER and PERSIST_LENGTHS and x.is_cuda and use_hip(x) and x.shape[-1] in (3, 5)
            and not x.requires_grad and persist_ok(H, 2, 1, ln=False, B=B))


BI_ENCODER = True   # False: projection + biLSTM + gather as separate ops (tests)


def lstm_stack(xp0: torch.Tensor, W_h: Sequence[torch.Tensor], h0: Sequence[torch.Tensor],
               c0: Sequence[torch.Tensor], W_in1: Optional[torch.Tensor] = None, b1: Optional[torch.Tensor] = None,
               reset: Optional[torch.Tensor] = None, nd: int = 1, drop_keep: float = 1.0, drop_seed=0,
               drop_stream: int = 0, forget_bias: float = 1.0,
               lengths: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, List[Tuple]]:
    """Run ``len(W_h)`` (1 or 2) stacked LSTM layers over ``xp0`` in one
    persistent launch. Returns the top layer's outputs ``[T, nd*B, H]`` and
    the final carried ``(h, c)`` of every layer.

    ``lengths [B]`` (one layer only; the same for every direction): rows are
    padding from their length on and nothing downstream reads them, so each
    32-row block stops after its longest row (TF ``dynamic_rnn`` with
    ``sequence_length`` skips those steps the same way). Outputs past a
    block's last step are zero and its final state is the one after that
    step."""
    L = len(W_h)
    meta = (L, nd, float(drop_keep), int(drop_stream), float(forget_bias))
    if L == 2:
        outs = _PersistLSTM.apply(xp0, W_in1, b1, W_h[0], W_h[1], h0[0], c0[0], h0[1], c0[1], reset, drop_seed, meta)
        return outs[0], [(outs[1], outs[2]), (outs[3], outs[4])]
    outs = _PersistLSTM.apply(xp0, None, None, W_h[0], None, h0[0], c0[0], None, None, reset, drop_seed, meta,
                              lengths)
    return outs[0], [(outs[1], outs[2])]
