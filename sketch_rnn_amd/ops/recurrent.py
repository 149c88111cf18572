"""Native recurrences on the GPU: per-step skinny GEMM + fused HIP cell kernel.

Step ``t`` of a layer is two launches: ``R = h_{t-1} @ W_h`` (the skinny
split-K MFMA GEMM of ``csrc/skinny_gemm.hip``; fp32 operands use its fp32
MFMA variant) and one fused cell kernel (``csrc/lstm_cell.hip``) that adds
the hoisted input projection, applies LayerNorm / hyper modulation / gates /
dropout / eoc reset and writes the next GEMM's operand directly. The
backward runs the mirror image in reverse and leaves all weight gradients
to single long-K GEMMs over the whole sequence after the scan
(``csrc/wgrad_gemm.hip``). Launched from Python but designed to be captured
whole into a HIP graph (no allocation depends on data, no host sync).

* ``_LSTMSeq`` handles ``nd`` independent recurrences of the same shape in
  one launch per step (``nd = 2``: both directions of the bidirectional
  encoder as ``2B`` rows, one batched GEMM, per-direction LN parameters).
* The HyperLSTM sequence (grouped GEMMs, fused modulation step) lives in
  :mod:`.hyper` and uses the cell launchers and geometry defined here.

Autograd boundaries are whole sequences, so no per-step autograd nodes exist.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

from ..utils import native
from . import gemm
from ._hipapi import FusedBwdArgs, FusedFwdArgs, LstmBwdArgs, LstmFwdArgs
from .reduce import colsum_many


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError("%s: launch failed (code %d)" % (what, rc))


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


_SEED_CONST = {}


def _seed_tensor(seed, device) -> torch.Tensor:
    if torch.is_tensor(seed):
        return seed.to(device=device, dtype=torch.int64).reshape(1)
    # constant seeds are cached on device: a host->device copy is not allowed
    # while a HIP graph is being captured (eager warm-up creates the entry)
    key = (str(device), int(seed))
    t = _SEED_CONST.get(key)
    if t is None:
        t = _SEED_CONST[key] = torch.tensor([int(seed)], dtype=torch.int64, device=device)
    return t


def _lp_kind(t: torch.Tensor) -> int:
    """GEMM-operand encoding written by the cell kernels: 1 bf16, 2 fp32."""
    return 1 if t.dtype == torch.bfloat16 else 2


def _inference(*ts) -> bool:
    """True when no backward will run (grad mode off or nothing requires
    grad): weights are then static, so derived copies are cached.
    Evaluated outside the autograd Function, whose
    forward always runs with grad mode off."""
    return not (torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in ts))


class _Saved:
    """Plain holder for the big per-sequence buffers (kept off autograd)."""


# ---- cell-kernel geometry (csrc/lstm_cell.hip) --------------------------------------
# A row of H hidden units runs on C workgroups (C == 1 and H > 256: one
# 1024-thread workgroup per row). Policy: 256-unit workgroups (measured
# fastest at H = 2048 with LayerNorm by the round-2 cell bench, despite the
# in-launch exchange). CELL_C > 0 overrides C (sweeps); SKR_CLUSTER=0 forces C = 1.
CLUSTER_ENABLED = os.environ.get("SKR_CLUSTER", "1") != "0"
CELL_C = 0
_ERR_FLAGS = {}


def cluster_error_flag(device) -> torch.Tensor:
    """Device int32 flag set by a clustered kernel whose in-launch wait timed
    out (results of that step are then invalid)."""
    key = str(device)
    if key not in _ERR_FLAGS:
        _ERR_FLAGS[key] = torch.zeros(1, dtype=torch.int32, device=device)
    return _ERR_FLAGS[key]


def check_cluster_errors(device) -> None:
    f = cluster_error_flag(device)
    if int(f.item()) != 0:
        f.zero_()
        raise RuntimeError("clustered LSTM cell kernel: in-launch wait timed out (workgroups not co-resident)")


_CAPACITY = {}


def _coresident_capacity() -> int:
    """Workgroups the LN cell kernels may keep resident at once: 4 per CU
    (the launcher re-checks each kernel against the occupancy API and
    refuses a grid that could strand a spinning workgroup)."""
    if not torch.cuda.is_available():
        return 1024
    d = torch.cuda.current_device()
    if d not in _CAPACITY:
        _CAPACITY[d] = 4 * torch.cuda.get_device_properties(d).multi_processor_count
    return _CAPACITY[d]


def cell_geometry(H: int, BB: int, ln: bool = True) -> int:
    """Workgroups per row (C) for the fused cell kernels."""
    if not CLUSTER_ENABLED:
        C = 1
    elif CELL_C > 0:
        C = CELL_C
    else:
        C = min(-(-H // 256), 16)
    # LayerNorm rows spin-wait on each other: keep every workgroup co-resident
    while ln and C > 1 and BB * C > _coresident_capacity():
        C //= 2
    per = -(-H // C)
    if (C == 1 and per > 2048) or (C > 1 and per > 2048):
        raise ValueError("cell kernels support at most 2048 hidden units per workgroup (H=%d, C=%d)" % (H, C))
    return C


class _ClusterSync:
    """Per-pass cell geometry + the tagged partial-statistics exchange buffer
    (zeroed once per pass; tags = step + 1 make earlier steps' slots stale)."""

    def __init__(self, T: int, BB: int, H: int, device, ln: bool = True, C: int = 0, oversub: bool = False):
        # oversub: rows past the co-resident capacity are accepted (the cell
        # launch is then made under skr_cell_set_oversub; see csrc/lstm_cell.hip)
        self.oversub = oversub
        if C > 0:   # a requested C: at least 256 units per workgroup, every workgroup co-resident
            C = min(C, max(1, H // 256))
            while ln and C > 1 and BB * C > _coresident_capacity() and not oversub:
                C //= 2
        self.C = C if C > 0 else cell_geometry(H, BB, ln)
        self.on = ln and self.C > 1
        if self.on:
            # [phase][row][workgroup][16 x 8-byte granules]: one 128-byte line per slot
            self.part = torch.zeros(2, BB, self.C, 16, dtype=torch.int64, device=device)
            self.err = cluster_error_flag(device)

    def set(self, args, t: int) -> None:
        args.cluster = self.C
        if self.on:
            args.part, args.err = self.part.data_ptr(), self.err.data_ptr()
        else:
            args.part, args.err = None, None


# ---- row-per-workgroup LayerNorm cells (csrc/row_cell.hip) --------------------------
# One workgroup per row, vector loads, workgroup-local LayerNorm statistics
# (no in-launch exchange) -- against the clustered kernels of lstm_cell.hip
# (C workgroups per row, scalar loads, tagged-slot exchanges). Measured on
# MI355X at the vae_large shapes (B = 100; profiles/r3/row_cells_ab.txt):
# faster for the HyperLSTM main-cell backward (15.4 vs 16.9 us), slower
# everywhere else (main forward 13.5 vs 9.5, hyper cell 11.6 / 8.2 vs
# 5.1 / 6.6): 100 rows occupy 100 CUs, and a CU streams only ~10-20 GB/s
# at these latencies, so spreading a row's bytes over 8 CUs wins whenever
# the row kernel saves no exchange-heavy phase. SKR_ROW_CELLS: "main"
# (default: the main-cell backward only), "all" (every eligible LayerNorm
# cell), "0" (none).
ROW_CELLS = os.environ.get("SKR_ROW_CELLS", "main")
ROW_STATS = {"row": 0, "cluster": 0, "chain": 0, "chain3": 0}   # launches by kind (tests check which kernels the hot path takes)


def _row_on(mod: int, fwd: bool) -> bool:
    if ROW_CELLS == "all":
        return True
    return ROW_CELLS == "main" and not fwd and mod == 2


def _cell_fwd(lib, a, ln: bool, mod: int, st: int, what: str) -> None:
    if ln and mod in (0, 3) and _row_on(mod, True):
        rc = lib.lib.skr_row_fwd_step(ctypes.byref(a), mod, st)
        if rc == 0:
            ROW_STATS["row"] += 1
            return
        if rc not in (-2, -3, -4):   # -2/-3/-4: shape, mode or layout the row kernels do not take
            _check(rc, what + " (row)")
    ROW_STATS["cluster"] += 1
    _check(lib.lib.skr_lstm_fwd_step(ctypes.byref(a), int(ln), mod, st), what)


def _cell_bwd(lib, a, ln: bool, mod: int, st: int, what: str) -> None:
    if ln and mod in (0, 2) and _row_on(mod, False):
        rc = lib.lib.skr_row_bwd_step(ctypes.byref(a), mod, st)
        if rc == 0:
            ROW_STATS["row"] += 1
            return
        if rc not in (-2, -3, -4):
            _check(rc, what + " (row)")
    ROW_STATS["cluster"] += 1
    _check(lib.lib.skr_lstm_bwd_step(ctypes.byref(a), int(ln), mod, st), what)


# ---- fused GEMM + cell forward step (csrc/lstm_fused.hip) ---------------------------
# Plain LSTM (no LayerNorm) layers with H in {256, 512} and bf16 operands run
# each forward step as ONE launch. SKR_FUSED=0 keeps the GEMM + cell pair.
FUSED_ENABLED = os.environ.get("SKR_FUSED", "1") != "0"


def _fused_ok(H: int, ln: bool, ldt) -> bool:
    return FUSED_ENABLED and not ln and ldt == torch.bfloat16 and H in (256, 512)


# Split-K of the per-step products of a LayerNorm-LSTM sequence: the planned
# factor (gemm.plan_splits) capped -- LN_FWD_SPLIT_CAP for h @ W_h (the cell
# sums the slabs while loading), LN_BWD_SPLIT_CAP for dG @ W_h^T (the next
# cell step sums them; up to kRecSlabs = 8 take the unrolled slab loads).
# Measured on vae_layernorm (H = 512; planned 8 / 32; same box, A B A B,
# profiles/r6/ln_split_ab.log): 10.25 / 10.31 ms/step uncapped, 9.51 / 9.52
# with the backward at 8, 9.15 / 9.16 with 2 / 8. 0: no cap. Plain LSTM
# sequences keep the planned factors.
LN_FWD_SPLIT_CAP = 2
LN_BWD_SPLIT_CAP = 8
# Chained LayerNorm-LSTM steps (csrc/chain_step.hip skr_chain_ln_fwd / _bwd):
# the cell rows of a step run INSIDE the launch of the product that feeds
# them (forward: h_{t-1} W_h; backward: dG_{t+1} W_h^T), with every operand
# but the slabs loaded before an in-launch wait -- one launch per step each
# way instead of two. Measured on vae_layernorm (same box, A B A B,
# profiles/r6/ln_chain_ab.log): 8.71 / 8.74 ms/step against 9.14 / 9.12 for
# the two launches (chained forward 12.5 us vs 5.3 + 7.7, backward 12.9 vs
# 5.3 + 8.8). LN_CHAIN_POISON (tests): NaN-fill the slabs before every
# chained launch, so a row reading ahead of its producers shows.
LN_CHAIN = True
LN_CHAIN_POISON = False
LN_CHAIN_STATS = {"fwd": 0, "bwd": 0}
# Skewed forward (csrc/chain_step.hip skr_skew_ln_fwd): launch t runs the cell
# rows of step t (their R slabs complete at launch start) and the h W_h tiles
# of step t + 1, which stage their weight slice in LDS while the rows compute
# and then wait for h_t -- the weight fetch off the critical path (probes,
# scripts/micro/ln_probe.py: the chained step is producers 5.7 + rows 5.9 us,
# fully serialised). Step 0's product is its own launch. OFF: measured
# slower, vae_layernorm 8.97 vs 8.76 ms/step (profiles/r6/skew/ab_ln.log;
# correct and poison-tested, tests/test_kernels_gpu.py).
LN_SKEW = False
LN_SKEW_STATS = {"fwd": 0}


def _lstm_splits(planned: int, cap: int, K: int) -> int:
    s = min(planned, cap) if cap > 0 and planned > 0 else planned
    return s if s > 0 and K % (64 * s) == 0 else planned


# =====================================================================================
# LSTM / LayerNorm-LSTM sequence (nd groups)
# =====================================================================================
class _LSTMSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xp, W_h, h0, c0, reset_h, reset_c, ln_g, ln_b, lnc_g, lnc_b, reset, seed, meta):
        forget_bias, keep, stream, nd, infer = meta   # infer: no autograd graph is being built
        lib = native.require_hip()
        T, BB, G = xp.shape
        H = G // 4
        dev = xp.device
        f32 = torch.float32
        ln = ln_g is not None
        xp = xp.contiguous()
        Bg = BB // nd
        ldt = gemm.lp_dtype()
        if infer and nd == 1:   # (nd > 1: W_h is a per-call stack of the directions -- nothing to cache)
            Wl = None
            WlT = gemm.derived(W_h, "lstmT%s" % ldt, lambda W: gemm.lp(W).t().contiguous())
        else:
            Wl = gemm.lp(W_h.reshape(nd, H, G)).contiguous()   # B^T of the backward product dG @ W^T
            WlT = Wl.transpose(1, 2).contiguous()              # B^T of the forward product h @ W
        S = _lstm_splits(gemm.plan_splits(Bg, G, H, nd, ldt), LN_FWD_SPLIT_CAP if ln else 0, H)
        A = torch.empty(T + 1, BB, H, device=dev, dtype=ldt)   # GEMM operands: carried h
        A[0].copy_(h0)
        CC = torch.empty(T + 1, BB, H, device=dev, dtype=f32)  # carried c
        CC[0].copy_(c0)
        Hout = torch.empty(T, BB, H, device=dev, dtype=f32)
        fused = _fused_ok(H, ln, ldt)
        # saves for the backward: LN layers keep xhat / rstd / chat (the kernel
        # recomputes the gate activations from xhat); plain layers keep act and
        # c'. Nothing is saved at inference (the fused kernel always writes them).
        keep_plain = not ln and (fused or not infer)
        Cout = torch.empty(T, BB, H, device=dev, dtype=f32) if keep_plain else None
        ACT = torch.empty(T, BB, G, device=dev, dtype=f32) if keep_plain else None
        slp = ln and _ln_saves_lp(infer)
        sdt = torch.bfloat16 if slp else f32
        XHAT = torch.empty(T, BB, G, device=dev, dtype=sdt) if ln and not infer else None
        RSTD = torch.empty(T, BB, 5, device=dev, dtype=f32) if ln and not infer else None
        CHAT = torch.empty(T, BB, H, device=dev, dtype=sdt) if ln and not infer else None
        rst = reset.contiguous().to(f32) if reset is not None else None
        # carried h differs from h' only on reset rows: without resets hT = h'_{T-1}
        HC = torch.empty(2, BB, H, device=dev, dtype=f32) if rst is not None else None
        R = torch.empty(max(S, 1), BB, G, device=dev, dtype=f32)
        rh = reset_h.contiguous() if reset_h is not None else None
        rc = reset_c.contiguous() if reset_c is not None else None
        lnp = [t.contiguous() if t is not None else None for t in (ln_g, ln_b, lnc_g, lnc_b)]
        sd = _seed_tensor(seed, dev)
        a = LstmFwdArgs()
        a.save_lp = int(slp)
        a.B, a.H, a.grp_rows = BB, H, BB // nd if nd > 1 else 0
        a.ld_xp, a.ld_R = G, G
        a.ln_g, a.ln_b, a.lnc_g, a.lnc_b = (_ptr(t) for t in lnp)
        a.init_h, a.init_c = _ptr(rh), _ptr(rc)
        a.forget_bias, a.keep = float(forget_bias), float(keep)
        a.seed, a.stream = sd.data_ptr(), int(stream)
        a.ld_lp, a.lp_kind = H, _lp_kind(A)
        a.R, a.R_nslab, a.R_slab = R.data_ptr(), max(S, 1), BB * G
        st = _stream()
        if fused:
            f = FusedFwdArgs()
            f.B, f.H, f.nd = Bg, H, nd
            f.lda, f.ld_xp, f.ld_next = H, G, H
            f.WT, f.w_gs = WlT.data_ptr(), (G * H if nd > 1 else 0)
            f.init_h, f.init_c = _ptr(rh), _ptr(rc)
            f.forget_bias, f.keep = float(forget_bias), float(keep)
            f.seed, f.stream = sd.data_ptr(), int(stream)
            for t in range(T):
                f.A, f.xp, f.c_prev = A[t].data_ptr(), xp[t].data_ptr(), CC[t].data_ptr()
                f.reset = _ptr(rst[t]) if rst is not None else None
                f.step = t
                f.h_out, f.c_out, f.act = Hout[t].data_ptr(), Cout[t].data_ptr(), ACT[t].data_ptr()
                f.h_carry = HC[t % 2].data_ptr() if HC is not None else None
                f.c_carry, f.h_next = CC[t + 1].data_ptr(), A[t + 1].data_ptr()
                _check(lib.lib.skr_lstm_fused_fwd(ctypes.byref(f), st), "lstm_fused_fwd")
            T_loop = 0
        else:
            T_loop = T
        cl = _ClusterSync(T, BB, H, dev, ln)
        # chained steps: one launch per step (product tiles + cell rows)
        chain_f = LN_CHAIN and ln and nd == 1 and rst is None and ldt == torch.bfloat16 and dev.type == "cuda" \
            and T_loop > 0 and H % 256 == 0 and H <= 2048 and 1 <= S <= 8
        cf = gemm.ChainCounters(dev, "ln_fwd", T) if chain_f else None
        WlT2 = WlT if WlT.dim() == 2 else WlT[0]
        skew = chain_f and LN_SKEW and BB <= 128 and H in (256, 512, 1024) and S in (1, 2, 4) and \
            H // S in (128, 256, 512) and T >= 2
        if skew:   # double-buffered slabs: launch t reads R2[t % 2], writes R2[(t + 1) % 2]
            R2 = torch.empty(2, S, BB, G, device=dev, dtype=f32)
            sk = gemm.ChainCounters(dev, "ln_skew", T)
            gemm.rec_gemm(A[0], WlT2, R2[0], S)
            a.R_nslab, a.R_slab = S, BB * G
        for t in range(T_loop):
            cl.set(a, t)
            a.xp = xp[t].data_ptr()
            a.c_prev = CC[t].data_ptr()
            a.reset = _ptr(rst[t]) if rst is not None else None
            a.step = t
            a.h_out = Hout[t].data_ptr()
            a.c_out = _ptr(Cout[t] if Cout is not None else None)
            a.act = _ptr(ACT[t] if ACT is not None else None)
            if XHAT is not None:
                a.xhat, a.rstd, a.chat = XHAT[t].data_ptr(), RSTD[t].data_ptr(), CHAT[t].data_ptr()
            a.h_carry = HC[t % 2].data_ptr() if HC is not None else None
            a.h_lp = A[t + 1].data_ptr()
            a.c_carry = CC[t + 1].data_ptr()
            if skew:
                a.R = R2[t % 2].data_ptr()
                if LN_CHAIN_POISON:
                    A[t + 1].fill_(float("nan"))
                rc = lib.lib.skr_skew_ln_fwd(ctypes.byref(a), WlT2.data_ptr(),
                                             R2[(t + 1) % 2].data_ptr() if t + 1 < T else None,
                                             ctypes.byref(sk.at(t)), st)
                if rc == 0:
                    LN_SKEW_STATS["fwd"] += 1
                    continue
                if t > 0 or rc not in (-2, -3, -4):
                    _check(rc if rc != 0 else -1, "skew_ln_fwd")
                skew = False   # step 0 not taken: the chained / two-launch steps (R2[0] holds step 0's product)
                sk.buf.zero_()
                a.R = R2[0].data_ptr()
                _cell_fwd(lib, a, ln, 0, st, "lstm_fwd_step")
                a.R = R.data_ptr()
                continue
            if chain_f:
                if LN_CHAIN_POISON:
                    R.fill_(float("nan"))
                if gemm.chain_ln_fwd([(A[t], WlT2, R, S)], a, cf.at(t)) == 0:
                    LN_CHAIN_STATS["fwd"] += 1
                    continue
                chain_f = False   # shape not taken: two launches from here on (counters cleared)
                cf.buf.zero_()
            gemm.rec_gemm(A[t], WlT, R, S, nd)
            _cell_fwd(lib, a, ln, 0, st, "lstm_fwd_step")
        if T == 0:
            hT = h0.clone()
        else:
            hT = HC[(T - 1) % 2].clone() if HC is not None else Hout[T - 1].clone()
        cT = CC[T].clone()
        s = _Saved()
        s.Wl, s.A, s.CC, s.Cout, s.ACT, s.XHAT, s.RSTD, s.CHAT = Wl, A, CC, Cout, ACT, XHAT, RSTD, CHAT
        s.slp = slp
        s.reset, s.seed, s.meta, s.lnp = rst, sd, meta, lnp
        s.wshape = W_h.shape
        ctx.s = s
        ctx.dims = (T, BB, H)
        if A.dtype == torch.bfloat16 and rst is None and nd == 1:
            # without resets the carried h is h': A[1:] is a bf16 copy of Hout
            # (read by the fused MDN head instead of Hout, ops.mdn_hip)
            Hout._skr_lp = A[1:]
        return Hout, hT, cT

    @staticmethod
    def backward(ctx, dHout, dhT, dcT):
        s = ctx.s
        T, BB, H = ctx.dims
        G = 4 * H
        forget_bias, keep, stream, nd, _ = s.meta
        B = BB // nd
        lib = native.require_hip()
        dev = s.A.device
        f32 = torch.float32
        ln = s.lnp[0] is not None
        dG = torch.empty(T, BB, G, device=dev, dtype=f32)
        lp_on = s.Wl.dtype == torch.bfloat16
        dG_lp = torch.empty(T, BB, G, device=dev, dtype=torch.bfloat16) if lp_on else None
        S = _lstm_splits(gemm.plan_splits(B, H, G, nd, s.Wl.dtype), LN_BWD_SPLIT_CAP if ln else 0, G)
        DH = torch.zeros(max(S, 1), BB, H, device=dev, dtype=f32)   # split-K slabs of dh into carried h
        if dhT is not None:
            DH[0].copy_(dhT)
        dc_rec = dcT.contiguous().clone() if dcT is not None else torch.zeros(BB, H, device=dev, dtype=f32)
        dHout = dHout.contiguous() if dHout is not None else None
        dinit_h = torch.zeros(BB, H, device=dev, dtype=f32) if s.reset is not None else None
        dinit_c = torch.zeros(BB, H, device=dev, dtype=f32) if s.reset is not None else None
        sdt = torch.bfloat16 if s.slp else f32
        DLNY = torch.empty(T, BB, G, device=dev, dtype=sdt) if ln else None
        DLNCY = torch.empty(T, BB, H, device=dev, dtype=sdt) if ln else None
        a = LstmBwdArgs()
        a.save_lp = int(s.slp)
        a.B, a.H, a.grp_rows = BB, H, B if nd > 1 else 0
        a.ld_dh_rec, a.dhr_nslab, a.dhr_slab = H, max(S, 1), BB * H
        a.dho_nslab = 1
        a.dh_rec, a.dc_rec = DH.data_ptr(), dc_rec.data_ptr()
        a.ln_g, a.lnc_g, a.lnc_b = _ptr(s.lnp[0]), _ptr(s.lnp[2]), _ptr(s.lnp[3])
        a.ln_b, a.forget_bias = _ptr(s.lnp[1]), float(forget_bias)
        a.keep, a.seed, a.stream = float(keep), s.seed.data_ptr(), int(stream)
        a.ld_dG, a.ld_dG_lp, a.dG_lp_kind = G, G, 1 if lp_on else 0
        a.dinit_h, a.dinit_c = _ptr(dinit_h), _ptr(dinit_c)
        st = _stream()
        if lp_on and _fused_ok(H, ln, s.Wl.dtype):
            # one launch per step: dh_rec = dG_{t+1} @ W^T fused with the cell backward
            f = FusedBwdArgs()
            f.B, f.H, f.nd = B, H, nd
            f.ld_dgn, f.W, f.w_gs = G, s.Wl.data_ptr(), H * G
            f.dc_rec = dc_rec.data_ptr()
            f.keep, f.seed, f.stream = float(keep), s.seed.data_ptr(), int(stream)
            f.dinit_h, f.dinit_c = _ptr(dinit_h), _ptr(dinit_c)
            dhT_c = dhT.contiguous() if dhT is not None else None
            for t in range(T - 1, -1, -1):
                f.dG_next = dG_lp[t + 1].data_ptr() if t < T - 1 else None
                f.dh_extra = _ptr(dhT_c) if t == T - 1 else None
                f.dh_out = dHout[t].data_ptr() if dHout is not None else None
                f.act, f.c_new, f.c_prev = s.ACT[t].data_ptr(), s.Cout[t].data_ptr(), s.CC[t].data_ptr()
                f.reset = _ptr(s.reset[t]) if s.reset is not None else None
                f.step = t
                f.dG, f.dG_lp = dG[t].data_ptr(), dG_lp[t].data_ptr()
                _check(lib.lib.skr_lstm_fused_bwd(ctypes.byref(f), st), "lstm_fused_bwd")
            if T > 0:
                gemm.rec_gemm(dG_lp[0], s.Wl, DH, S, nd)    # dh into the initial state
            T_loop = 0
        else:
            T_loop = T
        cl = _ClusterSync(T, BB, H, dev, ln)
        # chained steps: the cell rows of step t inside the dG_{t+1} W_h^T launch
        chain_b = LN_CHAIN and ln and nd == 1 and s.reset is None and lp_on and dev.type == "cuda" \
            and T_loop >= 2 and H % 256 == 0 and H <= 2048 and 1 <= S <= 8
        cb = gemm.ChainCounters(dev, "ln_bwd", T - 1) if chain_b else None
        for t in range(T_loop - 1, -1, -1):
            cl.set(a, t)
            a.dh_out = dHout[t].data_ptr() if dHout is not None else None
            a.c_prev = s.CC[t].data_ptr()
            if not ln:
                a.act, a.c_new = s.ACT[t].data_ptr(), s.Cout[t].data_ptr()
            else:
                a.xhat, a.rstd, a.chat = s.XHAT[t].data_ptr(), s.RSTD[t].data_ptr(), s.CHAT[t].data_ptr()
                a.dlny, a.dlncy = DLNY[t].data_ptr(), DLNCY[t].data_ptr()
            a.reset = _ptr(s.reset[t]) if s.reset is not None else None
            a.step = t
            a.dG = dG[t].data_ptr()
            a.dG_lp = dG_lp[t].data_ptr() if lp_on else None
            ran = False
            if chain_b and t < T - 1:   # dG_{t+1} W_h^T -> this step's rows, one launch
                if LN_CHAIN_POISON:
                    DH.fill_(float("nan"))
                ran = gemm.chain_ln_bwd([(dG_lp[t + 1], s.Wl[0], DH, S)], a, cb.at(T - 2 - t)) == 0
                if ran:
                    LN_CHAIN_STATS["bwd"] += 1
                else:   # shape not taken: unchained from here on (counters cleared)
                    chain_b = False
                    cb.buf.zero_()
                    gemm.rec_gemm(dG_lp[t + 1], s.Wl, DH, S, nd)
            if not ran:
                _cell_bwd(lib, a, ln, 0, st, "lstm_bwd_step")
            if not chain_b or t == 0:   # (chained: runs in the next step's launch)
                gemm.rec_gemm(dG_lp[t] if lp_on else dG[t], s.Wl, DH, S, nd)
        dh_rec = DH.sum(0) if DH.shape[0] > 1 else DH[0]
        dGs = dG_lp if lp_on else dG
        if nd == 1:
            dW = gemm.wgrad(s.A[:T].reshape(T * BB, H), dGs.view(T * BB, G)).view(s.wshape)
        else:
            An = s.A[:T].view(T, nd, B, H).permute(1, 0, 2, 3).reshape(nd, T * B, H)
            dGn = dGs.view(T, nd, B, G).permute(1, 0, 2, 3).reshape(nd, T * B, G)
            dW = gemm.wgrad(An, dGn).view(s.wshape)
        g_ln = [None] * 4
        if ln:   # gamma / beta: per direction group, rows (t, b) of the [T, nd, B, n] streams, one launch pair
            parts = colsum_many([(x.view(T, nd, B, n)[:, g], y.view(T, nd, B, n)[:, g])
                                 for x, y, n in ((DLNY, s.XHAT, G), (DLNCY, s.CHAT, H)) for g in range(nd)])

            def red(k, n):
                shape = s.lnp[0].shape[:-1] + (n,)
                pk = parts[k * nd:(k + 1) * nd]
                return torch.stack([p[0] for p in pk]).view(shape), torch.stack([p[1] for p in pk]).view(shape)
            g_ln = list(red(0, G) + red(1, H))
        ctx.s = None
        return (dG, dW, dh_rec, dc_rec, dinit_h, dinit_c, g_ln[0], g_ln[1], g_ln[2], g_ln[3], None, None, None)


def lstm_sequence_hip(xp, W_h, h0, c0, forget_bias=1.0, reset=None, reset_h=None, reset_c=None,
                      drop_keep=1.0, drop_seed=0, drop_stream=0, ln=None):
    if ln is None:
        ln = (None, None, None, None)
    if reset is not None and reset_h is None:
        raise ValueError("reset requires reset_h / reset_c")
    from . import persist
    lnp = ln[0] is not None
    if (reset is None and xp.shape[0] > 1 and not lnp and not _inference(xp, W_h, h0, c0)
            and persist.persist_ok(W_h.shape[0], 1, 1, B=xp.shape[1])):
        # a plain layer in training (the vae_small decoder): the whole
        # sequence, forward and backward, as one persistent launch each
        # (csrc/lstm_persist.hip)
        Hout, fin = persist.lstm_stack(xp, [W_h], [h0], [c0], drop_keep=drop_keep, drop_seed=drop_seed,
                                       drop_stream=drop_stream, forget_bias=forget_bias)
        return Hout, fin[0]
    Hout, hT, cT = _LSTMSeq.apply(xp, W_h, h0, c0, reset_h, reset_c, *ln, reset, drop_seed,
                                  (float(forget_bias), float(drop_keep), int(drop_stream), 1,
                                   _inference(xp, W_h, h0, c0)))
    return Hout, (hT, cT)


def bilstm_sequence_hip(xp_f, xp_b, W_f, W_b, h0, c0, drop_keep=1.0, drop_seed=0, streams=(0, 0),
                        ln_f=None, ln_b=None, forget_bias=1.0):
    """Both encoder directions in one launch per step (2B rows). Each
    direction keeps its own dropout stream via the row index (rows of the
    backward direction are offset by B*H in the hash index)."""
    return bilstm_sequence_packed_hip(torch.cat([xp_f, xp_b], 1), W_f, W_b, h0, c0, drop_keep, drop_seed, streams,
                                      ln_f, ln_b, forget_bias)


def bilstm_sequence_packed_hip(xp, W_f, W_b, h0, c0, drop_keep=1.0, drop_seed=0, streams=(0, 0),
                               ln_f=None, ln_b=None, forget_bias=1.0, lengths=None):
    """As :func:`bilstm_sequence_hip` with the input projections already in
    the ``[T, 2B, 4H]`` layout (forward-direction rows first; ops/inproj.py).
    ``lengths [B]``: steps at or past a row's length are padding that nothing
    reads -- the persistent kernel stops each row block after its longest row
    (outputs there are zero; :func:`.persist.lstm_stack`)."""
    B = xp.shape[1] // 2
    W = torch.stack([W_f, W_b], 0)
    h = torch.cat([h0, h0], 0)
    c = torch.cat([c0, c0], 0)
    from . import persist
    if ln_f is None and persist.persist_ok(W_f.shape[0], 2, 1, B=B):
        # both directions, every step, one persistent launch (csrc/lstm_persist.hip)
        Hout, _ = persist.lstm_stack(xp, [W], [h], [c], nd=2, drop_keep=drop_keep, drop_seed=drop_seed,
                                     drop_stream=streams[0], forget_bias=forget_bias,
                                     lengths=lengths if PERSIST_LENGTHS else None)
        return Hout[:, :B], Hout[:, B:]
    if ln_f is not None:
        ln = tuple(torch.stack([a, b], 0) for a, b in zip(ln_f, ln_b))
    else:
        ln = (None, None, None, None)
    Hout, hT, cT = _LSTMSeq.apply(xp, W, h, c, None, None, *ln, None, drop_seed,
                                  (float(forget_bias), float(drop_keep), int(streams[0]), 2,
                                   _inference(xp, W, h, c)))
    return Hout[:, :B], Hout[:, B:]


# Length-bounded persistent encoder (False: every row block runs all T steps;
# the equivalence tests compare the two).
PERSIST_LENGTHS = True


# LayerNorm saves (xhat, chat and their gradients dlny / dlncy) in bf16 in
# bf16 training: half the bytes of the cells' saves and of the gamma / beta
# reductions (csrc/lstm_args.h save_lp; the forward runs on fp32 values, the
# backward recomputes the gate activations from the bf16 save, like any bf16
# activation save). False keeps them fp32 (tests).
LN_SAVES_LP = True


def _ln_saves_lp(infer: bool) -> bool:
    return LN_SAVES_LP and not infer and gemm.lp_dtype() == torch.bfloat16
