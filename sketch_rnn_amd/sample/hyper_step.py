"""Lean per-stroke HyperLSTM decode step for :class:`~.sampler.GraphDecoder`
(reference per-stroke step ``model.py:213-249``).

The generic path (``SketchVAE.decode_step``) runs a whole T = 1 sequence per
stroke: per-call state copies into the operand buffers, zero fills, the
``z`` projections, a library head GEMM -- 20+ launches, ~60 % of them glue.
Here the decoder state lives in place for the whole decode, the per-sketch
constants (``z`` projections) are computed once, and every launch is a
hand-written kernel.

Four-launch stroke (:meth:`HyperStepDecoder.step_fused`, the
:class:`~.sampler.GraphDecoder` path whenever ``hyper_num_units == 256``,
embedding <= 32, ``dec_rnn_size % 32 == 0``):

1. grouped skinny GEMM ``{h W_h, [h | hh] W_y, h W_out}`` -- the head of the
   PREVIOUS stroke's ``h`` rides in the step's own GEMM launch;
2. ``skr_decode_hyper_cell`` (csrc/decode_step.hip): samples stroke t-1 from
   the head slabs (same keyed draws as ``skr_mdn_sample_slabs``), writes it
   out and forms the hyper cell's x-projection from it in-register, then the
   hyper LayerNorm cell;
3. ``skr_hyper_mod_fwd`` (csrc/hyper_mod.hip) in decode mode: the
   modulation vectors ``hh P + q`` on MFMA, the main cell's x-projection
   from the stroke, the modulated gate pre-activations and their LayerNorm
   partial sums;
4. the main LayerNorm cell (MOD 3: pre-activations precomputed).

After the last stroke :meth:`finish` runs the head GEMM + sampler once. Up to
1024 rows run as ONE decoder (128-row MFMA blocks inside each launch).

Other hyper widths take :meth:`HyperStepDecoder.step` (seven launches:
stroke projection, grouped GEMM, hyper cell, ``hh P`` GEMM, main cell, head
GEMM, sampler) on chunks of at most 128 rows.

GEMMs take bf16 operands with fp32 accumulation, except with ``fp8=True``
(BASELINE config 5, the fused stroke only): ``h W_h`` -- 80 % of the
stroke's GEMM FLOPs -- runs as an MX-fp8 GEMM (``ops/mx8.py``,
``csrc/mx8_gemm.hip``: e4m3 with one E8M0 scale per 32 k, twice the bf16
MFMA rate, half the weight bytes). ``W_h`` is quantized once per weight
version; the main cell writes the fp8 copy of ``h`` beside its bf16 copy
(``FwdArgs::h_q8``), so the stroke gains no conversion launch -- one launch
more than the bf16 stroke (the fp8 product leaves the grouped bf16 launch).
"""
from __future__ import annotations

import ctypes

import torch

from ..ops import gemm, mx8
from ..ops._hipapi import DecodeSample, LstmFwdArgs, ModDecode
from ..ops.hyper import _fold_ok
from ..ops.recurrent import _ClusterSync, _seed_tensor
from ..utils import native

# Main-cell workgroups per row above 128 rows (the wide decode): 1 keeps
# one 1024-thread workgroup per row; C > 1 splits rows over C workgroups with
# more rows than can be resident at once (consecutive workgroup ids share
# one dispatch position per XCD, so partners are never stranded). Measured
# (profiles/r6/decode_wide_knobs_ab.jsonl): C = 2 0.144 vs 0.157 ms per decode
# step at B = 1024, 0.084 vs 0.090 at B = 512 (4: 0.149 / 0.087, 8: 0.159 /
# 0.092).
WIDE_MAIN_C = 2


def hyper_step_ok(model, B: int) -> bool:
    cfg = model.cfg
    if cfg.dec_model != "hyper" or not torch.cuda.is_available():
        return False
    if next(model.parameters()).device.type != "cuda" or gemm.lp_dtype() != torch.bfloat16:
        return False
    from ..ops import get_compute_dtype
    if get_compute_dtype() != "bf16" or not model.dec.use_layer_norm:
        return False
    H, Hh = cfg.dec_rnn_size, cfg.hyper_num_units
    if B > 128 and not (wide_ok(model) and B % 128 == 0 and B <= 1024):
        return False
    return H % 64 == 0 and Hh % 64 == 0 and cfg.num_mixture <= 32


def wide_ok(model) -> bool:
    """One decoder over up to 1024 rows (128-row blocks inside each launch)
    instead of 128-row chunks on concurrent streams: the four-launch stroke's
    shape limits (:class:`HyperStepDecoder` ``fused``)."""
    cfg = model.cfg
    return WIDE and cfg.hyper_num_units == 256 and cfg.hyper_embedding_size <= 32 and cfg.dec_rnn_size % 32 == 0


WIDE = True   # one decoder over B > 128 rows (False: tests of the 128-row chunked decoders)


FUSED = True   # four-launch stroke where its shape limits allow (False: tests of the seven-launch step)


class HyperStepDecoder:
    """In-place decoder state of B <= 128 rows + the per-step launch sequence."""

    def __init__(self, model, B: int, device, cluster: bool = True, fp8: bool = False):
        """``cluster=False``: the main cell keeps each row in ONE workgroup (no
        in-launch LayerNorm exchange), so this decoder can run on a stream
        concurrent with another one's clustered cells without any
        co-residency requirement. ``fp8``: ``h W_h`` as an MX-fp8 GEMM (fused
        stroke, ``dec_rnn_size % 512 == 0`` and ``<= 2048``; else bf16)."""
        self.lib = native.require_hip().lib
        cfg, p = model.cfg, model.dec
        self.model, self.B, self.dev = model, B, device
        H, Hh = cfg.dec_rnn_size, cfg.hyper_num_units
        G, Gh, K = 4 * H, 4 * Hh, H + Hh
        self.H, self.Hh, self.G, self.Gh, self.K = H, Hh, G, Gh, K
        self.M = cfg.num_mixture
        self.nout = 3 + 6 * self.M
        self.E = p.embed
        bf, f32 = torch.bfloat16, torch.float32
        self.S_m = gemm.plan_splits(B, G, H, 1, bf)
        self.S_y = gemm.plan_splits(B, Gh, K, 1, bf)
        self.S_o = gemm.plan_splits(B, 128, H, 1, bf)
        assert min(self.S_m, self.S_y, self.S_o) >= 1
        # four-launch stroke (step_fused): hyper_mod's shape limits (Hh == 256,
        # E <= 32, 32-unit tiles, <= 4 main-GEMM slabs)
        self.fused = FUSED and Hh == 256 and self.E <= 32 and H % 32 == 0
        self.fp8 = bool(fp8) and self.fused and H % 512 == 0 and H <= 2048 and G % 128 == 0
        if self.fused:
            self.S_m = 4 if self.S_m >= 4 else 2 if self.S_m >= 2 else 1
            if self.fp8:   # MX-fp8 h W_h: one fp32 output (no split-K), h's fp8 copy from the main cell
                self.S_m = 1
                self.A8 = torch.zeros(B, H, dtype=torch.uint8, device=device)
                self.SA = torch.zeros(B, H // 32, dtype=torch.uint8, device=device)
            self.X = torch.zeros(B, 5, dtype=f32, device=device)
            self.GP = torch.empty(B, G, dtype=f32, device=device)
            self.GS = torch.empty(B, 4, H // 32, 2, dtype=f32, device=device)
        # state / operand buffers (resident for the whole decode)
        self.A = torch.zeros(B, K, dtype=bf, device=device)   # [h | hh] GEMM operand
        self.CC = torch.zeros(B, H, dtype=f32, device=device)
        self.HCC = torch.zeros(B, Hh, dtype=f32, device=device)
        self.Hout = torch.empty(B, H, dtype=f32, device=device)
        self.HH = torch.empty(B, Hh, dtype=f32, device=device)
        self.RM = torch.empty(self.S_m, B, G, dtype=f32, device=device)
        self.RY = torch.empty(self.S_y, B, Gh, dtype=f32, device=device)
        self.VEC = torch.empty(B, 12 * H, dtype=bf, device=device)
        self.XP = torch.empty(B, G + Gh, dtype=f32, device=device)   # [main | hyper] stroke projections
        self.ZP = torch.zeros(B, G + Gh, dtype=f32, device=device)   # per-sketch z projections
        self.ZS = torch.empty(self.S_o, B, 128, dtype=f32, device=device)
        self.clm = _ClusterSync(1, B, H, device)
        if not cluster or B > 128:   # (wide: 1024-thread rows, no co-residency requirement)
            self.clm.C, self.clm.on = 1, False
            if cluster and WIDE_MAIN_C > 1:   # wide rows split over C workgroups anyway (oversubscribed)
                self.clm = _ClusterSync(1, B, H, device, C=WIDE_MAIN_C, oversub=True)
        self.clh = _ClusterSync(1, B, Hh, device)
        self.sd = _seed_tensor(0, device)

    # -- weights (cached per weight version, like the inference path of _HyperSeq) -----
    def _weights(self):
        m, p = self.model, self.model.dec
        H, Hh, E, dt = self.H, self.Hh, self.E, torch.bfloat16
        IN = p.W_x.shape[0]

        def fold(W_z, b_z, W_a):
            if _fold_ok(H, Hh, E):   # the training path's fold kernel (csrc/hyper_fold.hip): P^T bf16, q
                Pl = torch.empty(Hh, 12 * H, dtype=dt, device=W_z.device)   # (both layouts are written)
                PlT = torch.empty(12 * H, Hh, dtype=dt, device=W_z.device)
                q = torch.empty(12, H, dtype=torch.float32, device=W_z.device)
                rc = self.lib.skr_hyper_fold(W_z.detach().contiguous().data_ptr(), b_z.detach().contiguous().data_ptr(),
                                             W_a.detach().contiguous().data_ptr(), None, Hh, H, E, Pl.data_ptr(),
                                             PlT.data_ptr(), q.data_ptr(), None,
                                             torch.cuda.current_stream().cuda_stream)
                if rc != 0:
                    raise RuntimeError("skr_hyper_fold failed (%d)" % rc)
                return PlT, q
            Wz3 = W_z.view(Hh, 12, E).permute(1, 0, 2)
            P = torch.bmm(Wz3, W_a).permute(1, 0, 2).reshape(Hh, 12 * H)
            q = torch.bmm(b_z.view(12, 1, E), W_a).reshape(12, H).contiguous()
            return P.t().to(dt).contiguous(), q

        def wy(a, b):
            return torch.cat([a[IN:], b], 0).to(dt).t().contiguous()

        def wout(W):
            Wt = torch.zeros(128, H, dtype=dt, device=W.device)
            Wt[: W.shape[1]] = W.t().to(dt)
            return Wt

        self._fold = lambda: gemm.derived((p.W_z, p.b_z, p.W_a), "hypP%s" % dt, fold)
        w = dict(
            WhT=gemm.derived(p.W_h, "hypWhT%s" % dt, lambda W: W.to(dt).t().contiguous()),
            WyT=gemm.derived((p.hyp_W_x, p.hyp_W_h), "hypWyT%s" % dt, wy),
            W5=gemm.derived((p.W_x, p.hyp_W_x), "stepW5",
                            lambda a, b: torch.cat([a[:5], b[:5]], 1).float().contiguous()),
            WoT=gemm.derived(m.output_w, "stepWoT", wout),
            bo=m.output_b.detach().float().contiguous(),
        )
        if self.fp8:     # W_h [H, 4H] -> e4m3 [4H, H] + E8M0 block scales, once per weight version
            w["Wh8"] = gemm.derived(p.W_h, "hypWh8", lambda W: mx8.quant_t(W.detach().float().contiguous()))
        if self.fused:   # bf16 folded P^T for csrc/hyper_mod.hip, q + the main bias on the shift block
            P, q = self._fold()

            def qbias(q, bias):
                qb = q.detach().clone()
                qb[8:] += bias.detach().view(4, H)
                return qb.reshape(12 * H).float().contiguous()
            w["PL"] = P
            w["QB"] = gemm.derived((q, p.bias), "hypQB", qbias)
        return w

    def _pq(self):
        """Folded modulation weights (P^T, q) of the seven-launch :meth:`step`."""
        if "PQ" not in self._w:
            P, q = self._fold()
            self._w["PQ"] = (P, q)
        return self._w["PQ"]

    @torch.no_grad()
    def prepare(self) -> None:
        """(Re)derive the low-precision weight operands (cached per weight
        version). Called by :meth:`begin`; callers running several decoders
        on forked streams call it on the parent stream first."""
        self._w = self._weights()
        if not self.fused:
            # the seven-launch step's folded (P^T, q): derived HERE, on the
            # parent stream, never lazily inside step() -- a decoder on a
            # forked chunk stream would otherwise find another chunk's P in
            # gemm.derived's global cache before that stream has written it
            self._pq()

    @torch.no_grad()
    def begin(self, zc, state, x0=None) -> None:
        """Load the initial state, the per-sketch z projections and (fused
        path) the first stroke ``x0 [B, 5]``."""
        if getattr(self, "_w", None) is None:
            self.prepare()
        p = self.model.dec
        H = self.H
        h0, c0, hh0, hc0 = state
        self.A[:, :H].copy_(h0)
        self.A[:, H:].copy_(hh0)
        self.CC.copy_(c0)
        self.HCC.copy_(hc0)
        if zc is not None:   # the per-sketch z projections, one grouped small-GEMM launch
            IN = p.W_x.shape[0]
            g = gemm.SmallGroup(self.dev)
            g.mm(zc.float().contiguous(), p.W_x[5:].detach(), out=self.ZP[:, :self.G])
            g.mm(zc.float().contiguous(), p.hyp_W_x[5:IN].detach(), out=self.ZP[:, self.G:])
            g.run()
        else:
            self.ZP.zero_()
        for cl in (self.clm, self.clh):
            if cl.on:
                cl.part.zero_()
        if x0 is not None and self.fused:
            self.X.copy_(x0)
        if self.fp8:   # the initial h's fp8 copy (later ones come from the main cell)
            mx8.quant_rows(self.A[:, :H], self.A8, self.SA)

    def _cell_args(self, t: int):
        p, w = self.model.dec, self._w
        B, H, Hh, G, Gh, K = self.B, self.H, self.Hh, self.G, self.Gh, self.K
        lnh = [t_.contiguous() for t_ in (p.hyp_ln_gamma, p.hyp_ln_beta, p.hyp_lnc_gamma, p.hyp_lnc_beta)]
        lnm = [t_.contiguous() for t_ in (p.ln_gamma, p.ln_beta, p.lnc_gamma, p.lnc_beta)]
        self._keep = lnh + lnm
        ah = LstmFwdArgs()
        ah.B, ah.H = B, Hh
        ah.xp, ah.ld_xp = self.XP[:, G:].data_ptr(), G + Gh
        ah.R, ah.ld_R, ah.R_nslab, ah.R_slab = self.RY.data_ptr(), Gh, self.S_y, B * Gh
        ah.ln_g, ah.ln_b, ah.lnc_g, ah.lnc_b = (x.data_ptr() for x in lnh)
        ah.forget_bias, ah.keep = 1.0, 1.0
        ah.seed, ah.stream, ah.step = self.sd.data_ptr(), 1, t
        ah.c_prev, ah.c_carry, ah.h_out = self.HCC.data_ptr(), self.HCC.data_ptr(), self.HH.data_ptr()
        ah.h_lp, ah.ld_lp, ah.lp_kind = self.A[:, H:].data_ptr(), K, 1
        self.clh.set(ah, t)
        am = LstmFwdArgs()
        am.B, am.H = B, H
        am.xp, am.ld_xp = self.XP.data_ptr(), G + Gh
        am.R, am.ld_R, am.R_nslab, am.R_slab = self.RM.data_ptr(), G, self.S_m, B * G
        if "PQ" in w:
            am.vec, am.vec_gs, am.vec_ld, am.vec_bias = self.VEC.data_ptr(), H, 12 * H, w["PQ"][1].data_ptr()
        am.bias = p.bias.data_ptr()
        am.ln_g, am.ln_b, am.lnc_g, am.lnc_b = (x.data_ptr() for x in lnm)
        am.forget_bias, am.keep = 1.0, 1.0
        am.seed, am.stream, am.step = self.sd.data_ptr(), 0, t
        am.c_prev, am.c_carry, am.h_out = self.CC.data_ptr(), self.CC.data_ptr(), self.Hout.data_ptr()
        am.h_lp, am.ld_lp, am.lp_kind = self.A.data_ptr(), K, 1
        if self.fp8:
            am.h_q8, am.ld_q8, am.h_qs = self.A8.data_ptr(), H, self.SA.data_ptr()
        self.clm.set(am, t)
        return ah, am

    @torch.no_grad()
    def step(self, x: torch.Tensor, t: int, sample) -> None:
        """One stroke: ``x [B, 5]`` (fp32, contiguous) -> decoder step -> head
        slabs -> ``sample(zs, ldz, nslab, slab, bias)`` (the caller's sampler)."""
        w = self._w
        PQ = self._pq()
        B, H, G, Gh = self.B, self.H, self.G, self.Gh
        st = torch.cuda.current_stream().cuda_stream
        rc = self.lib.skr_bproj_fwd(x.data_ptr(), w["W5"].data_ptr(), self.ZP.data_ptr(), self.XP.data_ptr(),
                                    1, B, 5, G + Gh, 0, st)
        if rc != 0:
            raise RuntimeError("skr_bproj_fwd failed (%d)" % rc)
        jobs = [(self.A[:, :H], w["WhT"], self.RM, self.S_m), (self.A, w["WyT"], self.RY, self.S_y)]
        gemm.rec_gemm_group(jobs)
        ah, am = self._cell_args(t)
        if self.lib.skr_lstm_fwd_step(ctypes.byref(ah), 1, 0, st) != 0:
            raise RuntimeError("hyper cell step failed")
        gemm.rec_gemm_bf16out(self.A[:, H:], PQ[0], self.VEC)
        prev = self.lib.skr_cell_set_oversub(1) if self.clm.oversub else None
        try:
            rc = self.lib.skr_lstm_fwd_step(ctypes.byref(am), 1, 2, st)
        finally:
            if prev is not None:
                self.lib.skr_cell_set_oversub(prev)
        if rc != 0:
            raise RuntimeError("main cell step failed (%d)" % rc)
        gemm.rec_gemm(self.A[:, :H], w["WoT"], self.ZS, self.S_o)
        sample(self.ZS, 128, self.S_o, B * 128, w["bo"])

    # -- four-launch stroke -------------------------------------------------------
    def sample_args(self, step: int, row0: int, out_row: torch.Tensor, done: torch.Tensor, seed: torch.Tensor,
                    M: int, mode: int, temp: float, greedy: bool, fix_pen: bool) -> DecodeSample:
        """Sampler of stroke ``step`` (written to ``out_row [B, 5]``, row
        stride ``out_row.stride(0)``) for :meth:`step_fused` of stroke step+1."""
        s = DecodeSample()
        s.active = 1
        s.zs, s.ldz, s.nslab, s.slab = self.ZS.data_ptr(), 128, self.S_o, self.B * 128
        s.bias, s.nout = self._w["bo"].data_ptr(), self.nout
        s.M, s.mode, s.temp, s.greedy, s.fix_pen = M, mode, float(temp), int(greedy), int(fix_pen)
        s.seed, s.step, s.row0 = seed.data_ptr(), step, row0
        s.out_row, s.ld_out = out_row.data_ptr(), out_row.stride(0)
        s.done = done.data_ptr()
        return s

    @torch.no_grad()
    def step_fused(self, t: int, smp: DecodeSample = None) -> None:
        """One stroke in four launches (module docstring). ``smp``: the sampler
        of stroke t-1 (:meth:`sample_args`), or None -- the stroke is
        ``self.X`` (t == 0, or teacher-forced)."""
        assert self.fused
        w, lib = self._w, self.lib
        B, H, Hh, G, Gh, K = self.B, self.H, self.Hh, self.G, self.Gh, self.K
        st = torch.cuda.current_stream().cuda_stream
        jobs = [(self.A, w["WyT"], self.RY, self.S_y)]
        if self.fp8:   # h W_h on the MX-fp8 GEMM, the rest grouped in bf16
            mx8.gemm(self.A8, self.SA, w["Wh8"][0], w["Wh8"][1], out=self.RM[0])
        else:
            jobs.insert(0, (self.A[:, :H], w["WhT"], self.RM, self.S_m))
        if smp is not None:
            jobs.append((self.A[:, :H], w["WoT"], self.ZS, self.S_o))
        gemm.rec_gemm_group(jobs)
        ah, am = self._cell_args(t)
        ah.xp = self.ZP[:, G:].data_ptr()          # z part; the stroke part is formed in the kernel
        if smp is None:
            smp = DecodeSample()
        rc = lib.skr_decode_hyper_cell(ctypes.byref(ah), ctypes.byref(smp), self.X.data_ptr(),
                                       w["W5"][:, G:].data_ptr(), G + Gh, st)
        if rc != 0:
            raise RuntimeError("skr_decode_hyper_cell failed (%d)" % rc)
        dec = ModDecode()
        dec.x5, dec.w5, dec.ldw5 = self.X.data_ptr(), w["W5"].data_ptr(), G + Gh
        dec.zp, dec.ldzp = self.ZP.data_ptr(), G + Gh
        from ..ops.hyper import apply_hm_zgrid
        apply_hm_zgrid(native.require_hip())
        rc = lib.skr_hyper_mod_fwd(self.A[:, H:].data_ptr(), K, w["PL"].data_ptr(),
                                   w["QB"].data_ptr(), None, self.RM.data_ptr(), B * G, self.S_m, None,
                                   self.GP.data_ptr(), None, self.GS.data_ptr(), B, H, Hh, ctypes.byref(dec), st)
        if rc != 0:
            raise RuntimeError("skr_hyper_mod_fwd (decode) failed (%d)" % rc)
        am.gpre, am.gstats, am.gstat_tiles = self.GP.data_ptr(), self.GS.data_ptr(), H // 32
        prev = lib.skr_cell_set_oversub(1) if self.clm.oversub else None
        try:
            rc = lib.skr_lstm_fwd_step(ctypes.byref(am), 1, 3, st)
        finally:
            if prev is not None:
                lib.skr_cell_set_oversub(prev)
        if rc != 0:
            raise RuntimeError("main cell step failed (%d)" % rc)

    @torch.no_grad()
    def head(self) -> None:
        """Head GEMM of the current ``h`` into the split-K slabs ``ZS``."""
        gemm.rec_gemm(self.A[:, :self.H], self._w["WoT"], self.ZS, self.S_o)
