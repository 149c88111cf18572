"""HyperLSTM sequence on the GPU (Ha et al. HyperNetworks, the sketch-rnn
decoder cell at vae_large width): per time step a grouped skinny GEMM
(``R_main = h @ W_h`` and ``R_hyp = [h | hh] @ W_y`` in one launch), the
LayerNorm hyper cell, the fused modulation step (``csrc/hyper_mod.hip``:
``vec = hh @ P + q``, the main gate pre-activations and their LayerNorm
partial sums) and the main LayerNorm cell; the backward mirrors it in
reverse and leaves every weight gradient to long-K GEMMs over the whole
sequence (``csrc/wgrad_gemm.hip``). The two-stage hyper-norm projections
``vec_k = (hh @ W_z_k + b_z_k) @ W_a_k`` are folded into ``vec = hh @ P + q``
with ``P = [W_z_k W_a_k]_k`` built once per call (``csrc/hyper_fold.hip``).

Reference recurrence: /root/reference model.py:66-95 (static unroll of the
decoder cell). Shared plumbing (argument structs, cell launchers, cluster
geometry, seeds) lives in :mod:`.recurrent`.
"""
from __future__ import annotations

import ctypes
import os

import torch

from ..utils import native
from . import gemm
from ._hipapi import LstmBwdArgs, LstmFwdArgs, ModDecode
from . import inproj
from .inproj import bproj_fwd, bproj_ok, bproj_reduce
from .recurrent import (ROW_STATS, _cell_bwd, _cell_fwd, _check, _ClusterSync, _inference, _ln_saves_lp, _lp_kind,
                        _ptr, _Saved, _seed_tensor, _stream, cell_geometry)
from .reduce import colsum_many

# The modulation GEMM fused with the main gates' pre-activations and
# LayerNorm partial sums (csrc/hyper_mod.hip). False (tests / shapes it does
# not take) keeps the plain bf16-output GEMM + the main cell's in-launch
# statistics exchange.
HYPER_MOD = True
HYPER_MAIN_C = 4   # workgroups per row of the MOD-3 main cell (0: policy; 4 measured 0.1 ms/step faster than the policy's 8, profiles/r6/main_cell_c_ab.log)
# Backward step as [main cell] -> [dvec P^T] -> [hyper cell + dR_main W_h^T in
# one launch, csrc/skinny_gemm.hip skr_skinny_gemm_group_cellbwd] -> [dR_hyp
# W_y^T]: the hyper cell (one workgroup per row) runs beside the tiles of the
# product only the next step reads. False (tests / shapes it does not take)
# keeps [main cell] -> [dR_main W_h^T + dvec P^T] -> [hyper cell] -> [dR_hyp W_y^T].
HYPER_BWD_FUSE = True
# Chained backward launch (csrc/chain_step.hip): the main-cell backward rows
# of step t run INSIDE the launch of step t + 1's dR_hyp W_y^T product (their
# other loads issued before an in-launch wait on the product's tiles): three
# launches per backward step instead of four. SKR_CHAIN=0 keeps the unchained
# launches (A/B).
CHAIN = os.environ.get("SKR_CHAIN", "1") != "0"
# Three-stage chained launch (csrc/chain_step.hip skr_chain_bwd_main3): the
# dvec P^T product of step t joins the chained launch too -- producer
# workgroups that finished their dR_hyp W_y^T tile stage their P^T slice in
# LDS while the main-cell rows compute, then run the tile on the rows' arrival
# counter: two launches per backward step instead of three. Bit-identical to
# the separate launch, but OFF: measured (profiles/r6/chain3_probe.jsonl, B =
# 100) 60.8 us per backward step against 50.9 for two-stage chain + separate
# launch. Producers that stay resident waiting on the rows cost 7.4 us by
# themselves (probe 3: no staging, no tile), and the tile tail -- 154 KB of
# dvec per workgroup through sc1 loads from the fabric -- another ~10 us,
# more than the 8 us launch it replaces. It also needs at least as many
# producer tiles as dvec P^T tail tiles: at SAY_CAP = 2 (below) the launch
# declines and the two-stage chain runs (the bitwise test pins SAY_CAP = 4).
CHAIN3 = False
# Workgroups per main-cell row in the chained backward launch (1 or 2): 2
# splits each row's ~300 KB of loads over two CUs and exchanges the two
# LayerNorm-backward row sums in-launch (csrc/chain_step.hip CL). Tested,
# 1 by default: measured 24.63 / 24.64 ms/step against 23.91 / 23.89
# (profiles/r6/chain_fwd_ab.log) -- the two exchanges (each both
# workgroups' arrival) cost more than the halved per-CU stream saves.
CHAIN_CL = 1
# Chained forward step (csrc/hyper_mod.hip skr_hyper_mod_chain): the main
# LayerNorm cell rows of step t run INSIDE step t's modulation launch -- every
# workgroup runs its modulation tile, arrives, and the first B * CHAIN_FWD_C
# then run the main cell over H / CHAIN_FWD_C units of one row (their c_prev
# and LayerNorm-parameter loads issued before the in-launch wait): three
# launches per forward step instead of four. Tested (oracle, poison, repeat),
# OFF: measured on MI355X (same box, A B C A B C, profiles/r6/chain_fwd_ab.log)
# 24.01 / 24.04 ms/step (C = 2) and 24.23 / 24.26 (C = 1) against 23.91 /
# 23.89 for the two launches: the chained launch takes 19.75 us per step
# against 10.5 + 8.8 for the pair -- the grid-wide arrival costs what the
# kernel boundary did, and the rows cannot keep the faster four-workgroup
# geometry (B * 4 > the 256 resident modulation workgroups).
CHAIN_FWD = False
CHAIN_FWD_C = 2
CHAIN_FWD_STATS = {"launches": 0}
# Debug (tests): NaN-fill the d[h | hh] slabs before every chained launch (and
# g / its partial sums before every chained forward launch), so a main-cell
# row that read them ahead of its producer tiles shows up as NaN.
CHAIN_POISON = False
# Hyper cell + modulation step in ONE forward launch (csrc/hyper_mod.hip
# hyper_cell_mod): wave 0 of modulation workgroup b runs the hyper cell of row
# b and publishes its hh row; every modulation tile fetches its P fragments,
# x-projection and R slabs while the rows compute, then waits for all rows
# (timing probes: the P fetch is 4.8 of the separate modulation launch's
# 10.9 us). 65 <= B <= 128. OFF: measured 28.2 us per launch against 4.9 + 10.9
# for the pair, vae_large 26.2 vs 23.65 ms/step (profiles/r6/cm2/): the
# one-wave hyper cell row takes ~11 us inside the launch (probes: no wait
# 24.9, no rows 13.5 us).
CELL_MOD = False
CELL_MOD_POISON = False   # tests: NaN-fill the hh rows before each such launch
CELL_MOD_STATS = {"launches": 0}
# The main input projection x W_x + z W_z ([T, B, 4H], the largest tensor the
# forward writes) stored in bf16 on the fused-modulation path; False keeps it
# fp32 (A/B, scripts/micro/xh_ab.py).
XH_BF16 = True
# The three long-K weight gradients of the backward (dW_h, dW_y, dP + its
# column sums) computed in T-chunks on a side stream WHILE the scan runs: once
# the scan has finished time steps [t, t + BG_CHUNK), their rows of dR_main /
# dR_hyp / dvec are final, and a bounded-grid launch (BG_GRID workgroups,
# csrc/wgrad_gemm.hip max_grid) adds that chunk's product into the gradient
# (fixed chunk order: deterministic); the last chunk runs at full width beside
# the post-scan reductions. OFF: measured on MI355X (round 6, same box, A B A B,
# profiles/r6/bg_wgrad_ab.log) 24.06 / 24.01 ms/step serial against 26.17 /
# 26.24 (64 workgroups), 28.60 / 28.42 (32) and 37.29 / 37.17 (16). The scan's
# own kernels slow only 2-5 % beside the side stream, but its 250-step span
# grows from ~10 to ~14 ms (profiles/r6/bg_wgrad_step_summary.txt): the gaps
# between its dependent launches widen while a second queue is active.
BG_WGRAD = False
BG_GRID = 32
BG_CHUNK = 50
# (Round 4 measured the hyper-norm projections unfolded -- vec = bf16(hh W_z)
# W_a + q forward, dz = dvec W_a^T / dh = dz W_z^T backward -- at 27.8 vs
# 24.6 ms per training step: W_z re-read from L2 by every workgroup costs more
# than the folded P it replaces; profiles/r4/unfold_ab.txt.)
# (Round 4 measured one-launch forward / backward steps -- R_hyp, hyper cell,
# h @ W_h and the modulation with in-launch hand-offs; the backward chain
# beside dR_main W_h^T -- at +1.5 / +3.8 ms per training step: every
# in-launch dependency level cost as much as a kernel boundary,
# profiles/r4/hyper_fused_step_ab.txt.)
# (The forward twin -- h W_y alone, then the hyper cell beside h W_h in one
# launch -- measured 0.15 ms/step slower on vae_large and was removed:
# profiles/r3/hyper_fused_cell_ab.txt.)


# Row blocks of a wide (B > 128) modulation launch run in parallel (0: all,
# one workgroup per block) or walked by HM_ZGRID workgroups per tile, each
# loading its P fragments once (csrc/hyper_mod.hip skr_hyper_mod_set_zgrid).
# Measured on GraphDecoder steps (profiles/r6/decode_wide_knobs_ab.jsonl):
# 1 walker per tile 0.146 vs 0.157 ms per step at B = 1024, 0.084 vs 0.090 at
# B = 512 (2: 0.148 / 0.087, 4: 0.153 / 0.089). Bit-identical.
HM_ZGRID = 1
_ZGRID_SET = [0]


def apply_hm_zgrid(lib) -> None:
    if HM_ZGRID != _ZGRID_SET[0]:
        lib.lib.skr_hyper_mod_set_zgrid(int(HM_ZGRID))
        _ZGRID_SET[0] = HM_ZGRID


SAY_CAP = 2   # split-K ceiling of dR_hyp W_y^T (backward; see _HyperSeq.backward)

# Split-K tuning knobs of the per-step products (sweeps set them from Python:
# "sm" h W_h, "sy" [h | hh] W_y, "sh" dvec P^T, "sam" dR_main W_h^T, "say"
# dR_hyp W_y^T); empty = the planned factors.
SPLITS = {}


def _split_override(name: str, planned: int, K: int) -> int:
    """Split-K factor of a per-step HyperLSTM product: the planned one, or
    ``SPLITS[name]`` when it divides K into whole 64-wide K tiles."""
    v = int(SPLITS.get(name, 0))
    return v if v > 0 and planned > 0 and K % (64 * v) == 0 else planned


def _fold_ok(H: int, Hh: int, E: int) -> bool:
    """Shapes of csrc/hyper_fold.hip (the vae_large / vae_classcond decoders)."""
    return H % 256 == 0 and Hh % 16 == 0 and 1 <= E <= 32


def _hyper_proj_grads(dP1, sV, s, Hh, H, E):
    """Hyper-norm projection gradients from ``dP1 = hh^T dvec`` and the
    column sums ``sV`` of dvec."""
    if dP1.is_cuda:   # per-block products as batched strided GEMMs over the 12 blocks (csrc/small_gemm.hip)
        dev = dP1.device
        dP1, sV = dP1.contiguous(), sV.contiguous()
        Wz, bz, Wa = (t.detach().contiguous() for t in (s.W_z, s.b_z, s.W_a))
        NC = 12 * H
        dW_z = torch.empty(Hh, 12 * E, device=dev)
        db_z = torch.empty(12 * E, device=dev)
        dWa = torch.empty(12, E, H, device=dev)
        # dW_a[j] = W_z[:, jE:(j+1)E]^T dP[:, jH:(j+1)H] + b_z[jE:(j+1)E] (x) sV[jH:(j+1)H]
        # dW_z[:, jE:(j+1)E] = dP[:, jH:(j+1)H] W_a[j]^T;  db_z[jE:(j+1)E] = sV[jH:(j+1)H] W_a[j]^T
        # (the three independent products in one launch, then the accumulation into dW_a)
        g = gemm.SmallGroup(dev)
        g.batched(bz, 0, E, 1, 0, sV, 0, H, 0, 1, dWa, 0, E * H, H, E, H, 1, 12)
        g.batched(dP1, 0, H, NC, 1, Wa, 0, E * H, 1, H, dW_z, 0, E, 12 * E, Hh, E, H, 12)
        g.batched(sV, 0, H, 0, 1, Wa, 0, E * H, 1, H, db_z, 0, E, 0, 1, E, H, 12)
        g.run()
        gemm.small_mm_batched(Wz, 0, E, 1, 12 * E, dP1, 0, H, NC, 1, dWa, 0, E * H, H, E, H, Hh, 12, acc=True)
        return dW_z, db_z, dWa, sV[8 * H:].reshape(4 * H)
    dP = dP1.view(Hh, 12, H).transpose(0, 1)                       # [12, Hh, H]
    sV = sV.view(12, H)
    Wz3 = s.W_z.view(Hh, 12, E).transpose(0, 1)                    # [12, Hh, E]
    dW_z = torch.bmm(dP, s.W_a.transpose(1, 2)).transpose(0, 1).reshape(Hh, 12 * E)
    dWa = torch.bmm(Wz3.transpose(1, 2), dP) + s.b_z.view(12, E, 1) * sV.view(12, 1, H)
    db_z = torch.bmm(sV.view(12, 1, H), s.W_a.transpose(1, 2)).reshape(12 * E)
    dbias = sV[8:].reshape(4 * H)                                  # shift-vector grads = bias grads
    return dW_z, db_z, dWa, dbias


class _HyperSeq(torch.autograd.Function):
    """HyperLSTM layer (LN main cell modulated by a LN hyper cell).

    Forward per step: [grouped GEMM R_main + R_hyp] -> [hyper cell] ->
    [vec = hh @ P + q] -> [main cell]; backward per step: [main cell bwd] ->
    [grouped GEMM dR_main W_h^T + dvec P^T] -> [hyper cell bwd] ->
    [dR_hyp W_y^T]; weight gradients are long-K GEMMs over all T*B rows after
    the scan. (A persistent one-launch forward was built in round 3 and
    measured slower, 45.6 vs 36.5 us per step: profiles/r3/hyper_persist_*.)
    """

    @staticmethod
    def forward(ctx, x, zc, h0, c0, hh0, hc0, seed, W_x, W_h, bias, hW_x, hW_h, hln_g, hln_b, hlnc_g, hlnc_b,
                W_z, b_z, W_a, ln_g, ln_b, lnc_g, lnc_b, meta):
        forget_bias, keep, hkeep, stream, E, infer = meta   # infer: no autograd graph is being built
        # unused outputs (the final states in training) get None grads, not
        # materialised zero tensors (fills + copies inside the captured step)
        ctx.set_materialize_grads(False)
        lib = native.require_hip()
        T, B, IX = x.shape                      # input = [x | zc broadcast over T]
        IN = W_x.shape[0]
        H, Hh = W_h.shape[0], hW_h.shape[0]
        G, Gh = 4 * H, 4 * Hh
        K = H + Hh
        dev = x.device
        f32 = torch.float32
        TB = T * B
        bp = bproj_ok(x) and not x.requires_grad
        xl = None
        if bp:   # stroke rows per position, z rows once per sequence (csrc/inproj.hip)
            zw = zwy = None
            if zc is not None:   # both z projections in one launch
                g = gemm.SmallGroup(dev)
                zw, zwy = g.mm(zc, W_x[IX:]), g.mm(zc, hW_x[IX:IN])
                g.run()
            XH = None   # (after the modulation-path choice below: bf16 when hyper_mod reads it)
            XHY = bproj_fwd(x, hW_x[:IX], zwy)
        else:
            if zc is not None:
                x = torch.cat([x, zc.unsqueeze(0).expand(T, B, zc.shape[-1])], -1)
            xl = gemm.lp(x.reshape(TB, IN).contiguous())
            if infer:
                XH = gemm.mm(xl, gemm.derived(W_x, "lp%s" % gemm.lp_dtype(), gemm.lp)).view(T, B, G)
                XHY = gemm.mm(xl, gemm.derived(hW_x, "lpx%d%s" % (IN, gemm.lp_dtype()),
                                               lambda W: gemm.lp(W[:IN]).contiguous())).view(T, B, Gh)
            else:
                XH = gemm.mm(xl, gemm.lp(W_x)).view(T, B, G)
                XHY = gemm.mm(xl, gemm.lp(hW_x[:IN])).view(T, B, Gh)
        dt = gemm.lp_dtype()

        def wy(hW_x, hW_h):                      # [K, Gh]: B^T of dR_hyp @ W_y^T
            return torch.cat([hW_x[IN:], hW_h], 0).to(dt).contiguous()

        def fold(W_z, b_z, W_a):                 # hyper-norm projections folded: vec = hh @ P + q
            Wz3 = W_z.view(Hh, 12, E).permute(1, 0, 2)                      # [12, Hh, E]
            P = torch.bmm(Wz3, W_a).permute(1, 0, 2).reshape(Hh, 12 * H)   # [Hh, 12H]
            q = torch.bmm(b_z.view(12, 1, E), W_a).reshape(12, H).contiguous()
            return P.to(dt).contiguous(), q

        qb_f = None
        if infer:
            Whl = Wyl = Pl = None
            WhT = gemm.derived(W_h, "hypWhT%s" % dt, lambda W: gemm.lp(W).t().contiguous())
            WyT = gemm.derived((hW_x, hW_h), "hypWyT%s" % dt, lambda a, b: wy(a, b).t().contiguous())
            PlT, q = gemm.derived((W_z, b_z, W_a), "hypP%s" % dt,
                                  lambda a, b, c: (lambda P, q: (P.t().contiguous(), q))(*fold(a, b, c)))
        elif dt == torch.bfloat16 and W_h.is_cuda:
            # both bf16 layouts of each weight in one pass (csrc/convert.hip)
            Whl, WhT = gemm.cast_transpose(W_h)  # [H, G]: B^T of dR_main @ W_h^T; [G, H]: B^T of h @ W_h
            Wyl = torch.empty(K, Gh, dtype=dt, device=dev)
            WyT = torch.empty(Gh, K, dtype=dt, device=dev)
            gemm.cast_transpose(hW_x[IN:], Wyl[:H], WyT[:, :H])
            gemm.cast_transpose(hW_h, Wyl[H:], WyT[:, H:])
            if _fold_ok(H, Hh, E):   # P and q in both bf16 layouts, one launch (csrc/hyper_fold.hip)
                Pl = torch.empty(Hh, 12 * H, dtype=dt, device=dev)
                PlT = torch.empty(12 * H, Hh, dtype=dt, device=dev)
                q = torch.empty(12, H, device=dev, dtype=f32)
                qb_f = torch.empty(12 * H, device=dev, dtype=f32)
                _check(lib.lib.skr_hyper_fold(W_z.detach().contiguous().data_ptr(), b_z.detach().contiguous().data_ptr(),
                                              W_a.detach().contiguous().data_ptr(), bias.detach().contiguous().data_ptr(),
                                              Hh, H, E, Pl.data_ptr(), PlT.data_ptr(), q.data_ptr(), qb_f.data_ptr(),
                                              _stream()), "hyper_fold")
            else:
                Wz3 = W_z.view(Hh, 12, E).permute(1, 0, 2)
                Pf = torch.bmm(Wz3, W_a).permute(1, 0, 2).reshape(Hh, 12 * H)
                q = torch.bmm(b_z.view(12, 1, E), W_a).reshape(12, H).contiguous()
                Pl, PlT = gemm.cast_transpose(Pf)    # B^T for the backward dvec @ P^T / the forward hh @ P
                qb_f = None
        else:
            Whl = gemm.lp(W_h).contiguous()      # [H, G]: B^T of dR_main @ W_h^T
            WhT = Whl.t().contiguous()           # [G, H]: B^T of h @ W_h
            Wyl = wy(hW_x, hW_h)
            WyT = Wyl.t().contiguous()           # [Gh, K]
            Pl, q = fold(W_z, b_z, W_a)          # B^T for the backward dvec @ P^T
            PlT = Pl.t().contiguous()            # B^T for the forward  hh @ P
        S_m = _split_override("sm", gemm.plan_splits(B, G, H, 1, dt), H)
        S_y = _split_override("sy", gemm.plan_splits(B, Gh, K, 1, dt), K)
        S_v = gemm.plan_splits(B, 12 * H, Hh, 1, dt, max_splits=1)
        rgemm = gemm.rec_gemm
        A = torch.empty(T + 1, B, K, device=dev, dtype=dt)
        A[0, :, :H].copy_(h0)
        A[0, :, H:].copy_(hh0)
        # modulation step fused with the gate pre-activations and their
        # LayerNorm partial sums (csrc/hyper_mod.hip, 128-row blocks: B <= 256
        # here): the main cell then needs no statistics exchange for the gates
        # (MOD 3) and VEC carries q (and the main bias in its shift block) --
        # the backward uses a zero vec_bias
        hm_ok = HYPER_MOD and dev.type == "cuda" and Hh == 256 and H % 32 == 0 and S_m in (1, 2, 4) and B <= 256
        # bf16 modulation vectors (the bf16-output GEMM takes <= 128 rows, hyper_mod 256)
        vbf = dt == torch.bfloat16 and S_v == 1 and (B <= 128 or hm_ok)
        # R_main: the backward re-reads it (the hyper-modulation gradient
        # dg * R) as the bf16 copy the main cell saves (RLP); with fp32 GEMM
        # operands the fp32 split-K slabs of every step are kept instead
        RLP = torch.empty(T, B, G, device=dev, dtype=torch.bfloat16) if (vbf and not infer) else None
        CC = torch.empty(T + 1, B, H, device=dev, dtype=f32)
        c0c = c0.contiguous()   # step 0 reads c0 / hc0 in place (CC[0], HCC[0] stay unused: no copies)
        HCC = torch.empty(T + 1, B, Hh, device=dev, dtype=f32)
        hc0c = hc0.contiguous()
        Hout = torch.empty(T, B, H, device=dev, dtype=f32)
        HH = torch.empty(T, B, Hh, device=dev, dtype=f32)
        # saves for the backward (both cells are LayerNorm cells: xhat / rstd /
        # chat; the kernels recompute the gate activations); none at inference
        slp = _ln_saves_lp(infer)
        sdt = torch.bfloat16 if slp else f32
        sv = (lambda *shape, dt=f32: None) if infer else (lambda *shape, dt=f32: torch.empty(*shape, device=dev, dtype=dt))
        mln_on = ln_g is not None   # LayerNorm main cell (use_layer_norm); the hyper cell always is one
        if mln_on:
            XHAT, RSTD, CHAT = sv(T, B, G, dt=sdt), sv(T, B, 5), sv(T, B, H, dt=sdt)
            ACT = COUT = None
        else:   # plain main cell: gate activations + c' (csrc/cell_fwd_body.h !LN saves)
            XHAT = RSTD = CHAT = None
            ACT, COUT = sv(T, B, G), sv(T, B, H)
        HXHAT, HRSTD, HCHAT = sv(T, B, Gh, dt=sdt), sv(T, B, 5), sv(T, B, Hh, dt=sdt)
        # modulation vectors in bf16 when the GEMMs are bf16 (read only by the main cells)
        VEC = torch.empty(T, B, 12 * H, device=dev, dtype=torch.bfloat16 if vbf else f32)
        sd = _seed_tensor(seed, dev)
        hln = [t.contiguous() for t in (hln_g, hln_b, hlnc_g, hlnc_b)]
        mln = [t.contiguous() for t in (ln_g, ln_b, lnc_g, lnc_b)] if mln_on else [None] * 4
        bias_c = bias.contiguous()
        RM = torch.empty(T if (RLP is None and not infer) else 1, max(S_m, 1), B, G, device=dev, dtype=f32)
        rmi = (lambda t: t) if RM.shape[0] == T else (lambda t: 0)
        RY = torch.empty(max(S_y, 1), B, Gh, device=dev, dtype=f32)
        mod = 2 if vbf else 1
        hmod = hm_ok and vbf
        if hmod:
            mod = 3
            if qb_f is not None:   # q + the main bias on the shift block, from the fold kernel
                qb = qb_f
            else:
                qb = q.detach().clone()
                qb[8:] += bias_c.detach().view(4, H)
                qb = qb.reshape(12 * H).contiguous()
            GP = torch.empty(B, G, device=dev, dtype=f32)
            GS = torch.empty(B, 4, H // 32, 2, device=dev, dtype=f32)
        if XH is None:
            # the main input projection [T, B, 4H]: bf16 on the fused-modulation
            # path (hyper_mod and the backward main cell read it as bf16 -- half
            # the bytes of the largest tensor the forward writes), else fp32
            XH = bproj_fwd(x, W_x[:IX], zw, bf16=hmod and XH_BF16)
        if hmod:
            XHc = XH.contiguous()
            xh_dec = ModDecode()
            xh_dec.xh_bf16 = int(XHc.dtype == torch.bfloat16)
        # hyper cell args (LN-LSTM, no modulation)
        ah = LstmFwdArgs()
        ah.save_lp = int(slp)
        ah.B, ah.H = B, Hh
        ah.ld_xp, ah.ld_R = Gh, Gh
        ah.R, ah.R_nslab, ah.R_slab = RY.data_ptr(), max(S_y, 1), B * Gh
        ah.ln_g, ah.ln_b, ah.lnc_g, ah.lnc_b = (t.data_ptr() for t in hln)
        ah.forget_bias, ah.keep = float(forget_bias), float(hkeep)
        ah.seed, ah.stream = sd.data_ptr(), int(stream) + 1
        ah.ld_lp, ah.lp_kind = K, _lp_kind(A)
        # main cell args (LN + modulation)
        am = LstmFwdArgs()
        am.save_lp = int(slp)
        am.B, am.H = B, H
        am.ld_xp, am.ld_R = G, G
        am.R_nslab, am.R_slab = max(S_m, 1), B * G
        am.vec_gs, am.vec_ld, am.vec_bias, am.bias = H, 12 * H, q.data_ptr(), bias_c.data_ptr()
        am.ln_g, am.ln_b, am.lnc_g, am.lnc_b = (_ptr(t) for t in mln)
        am.forget_bias, am.keep = float(forget_bias), float(keep)
        am.seed, am.stream = sd.data_ptr(), int(stream)
        am.ld_lp, am.lp_kind = K, _lp_kind(A)
        # chained modulation + main cell (one row block, LayerNorm main cell, no fp8 copy)
        chain_f = CHAIN_FWD and hmod and mln_on and B <= 128 and T >= 2 and H % max(CHAIN_FWD_C, 1) == 0
        cf = gemm.ChainCounters(dev, "hyp_fwd_m", T) if chain_f else None
        cell_mod = CELL_MOD and hmod and not chain_f and 65 <= B <= 128 and T >= 2 and Hh == 256 and \
            _lp_kind(A) == 1
        cmc = gemm.ChainCounters(dev, "hyp_cell_mod", T) if cell_mod else None
        clm = _ClusterSync(T, B, H, dev, ln=mln_on,
                           C=(max(CHAIN_FWD_C, 1) if chain_f else HYPER_MAIN_C) if hmod else 0)
        clh = _ClusterSync(T, B, Hh, dev)
        st = _stream()
        group = gemm.GROUPED and S_m >= 1 and S_y >= 1 and dt == torch.bfloat16

        def _main_saves(am, t):   # the backward's inputs from the main cell (none at inference)
            if infer:
                return
            if mln_on:
                am.xhat, am.rstd, am.chat = XHAT[t].data_ptr(), RSTD[t].data_ptr(), CHAT[t].data_ptr()
            else:
                am.act, am.c_out = ACT[t].data_ptr(), COUT[t].data_ptr()
        for t in range(T):
            clm.set(am, t)
            clh.set(ah, t)
            ah.xp, ah.c_prev, ah.step = XHY[t].data_ptr(), (hc0c if t == 0 else HCC[t]).data_ptr(), t
            ah.h_out = HH[t].data_ptr()
            if not infer:
                ah.xhat, ah.rstd, ah.chat = HXHAT[t].data_ptr(), HRSTD[t].data_ptr(), HCHAT[t].data_ptr()
            ah.h_lp, ah.c_carry = A[t + 1, :, H:].data_ptr(), HCC[t + 1].data_ptr()
            if group:   # R_main and R_hyp in one launch
                gemm.rec_gemm_group([(A[t, :, :H], WhT, RM[rmi(t)], S_m), (A[t], WyT, RY, S_y)])
            else:
                rgemm(A[t, :, :H], WhT, RM[rmi(t)], S_m)
                rgemm(A[t], WyT, RY, S_y)
            if not cell_mod:
                _cell_fwd(lib, ah, True, 0, st, "hyper_fwd_step")
            am.xp, am.R, am.vec = XH[t].data_ptr(), RM[rmi(t)].data_ptr(), VEC[t].data_ptr()
            am.r_lp = RLP[t].data_ptr() if (RLP is not None and not hmod) else None
            am.c_prev, am.step = (c0c if t == 0 else CC[t]).data_ptr(), t
            am.h_out = Hout[t].data_ptr()
            _main_saves(am, t)
            am.h_lp, am.c_carry = A[t + 1, :, :H].data_ptr(), CC[t + 1].data_ptr()
            if hmod:
                am.gpre, am.gstats, am.gstat_tiles = GP.data_ptr(), GS.data_ptr(), H // 32
            if chain_f:   # modulation tiles -> this step's main cell rows, one launch
                if CHAIN_POISON:
                    GP.fill_(float("nan"))
                    GS.fill_(float("nan"))
                rc = lib.lib.skr_hyper_mod_chain(A[t + 1, :, H:].data_ptr(), K, PlT.data_ptr(), qb.data_ptr(),
                                                 XHc[t].data_ptr(), xh_dec.xh_bf16, RM[rmi(t)].data_ptr(), B * G, S_m,
                                                 VEC[t].data_ptr(), _ptr(RLP[t] if RLP is not None else None),
                                                 ctypes.byref(am), ctypes.byref(cf.at(t)), st)
                if rc == 0:
                    CHAIN_FWD_STATS["launches"] += 1
                    continue
                if rc not in (-2, -3, -4, -8):
                    _check(rc, "hyper_mod_chain")
                # shape or residency not taken: two launches from here on (the
                # counters of launches 0 .. t-1 are cleared for the next sequence;
                # the cluster buffer keeps its C: the MOD-3 cell takes C = 2 too)
                chain_f = False
                cf.buf.zero_()
            if cell_mod:   # hyper cell rows + modulation tiles, one launch
                if CELL_MOD_POISON:
                    A[t + 1, :, H:].fill_(float("nan"))
                rc = lib.lib.skr_hyper_cell_mod(ctypes.byref(ah), PlT.data_ptr(), qb.data_ptr(), XHc[t].data_ptr(),
                                                xh_dec.xh_bf16, RM[rmi(t)].data_ptr(), B * G, S_m, VEC[t].data_ptr(),
                                                GP.data_ptr(), _ptr(RLP[t] if RLP is not None else None),
                                                GS.data_ptr(), H, ctypes.byref(cmc.at(t)), st)
                if rc == 0:
                    CELL_MOD_STATS["launches"] += 1
                    _cell_fwd(lib, am, mln_on, mod, st, "hyper_main_fwd_step")
                    continue
                if rc not in (-2, -3, -4):
                    _check(rc, "hyper_cell_mod")
                # not taken: the two launches from here on (counters cleared for the next sequence)
                cell_mod = False
                cmc.buf.zero_()
                _cell_fwd(lib, ah, True, 0, st, "hyper_fwd_step")
            if hmod:
                apply_hm_zgrid(lib)
                _check(lib.lib.skr_hyper_mod_fwd(A[t + 1, :, H:].data_ptr(), K, PlT.data_ptr(), qb.data_ptr(),
                                                 XHc[t].data_ptr(), RM[rmi(t)].data_ptr(), B * G, S_m,
                                                 VEC[t].data_ptr(), GP.data_ptr(), _ptr(RLP[t] if RLP is not None else None),
                                                 GS.data_ptr(), B, H, Hh, ctypes.byref(xh_dec), st), "hyper_mod_fwd")
            elif vbf:
                gemm.rec_gemm_bf16out(A[t + 1, :, H:], PlT, VEC[t])
            else:
                rgemm(A[t + 1, :, H:], PlT, VEC[t].unsqueeze(0), S_v)
            _cell_fwd(lib, am, mln_on, mod, st, "hyper_main_fwd_step")
        hT = Hout[T - 1].clone()    # no resets: the carried h is h'
        hhT = HH[T - 1].clone()
        s = _Saved()
        for k, v in dict(xl=xl, x=x, zc=zc, bp=bp, XH=XH, Whl=Whl, Wyl=Wyl, Pl=Pl, q=q, S_m=S_m, A=A, RM=RM,
                         RLP=RLP, CC=CC, HCC=HCC, c0=c0c, hc0=hc0c, XHAT=XHAT, RSTD=RSTD, CHAT=CHAT, HH=HH, HXHAT=HXHAT, HRSTD=HRSTD,
                         HCHAT=HCHAT, VEC=VEC, seed=sd, meta=meta, slp=slp, W_h=W_h, W_x=W_x, hW_x=hW_x, hW_h=hW_h, W_z=W_z,
                         b_z=b_z, W_a=W_a,
                         mln=mln, hln=hln, vec_folded=hmod, mln_on=mln_on, ACT=ACT, COUT=COUT).items():
            setattr(s, k, v)
        ctx.s = s
        ctx.dims = (T, B, IX, IN, H, Hh, E)
        if A.dtype == torch.bfloat16:
            # the bf16 copy of every h the next step's GEMM read: the fused MDN
            # head reads it instead of Hout (ops.mdn_hip, same bf16 operands)
            Hout._skr_lp = A[1:, :, :H]
        # (views of internal buffers nothing writes again)
        return Hout, hT, (CC[T] if T > 0 else c0c), hhT, (HCC[T] if T > 0 else hc0c)

    @staticmethod
    def backward(ctx, dHout, dhT, dcT, dhhT, dhcT):
        s = ctx.s
        T, B, IX, IN, H, Hh, E = ctx.dims
        forget_bias, keep, hkeep, stream, _, _ = s.meta
        lib = native.require_hip()
        dev = s.A.device
        f32 = torch.float32
        G, Gh = 4 * H, 4 * Hh
        K = H + Hh
        TB = T * B
        lp_on = s.Whl.dtype == torch.bfloat16
        ldt = torch.bfloat16 if lp_on else f32
        # d(recurrent pre-activations): only GEMM operands downstream, so with
        # bf16 operands the cell kernels write the bf16 copy alone
        dRM = None if lp_on else torch.empty(T, B, G, device=dev, dtype=f32)
        dRY = None if lp_on else torch.empty(T, B, Gh, device=dev, dtype=f32)
        dRM_lp = torch.empty(T, B, G, device=dev, dtype=ldt) if lp_on else dRM
        dRY_lp = torch.empty(T, B, Gh, device=dev, dtype=ldt) if lp_on else dRY
        dXH = torch.empty(T, B, G, device=dev, dtype=ldt)   # only a GEMM operand downstream
        sdt = torch.bfloat16 if s.slp else f32
        DLNY = torch.empty(T, B, G, device=dev, dtype=sdt) if s.mln_on else None
        DLNCY = torch.empty(T, B, H, device=dev, dtype=sdt) if s.mln_on else None
        HDLNY = torch.empty(T, B, Gh, device=dev, dtype=sdt)
        HDLNCY = torch.empty(T, B, Hh, device=dev, dtype=sdt)
        dVEC = torch.empty(T, B, 12 * H, device=dev, dtype=ldt)
        clh_C = cell_geometry(Hh, B, True) if lp_on else 0
        bfuse = HYPER_BWD_FUSE and lp_on and dev.type == "cuda" and Hh <= 256 and clh_C == 1 and \
            gemm.plan_splits(B, H, G, 1, ldt) >= 1
        # dvec P^T: the planned 32 splits also in the fused order (64 measured
        # 0.15 ms/step slower: 25.03 / 25.00 vs 24.83 / 24.88, profiles/r3/hyper_fused_cell_ab.txt)
        S_h = _split_override("sh", gemm.plan_splits(B, Hh, 12 * H, 1, ldt), 12 * H)
        S_am = _split_override("sam", gemm.plan_splits(B, H, G, 1, ldt), G)
        # d[h | hh] = dR_hyp @ W_y^T: at most SAY_CAP split-K slabs -- the next
        # step's two cells read every slab (the main-cell rows with sc1 loads
        # inside the chained launch); measured on MI355X (vae_large, same box):
        # round 3, 4 slabs 26.67 / 26.57 vs 8 (the plan) 26.76 / 26.86 ms/step;
        # round 6 (profiles/r6/hyper_splits2_ab.log, A B C D x3), 2 slabs
        # 23.67 / 23.68 / 23.69 vs 4 23.89 / 23.91 / 23.86, 1 slab 24.46-24.48
        S_ay = gemm.plan_splits(B, K, Gh, 1, ldt)
        if S_ay > SAY_CAP:
            S_ay = next(d for d in (SAY_CAP, 4, 3, 2, 1) if d <= SAY_CAP and (Gh // 64) % d == 0)
        S_ay = _split_override("say", S_ay, Gh)
        DHZ = torch.empty(max(S_h, 1), B, Hh, device=dev, dtype=f32)    # slabs of dhh from the vec path
        # dh slabs of step t + 1 read by step t; the last step reads none (null
        # sources) unless gradients flow into the final states
        fin = dhT is not None or dhhT is not None
        alloc = torch.zeros if (fin or T == 0) else torch.empty
        DAM = alloc(max(S_am, 1), B, H, device=dev, dtype=f32)    # slabs of dh from the main gates
        DAY = alloc(max(S_ay, 1), B, K, device=dev, dtype=f32)    # slabs of d[h | hh] from the hyper gates
        if dhT is not None:
            DAY[0, :, :H].copy_(dhT)
        if dhhT is not None:
            DAY[0, :, H:].copy_(dhhT)
        dc_rec = dcT.contiguous().clone() if dcT is not None else torch.zeros(B, H, device=dev, dtype=f32)
        dhc_rec = dhcT.contiguous().clone() if dhcT is not None else torch.zeros(B, Hh, device=dev, dtype=f32)
        dHout = dHout.contiguous() if dHout is not None else None
        am = LstmBwdArgs()
        am.save_lp = int(s.slp)
        am.B, am.H = B, H
        am.dh_rec, am.ld_dh_rec, am.dhr_nslab, am.dhr_slab = DAY.data_ptr(), K, max(S_ay, 1), B * K
        am.dh_rec2, am.ld_dh_rec2, am.dhr2_nslab, am.dhr2_slab = DAM.data_ptr(), H, max(S_am, 1), B * H
        am.dc_rec, am.dho_nslab = dc_rec.data_ptr(), 1
        am.ln_g, am.lnc_g, am.lnc_b = _ptr(s.mln[0]), _ptr(s.mln[2]), _ptr(s.mln[3])
        am.ln_b, am.forget_bias = _ptr(s.mln[1]), float(forget_bias)
        am.ld_xp, am.ld_R = G, G
        am.R_nslab, am.R_slab = max(s.S_m, 1), B * G
        # csrc/hyper_mod.hip folds q into the saved vectors: no bias to add (and
        # none to load -- 64 KB per row of the main-cell backward)
        am.vec_gs, am.vec_ld, am.vec_bias = H, 12 * H, None if s.vec_folded else s.q.data_ptr()
        am.keep, am.seed, am.stream = float(keep), s.seed.data_ptr(), int(stream)
        am.ld_dG, am.ld_dG_lp, am.dG_lp_kind = G, G, 1 if lp_on else 0
        am.ld_dxp, am.dxp_kind, am.dvec_kind = G, 1 if lp_on else 2, 1 if lp_on else 2
        ah = LstmBwdArgs()
        ah.save_lp = int(s.slp)
        ah.B, ah.H = B, Hh
        ah.dh_out, ah.dho_nslab, ah.dho_slab = DHZ.data_ptr(), max(S_h, 1), B * Hh
        ah.dh_rec, ah.ld_dh_rec, ah.dc_rec = DAY[0, :, H:].data_ptr(), K, dhc_rec.data_ptr()
        ah.dhr_nslab, ah.dhr_slab = max(S_ay, 1), B * K
        ah.ln_g, ah.lnc_g, ah.lnc_b = s.hln[0].data_ptr(), s.hln[2].data_ptr(), s.hln[3].data_ptr()
        ah.ln_b, ah.forget_bias = s.hln[1].data_ptr(), float(forget_bias)
        ah.keep, ah.seed, ah.stream = float(hkeep), s.seed.data_ptr(), int(stream) + 1
        ah.ld_dG, ah.ld_dG_lp, ah.dG_lp_kind = Gh, Gh, 1 if lp_on else 0
        clm, clh = _ClusterSync(T, B, H, dev, ln=s.mln_on), _ClusterSync(T, B, Hh, dev)
        st = _stream()
        group = lp_on and gemm.GROUPED and S_am >= 1 and S_h >= 1
        first = not fin   # (the last time step runs first)
        # chained launch (csrc/chain_step.hip): the main cell of step t inside
        # the dR_hyp W_y^T launch of step t + 1 (row kernel geometry: H = 2048,
        # bf16 vectors, LayerNorm main cell)
        chain_m = CHAIN and lp_on and dev.type == "cuda" and T >= 3 and H == 2048 and s.mln_on and \
            s.VEC.dtype == torch.bfloat16 and s.RLP is not None and dHout is not None and S_ay <= 8
        cm = gemm.ChainCounters(dev, "hyp_bwd_m", T - 1) if chain_m else None
        # three-stage launches (CHAIN3): dvec P^T inside the chained launch, on
        # the rows' own rotating counters; the bf16 fused-order backward only
        chain3 = chain_m and CHAIN3 and bfuse
        if chain_m and CHAIN_CL == 2 and not chain3:   # two workgroups per chained row (exchange buffer C = 2)
            clm = _ClusterSync(T, B, H, dev, ln=s.mln_on, C=2)
        cm3 = gemm.ChainCounters(dev, "hyp_bwd_m3", T - 1) if chain3 else None
        # weight gradients beside the scan (BG_WGRAD): destinations allocated
        # here, on the scan's stream; chunks [t, hi) issued as the scan passes t
        A2 = s.A[:T].reshape(TB, K)
        HHl = s.A[1:T + 1].reshape(TB, K)[:, H:] if lp_on else s.HH.view(TB, Hh)
        bg = None
        if BG_WGRAD and lp_on and dev.type == "cuda" and T >= 2 * BG_CHUNK and gemm._wgrad_hip_ok(A2[:, :H], dRM_lp.view(TB, G)) \
                and gemm._wgrad_hip_ok(A2, dRY_lp.view(TB, Gh)) and gemm._wgrad_hip_ok(HHl, dVEC.view(TB, 12 * H)):
            bg = gemm.Background(dev)
            dW_h = gemm.grad_slot(s.W_h, (H, G))
            dW_h = dW_h if dW_h is not None else torch.empty(H, G, device=dev, dtype=f32)
            dW_y = torch.empty(K, Gh, device=dev, dtype=f32)
            dP1 = torch.empty(Hh, 12 * H, device=dev, dtype=f32)
            sV = torch.empty(12 * H, device=dev, dtype=f32)
            bg_hi, bg_first = T, True

            def bg_chunk(lo, hi, first, grid):
                r0, r1 = lo * B, hi * B
                gemm.wgrad(A2[r0:r1, :H], dRM_lp.view(TB, G)[r0:r1], out=dW_h, acc=not first, max_grid=grid)
                gemm.wgrad(A2[r0:r1], dRY_lp.view(TB, Gh)[r0:r1], out=dW_y, acc=not first, max_grid=grid)
                gemm.wgrad(HHl[r0:r1], dVEC.view(TB, 12 * H)[r0:r1], colsum=True, out=dP1, cs_out=sV,
                           acc=not first, max_grid=grid)
        for t in range(T - 1, -1, -1):
            clm.set(am, t)
            clh.set(ah, t)
            if t == T - 1 or t == T - 2:   # null dh sources on the first backward step only
                am.dh_rec = None if (first and t == T - 1) else DAY.data_ptr()
                am.dh_rec2 = None if (first and t == T - 1) else DAM.data_ptr()
                ah.dh_rec = None if (first and t == T - 1) else DAY[0, :, H:].data_ptr()
            am.dh_out = dHout[t].data_ptr() if dHout is not None else None
            am.c_prev = (s.c0 if t == 0 else s.CC[t]).data_ptr()
            if s.mln_on:
                am.xhat, am.rstd, am.chat = s.XHAT[t].data_ptr(), s.RSTD[t].data_ptr(), s.CHAT[t].data_ptr()
                am.dlny, am.dlncy = DLNY[t].data_ptr(), DLNCY[t].data_ptr()
            else:
                am.act, am.c_new = s.ACT[t].data_ptr(), s.COUT[t].data_ptr()
            am.xp, am.vec = s.XH[t].data_ptr(), s.VEC[t].data_ptr()
            am.xp_lp = int(s.XH.dtype == torch.bfloat16)
            if s.RLP is not None:
                am.R, am.r_lp = None, s.RLP[t].data_ptr()
            else:
                am.R, am.r_lp = s.RM[t].data_ptr(), None
            am.step = t
            am.dG = None if lp_on else dRM[t].data_ptr()
            am.dG_lp = dRM_lp[t].data_ptr() if lp_on else None
            am.dxp, am.dvec = dXH[t].data_ptr(), dVEC[t].data_ptr()
            ran = ran3 = False
            if chain_m and t < T - 1:   # dR_hyp W_y^T of step t + 1 -> this main cell, one launch
                if CHAIN_POISON:
                    DAY.fill_(float("nan"))
                    if chain3:
                        dVEC[t].fill_(float("nan"))
                if chain3:   # ... -> dvec P^T of this step, the same launch
                    ran3 = gemm.chain_bwd_main3([(dRY_lp[t + 1], s.Wyl, DAY, S_ay)], (dVEC[t], s.Pl, DHZ, S_h), am,
                                                cm.at(T - 2 - t), cm3.at(T - 2 - t)) == 0
                    if not ran3:
                        chain3 = False
                        cm3.buf.zero_()
                    ran = ran3
                if not ran:
                    ran = gemm.chain_bwd_main([(dRY_lp[t + 1], s.Wyl, DAY, S_ay)], am, cm.at(T - 2 - t)) == 0
                if not ran:   # shape not taken by the chained row: unchained launches from here on
                    chain_m = False
                    # launches 0 .. k-1 left counts in their counters (only launch
                    # n - 1 clears counter 0): reset, so the next sequence starts clean
                    cm.buf.zero_()
                    gemm.rec_gemm(dRY_lp[t + 1], s.Wyl, DAY, S_ay)
                else:
                    ROW_STATS["chain"] += 1
                    ROW_STATS["chain3"] += int(ran3)
            if not ran:
                _cell_bwd(lib, am, s.mln_on, 2 if s.VEC.dtype == torch.bfloat16 else 1, st, "hyper_main_bwd_step")
            ah.c_prev = (s.hc0 if t == 0 else s.HCC[t]).data_ptr()
            ah.xhat, ah.rstd, ah.chat = s.HXHAT[t].data_ptr(), s.HRSTD[t].data_ptr(), s.HCHAT[t].data_ptr()
            ah.step = t
            ah.dG = None if lp_on else dRY[t].data_ptr()
            ah.dG_lp = dRY_lp[t].data_ptr() if lp_on else None
            ah.dlny, ah.dlncy = HDLNY[t].data_ptr(), HDLNCY[t].data_ptr()
            if bfuse:   # dvec P^T, then the hyper cell beside dR_main W_h^T (one launch)
                if not ran3:   # (chained: ran in the launch above)
                    gemm.rec_gemm(dVEC[t], s.Pl, DHZ, S_h)
                gemm.rec_gemm_group_cellbwd([(dRM_lp[t], s.Whl, DAM, S_am)], ah)
                ROW_STATS["cluster"] += 1   # (the clustered cell body, C = 1)
            else:
                if group:   # dR_main @ W_h^T and dvec @ P^T in one launch
                    gemm.rec_gemm_group([(dRM_lp[t], s.Whl, DAM, S_am), (dVEC[t], s.Pl, DHZ, S_h)])
                else:
                    gemm.rec_gemm(dRM_lp[t], s.Whl, DAM, S_am)
                    gemm.rec_gemm(dVEC[t], s.Pl, DHZ, S_h)
                _cell_bwd(lib, ah, True, 0, st, "hyper_bwd_step")
            if not chain_m or t == 0:   # (chained: runs in the next main-cell launch)
                gemm.rec_gemm(dRY_lp[t], s.Wyl, DAY, S_ay)
            if bg is not None and t > 0 and bg_hi - t >= BG_CHUNK:   # rows [t, bg_hi) are final
                bg.run(lambda lo=t, hi=bg_hi, f=bg_first: bg_chunk(lo, hi, f, BG_GRID))
                bg_hi, bg_first = t, False
        if bg is not None:   # the last chunk at full width, beside the reductions below
            bg.run(lambda: bg_chunk(0, bg_hi, bg_first, 0))
        if not DAY.is_cuda:
            dh0 = DAY[:, :, :H].sum(0) + DAM.sum(0)
            dhh0 = DAY[:, :, H:].sum(0)
        else:   # the initial-state gradients from step 0's dh slabs, one launch each (csrc/reduce.hip)
            dh0 = torch.empty(B, H, device=dev, dtype=f32)
            dhh0 = torch.empty(B, Hh, device=dev, dtype=f32)
            _check(lib.lib.skr_slab_sum2(DAY.data_ptr(), DAY.shape[0], B * K, K, DAM.data_ptr(), DAM.shape[0], B * H, H,
                                         B, H, dh0.data_ptr(), st), "slab_sum2 dh0")
            _check(lib.lib.skr_slab_sum2(DAY[0, :, H:].data_ptr(), DAY.shape[0], B * K, K, None, 0, 0, 0, B, Hh,
                                         dhh0.data_ptr(), st), "slab_sum2 dhh0")
        # weight / LayerNorm-parameter gradients: long-K products over the T*B saved rows
        # hyper-norm projections, vec_k = (hh @ W_z_k + b_z_k) @ W_a_k: ONE long-K
        # GEMM dP = hh^T @ dvec gives dP_k = hh^T dvec_k, and the same pass over
        # dvec its column sums; the per-k factors are then tiny batched products.
        # (hh_t rows, HHl: the bf16 GEMM operand of step t + 1 -- no resets on
        # this path, so it is exactly bf16(HH[t]) -- no conversion pass)
        # dW_y = [dW_y_h; dW_y_hh] straight into the arena when hW_x's slot (rows
        # IN..) and hW_h's follow each other there: no gather copy afterwards
        dW_y_arena = None if (bg is not None or s.hW_x.shape[0] != IN + H) else \
            gemm.grad_span(s.hW_x, s.hW_h, IN * Gh, (K, Gh))
        if bg is None:
            dW_h = gemm.wgrad(A2[:, :H], dRM_lp.view(TB, G), out=gemm.grad_slot(s.W_h, (H, G)))
            dW_y = gemm.wgrad(A2, dRY_lp.view(TB, Gh), out=dW_y_arena)
            dP1, sV = gemm.wgrad(HHl, dVEC.view(TB, 12 * H), colsum=True)
        # the four LayerNorm gamma / beta reductions in two launches (csrc/reduce.hip)
        lnp = [(DLNY, s.XHAT, G), (DLNCY, s.CHAT, H)] if DLNY is not None else []
        lnp += [(HDLNY, s.HXHAT, Gh), (HDLNCY, s.HCHAT, Hh)]
        sums = colsum_many([(dy.view(-1, n), xh.view(-1, n)) for dy, xh, n in lnp])
        flat = [v for pr in sums for v in pr]
        if DLNY is None:   # plain main cell: no LayerNorm parameters
            g_ln, g_hln = [None] * 4, flat
        else:
            g_ln, g_hln = flat[:4], flat[4:]
        if dW_y_arena is not None:   # the slots themselves (fresh views: autograd adopts them, no copies)
            dhW_x, dhW_h = gemm.grad_slot(s.hW_x, tuple(s.hW_x.shape)), gemm.grad_slot(s.hW_h, tuple(s.hW_h.shape))
        else:
            dhW_x, dhW_h = torch.empty_like(s.hW_x), None
        dx = dzc = None
        if s.bp:   # input-side gradients from one read of dXH / dR_hyp each
            if s.zc is not None and not inproj.GROUPED_REDUCE:
                S_m, P_m = bproj_reduce(s.x, dXH)
                S_y, P_y = bproj_reduce(s.x, dRY_lp)
                dW_x = gemm.grad_slot(s.W_x, tuple(s.W_x.shape))
                dW_x = torch.empty_like(s.W_x) if dW_x is None else dW_x
                dW_x[:IX] = P_m
                dhW_x[:IX] = P_y
                g = gemm.SmallGroup(dev)
                g.mm(s.zc.t(), S_m, out=dW_x[IX:])
                g.mm(s.zc.t(), S_y, out=dhW_x[IX:IN])
                dzc = g.mm(S_m, s.W_x[IX:].t())
                g.run()
                gemm.small_mm(S_y, s.hW_x[IX:IN].t(), out=dzc, acc=True)
            elif s.zc is not None:
                S_m, P_m = bproj_reduce(s.x, dXH, raw=True)      # P: per-row partials [B, IX, *]
                S_y, P_y = bproj_reduce(s.x, dRY_lp, raw=True)
                dW_x = gemm.grad_slot(s.W_x, tuple(s.W_x.shape))
                dW_x = torch.empty_like(s.W_x) if dW_x is None else dW_x
                one = gemm.ones_row(B, dev)
                g = gemm.SmallGroup(dev)   # the row sums of P and the three z-side products in one launch
                g.mm(one, P_m.view(B, IX * G), out=dW_x[:IX].view(1, IX * G))
                g.mm(one, P_y.view(B, IX * Gh), out=dhW_x[:IX].view(1, IX * Gh))
                g.mm(s.zc.t(), S_m, out=dW_x[IX:])
                g.mm(s.zc.t(), S_y, out=dhW_x[IX:IN])
                dzc = g.mm(S_m, s.W_x[IX:].t())
                g.run()
                gemm.small_mm(S_y, s.hW_x[IX:IN].t(), out=dzc, acc=True)
            else:
                S_m, dW_x = bproj_reduce(s.x, dXH)
                S_y, dhW_x[:IN] = bproj_reduce(s.x, dRY_lp)
        else:
            dXHl, dXHYl = gemm.lp(dXH.view(TB, G)), gemm.lp(dRY_lp.view(TB, Gh))
            dW_x = gemm.wgrad(s.xl, dXHl)
            dhW_x[:IN] = gemm.wgrad(s.xl, dXHYl)
            dxf = gemm.mm(dXHl, gemm.lp(s.W_x).t())
            dxf += gemm.mm(dXHYl, gemm.lp(s.hW_x[:IN]).t())
            dxf = dxf.view(T, B, IN)
            if s.zc is not None:
                dx, dzc = dxf[..., :IX], dxf[..., IX:].sum(0)
            else:
                dx = dxf
        if bg is not None:   # the side stream's products are complete from here on
            bg.join()
        if dW_y_arena is None:
            dhW_x[IN:] = dW_y[:H]
            dhW_h = dW_y[H:]
        dW_z, db_z, dWa, dbias = _hyper_proj_grads(dP1, sV, s, Hh, H, E)
        ctx.s = None
        return (dx, dzc, dh0, dc_rec, dhh0, dhc_rec, None, dW_x, dW_h, dbias, dhW_x, dhW_h,
                g_hln[0], g_hln[1], g_hln[2], g_hln[3], dW_z, db_z, dWa, g_ln[0], g_ln[1], g_ln[2], g_ln[3], None)


def hyper_sequence_hip(p, x, h0, c0, hh0, hc0, forget_bias=1.0, drop_keep=1.0, drop_seed=0, drop_stream=0,
                       hyp_drop_keep=1.0, zc=None):
    ln = [p.ln_gamma, p.ln_beta, p.lnc_gamma, p.lnc_beta] if p.use_layer_norm else [None] * 4
    outs = _HyperSeq.apply(x, zc, h0, c0, hh0, hc0, drop_seed, p.W_x, p.W_h, p.bias, p.hyp_W_x, p.hyp_W_h,
                           p.hyp_ln_gamma, p.hyp_ln_beta, p.hyp_lnc_gamma, p.hyp_lnc_beta, p.W_z, p.b_z, p.W_a,
                           *ln,
                           (float(forget_bias), float(drop_keep), float(hyp_drop_keep), int(drop_stream), p.embed,
                            _inference(x, zc, h0, p.W_h, p.W_x)))
    Hout, hT, cT, hhT, hcT = outs
    return Hout, (hT, cT, hhT, hcT)
