// Backward cell step of the LSTM-family cell kernels as a device function,
// shared by the per-step cell launch (csrc/lstm_cell.hip: workgroup (c, b) =
// (blockIdx.x, blockIdx.y)) and the grouped GEMM launch that runs the
// HyperLSTM hyper cell's backward beside the dR_main W_h^T tiles
// (csrc/skinny_gemm.hip, skr_skinny_gemm_group_cellbwd). Semantics and
// geometry: csrc/lstm_cell.hip header comment.
#pragma once
#include "cell_fwd_body.h"

namespace {

using namespace skr;

// DHS > 0: the dh split-K sources are loaded up front with compile-time
// ceilings (slab_load) -- DHS slabs for dh_out, kRecSlabs for dh_rec /
// dh_rec2; 0: runtime-count loops (any count).
template <int NT, int UPT, int NS, bool LN, int MOD, int DHS = 0>
__device__ __forceinline__ void cell_bwd_body(const BwdArgs& a, const int c, const int b, const int C) {
    constexpr int NW = NT / 64;
    __shared__ float lds[NW * 8];
    __shared__ float mine[8];
    __shared__ float all[kMaxCluster * 8];
    const int tid = threadIdx.x, H = a.H;
    const int span = UPT * NT, base = c * span;
    const int grp = a.grp_rows > 0 ? b / a.grp_rows : 0;
    const float* ln_g = LN ? a.ln_g + grp * 4 * H : nullptr;
    const float* ln_b = LN ? a.ln_b + grp * 4 * H : nullptr;
    const float* lnc_g = LN ? a.lnc_g + grp * H : nullptr;
    const float* lnc_b = LN ? a.lnc_b + grp * H : nullptr;
    const bool keep_on = a.keep < 1.0f;
    const uint32_t key = keep_on ? hash_key(*a.seed, a.stream, a.step) : 0u;
    const bool r = a.reset != nullptr && a.reset[b] != 0.f;

    // ---- every load up front
    float dhc[UPT], dho[UPT], dcc[UPT], ac[UPT][4], cp[UPT], cx[UPT], lcg[UPT], lcb[UPT];
    float xh[UPT][4], lg[UPT][4], lb[UPT][4], xv[UPT][4], rv[UPT][4], ax[UPT][4], ah[UPT][4];
    constexpr int D = DHS > 0 ? DHS : 1, DR = DHS > 0 ? kRecSlabs : 1;
    float t1[UPT][DR], t2[UPT][DR], t3[UPT][D];   // DHS > 0: raw dh slab loads, folded after all loads
    bool on[UPT];
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
        const int u = base + k * NT + tid;
        on[k] = u < H;
        const int uc = min(u, H - 1);
        const int64_t ro = (int64_t)b * H + uc;
        if constexpr (DHS > 0) {
            slab_load<DR>(a.dh_rec, b * a.ld_dh_rec + uc, a.dhr_nslab, a.dhr_slab, t1[k]);
            slab_load<DR>(a.dh_rec2, b * a.ld_dh_rec2 + uc, a.dhr2_nslab, a.dhr2_slab, t2[k]);
            slab_load<D>(a.dh_out, ro, a.dho_nslab, a.dho_slab, t3[k]);
        } else {
            dhc[k] = (a.dh_rec ? slab_sum<0>(a.dh_rec, b * a.ld_dh_rec + uc, a.dhr_nslab, a.dhr_slab) : 0.f) +
                     (a.dh_rec2 ? slab_sum<0>(a.dh_rec2, b * a.ld_dh_rec2 + uc, a.dhr2_nslab, a.dhr2_slab) : 0.f);
            dho[k] = a.dh_out ? slab_sum<0>(a.dh_out, ro, a.dho_nslab, a.dho_slab) : 0.f;
        }
        dcc[k] = a.dc_rec[ro];
        cp[k] = a.c_prev[ro];
        if (LN) {
            cx[k] = ld_save(a.chat, ro, a.save_lp);
            lcg[k] = lnc_g[uc];
            lcb[k] = lnc_b[uc];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                xh[k][q] = ld_save(a.xhat, (int64_t)b * 4 * H + q * H + uc, a.save_lp);
                lg[k][q] = ln_g[q * H + uc];
                lb[k][q] = ln_b[q * H + uc];
            }
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) ac[k][q] = a.act[(int64_t)b * 4 * H + q * H + uc];
            cx[k] = a.c_new[ro];
        }
        if (MOD) {
            const int64_t vo = (int64_t)b * a.vec_ld + uc;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                xv[k][q] = a.xp_lp ? __bfloat162float(((const __hip_bfloat16*)a.xp)[b * a.ld_xp + q * H + uc])
                                   : a.xp[b * a.ld_xp + q * H + uc];
                rv[k][q] = a.r_lp != nullptr ? __bfloat162float(a.r_lp[b * a.ld_R + q * H + uc])
                                             : slab_sum<NS>(a.R, b * a.ld_R + q * H + uc, a.R_nslab, a.R_slab);
                // (vec_bias null: the saved vectors already carry q, csrc/hyper_mod.hip)
                ax[k][q] = ldvec<MOD>(a.vec, q * a.vec_gs + vo) + (a.vec_bias ? a.vec_bias[q * H + uc] : 0.f);
                ah[k][q] = ldvec<MOD>(a.vec, (4 + q) * a.vec_gs + vo) + (a.vec_bias ? a.vec_bias[(4 + q) * H + uc] : 0.f);
            }
        }
    }
    if constexpr (DHS > 0) {
#pragma unroll
        for (int k = 0; k < UPT; ++k) {
            dhc[k] = slab_fold<DR>(t1[k], a.dhr_nslab) + slab_fold<DR>(t2[k], a.dhr2_nslab);
            dho[k] = slab_fold<D>(t3[k], a.dho_nslab);
        }
    }
    // ---- LN: gate activations from the saved xhat (same expressions as the forward)
    if (LN) {
#pragma unroll
        for (int k = 0; k < UPT; ++k) {
            ac[k][0] = cell_sig(xh[k][0] * lg[k][0] + lb[k][0]);
            ac[k][1] = cell_tanh(xh[k][1] * lg[k][1] + lb[k][1]);
            ac[k][2] = cell_sig(xh[k][2] * lg[k][2] + lb[k][2] + a.forget_bias);
            ac[k][3] = cell_sig(xh[k][3] * lg[k][3] + lb[k][3]);
        }
    }
    // ---- output: h' = th * o
    // (the LN-path saves dlncy / dc_rec / dlny are stored after the last
    // exchange: stores queued on a CU delay its in-launch hand-offs)
    float dc[UPT], dout[UPT], dch[UPT], dlc[UPT], dcr[UPT];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
        const int u = base + k * NT + tid;
        const int64_t ro = (int64_t)b * H + u;
        const float dh = dho[k] + (r ? 0.f : dhc[k]);
        dc[k] = r ? 0.f : dcc[k];
        if (on[k] && r && a.dinit_h) {
            a.dinit_h[ro] += dhc[k];
            a.dinit_c[ro] += dcc[k];
        }
        const float o = ac[k][3];
        const float t = LN ? cell_tanh(cx[k] * lcg[k] + lcb[k]) : cell_tanh(cx[k]);
        dout[k] = dh * t;
        const float dcn = dh * o * (1.f - t * t);
        if (LN) {
            dlc[k] = dcn;
            dch[k] = on[k] ? dcn * lcg[k] : 0.f;
            s1 += dch[k];
            s2 += dch[k] * cx[k];
        } else {
            dc[k] += dcn;
        }
    }
    if (LN) {
        float s[2] = {s1, s2};
        row_sum<2, NW>(s, lds, mine, all, a.part, a.err, a.step + 1, b, c, C);
        const float rc = a.rstd[b * 5 + 4];
#pragma unroll
        for (int k = 0; k < UPT; ++k) dc[k] += rc * (dch[k] - s[0] / (float)H - cx[k] * s[1] / (float)H);
    }
    // ---- cell: c' = c*f + i*tj*m
    float dy[UPT][4];
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
        const int u = base + k * NT + tid;
        const int64_t ro = (int64_t)b * H + u;
        const float i = ac[k][0], tj = ac[k][1], f = ac[k][2], o = ac[k][3];
        const float m = dropout_mult(keep_on, key, ro, a.keep);
        dy[k][0] = dc[k] * tj * m * i * (1.f - i);
        dy[k][1] = dc[k] * i * m * (1.f - tj * tj);
        dy[k][2] = dc[k] * cp[k] * f * (1.f - f);
        dy[k][3] = dout[k] * o * (1.f - o);
        dcr[k] = dc[k] * f;
        if (!LN && on[k]) a.dc_rec[ro] = dcr[k];
    }
    // ---- LayerNorm over each gate block
    if (LN) {
        float acc[8], dly[UPT][4];
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] = 0.f;
#pragma unroll
        for (int k = 0; k < UPT; ++k) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                dly[k][q] = dy[k][q];
                const float dg = on[k] ? dy[k][q] * lg[k][q] : 0.f;
                dy[k][q] = dg;
                acc[q] += dg;
                acc[4 + q] += dg * xh[k][q];
            }
        }
        row_sum<8, NW>(acc, lds, mine, all, a.part + (int64_t)a.B * C * kSlots, a.err, a.step + 1, b, c, C);
#pragma unroll
        for (int k = 0; k < UPT; ++k) {
            if (!on[k]) continue;
            const int u = base + k * NT + tid;
            const int64_t ro = (int64_t)b * H + u;
            st_save(a.dlncy, ro, dlc[k], a.save_lp);
            a.dc_rec[ro] = dcr[k];
#pragma unroll
            for (int q = 0; q < 4; ++q) st_save(a.dlny, (int64_t)b * 4 * H + q * H + u, dly[k][q], a.save_lp);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float rs = a.rstd[b * 5 + q];
#pragma unroll
            for (int k = 0; k < UPT; ++k)
                dy[k][q] = rs * (dy[k][q] - acc[q] / (float)H - xh[k][q] * acc[4 + q] / (float)H);
        }
    }
    // ---- outputs
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
        if (!on[k]) continue;
        const int u = base + k * NT + tid;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float dg = dy[k][q];
            float dr = dg;
            if (MOD) {
                if (a.dxp_kind == 1) ((__hip_bfloat16*)a.dxp)[b * a.ld_dxp + q * H + u] = to_bf16(dg * ax[k][q]);
                else ((float*)a.dxp)[b * a.ld_dxp + q * H + u] = dg * ax[k][q];
                dr = dg * ah[k][q];
                const int64_t o0 = (int64_t)b * a.vec_ld + u;
                const float d3[3] = {dg * xv[k][q], dg * rv[k][q], dg};
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const int64_t oi = (4 * j + q) * a.vec_gs + o0;
                    if (a.dvec_kind == 1) ((__hip_bfloat16*)a.dvec)[oi] = to_bf16(d3[j]);
                    else ((float*)a.dvec)[oi] = d3[j];
                }
            }
            if (a.dG != nullptr) a.dG[b * a.ld_dG + q * H + u] = dr;   // (null: only the bf16 copy is read)
            if (a.dG_lp_kind == 1) ((__hip_bfloat16*)a.dG_lp)[b * a.ld_dG_lp + q * H + u] = to_bf16(dr);
        }
    }
}

}  // namespace
