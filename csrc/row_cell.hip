// Row-per-workgroup LayerNorm-LSTM cell kernels (forward and backward step):
// one workgroup owns one batch row, each thread V contiguous hidden units.
//
// Why: the clustered cell kernels (csrc/lstm_cell.hip) split a wide row over
// C workgroups and exchange the LayerNorm statistics in-launch through
// tagged global slots -- about 3 us per exchange on MI355X, two per
// backward step -- and load every operand as a scalar (2-4 bytes per lane:
// one vector-memory instruction per unit per operand). At the HyperLSTM
// shapes (H = 2048 main cell, H = 256 hyper cell, B = 100) the step is then
// bound by exchange latency and instruction issue, not bytes. Here every
// statistic is a workgroup reduction (DPP + LDS, no global exchange) and
// every operand is a 16-byte (fp32 x4, bf16 x8) or 8-byte (bf16 x4) vector
// load, all issued before the first use. A row block of 100 workgroups
// leaves CUs idle, but each one streams its row with few instructions.
//
// Semantics: identical expressions to cell_fwd_body / cell_bwd with LN
// (csrc/cell_fwd_body.h, csrc/lstm_cell.hip) -- LayerNorm over each gate
// block and over c (var = E[x^2] - mean^2, clamped, eps kLnEps), forget
// bias, stateless recurrent dropout on tanh(j) keyed by (seed, stream, step,
// b*H + u), the HyperLSTM modulation g = xh*ax + R*ah + bh + bias (MOD 3:
// precomputed by csrc/hyper_mod.hip with per-tile statistics). Reference
// cell: /root/reference model.py:19-27 (LayerNormLSTM / HyperLSTM cells
// inside the static unroll of model.py:66-95); no eoc resets on these paths
// (the VAE decoders), so `reset` must be null.
#include <cstdlib>

#include "row_cell.h"

namespace {

using namespace skr;

// ---- forward -------------------------------------------------------------------------
// MOD 0: g = xp + sum of the R slabs (LN-LSTM / hyper cell; DS = compile-time
// slab ceiling); MOD 3: g = gpre with the gate statistics summed from gstats
// (HyperLSTM main cell).
template <int NT, int V, int MOD, int DS>
__global__ __launch_bounds__(NT) void row_fwd(const FwdArgs a) {
    constexpr int NW = NT / 64;
    __shared__ float lds[NW * 8];
    const int b = blockIdx.x, tid = threadIdx.x, H = a.H, u0 = tid * V;
    const int grp = a.grp_rows > 0 ? b / a.grp_rows : 0;
    const float* ln_g = a.ln_g + grp * 4 * H;
    const float* ln_b = a.ln_b + grp * 4 * H;
    const int64_t ro = (int64_t)b * H + u0;
    const bool save = a.xhat != nullptr;
    const float invH = 1.0f / (float)H;
    const bool keep_on = a.keep < 1.0f;
    const uint32_t key = keep_on ? hash_key(*a.seed, a.stream, a.step) : 0u;

    // ---- every load up front
    float g[4][V], lg[4][V], lb[4][V], cp[V], lcg[V], lcb[V];
    float rt[MOD == 0 ? 4 : 1][DS][V];
    const int nr = min(a.R_nslab, DS);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if constexpr (MOD == 3) {
            ldf<V>(a.gpre + (int64_t)b * 4 * H + q * H + u0, g[q]);
        } else {
            ldf<V>(a.xp + b * a.ld_xp + q * H + u0, g[q]);
            load_slabs<V, DS>(a.R + b * a.ld_R + q * H + u0, nr, a.R_slab, rt[q]);
        }
        ldf<V>(ln_g + q * H + u0, lg[q]);
        ldf<V>(ln_b + q * H + u0, lb[q]);
    }
    ldf<V>(a.c_prev + ro, cp);
    ldf<V>(a.lnc_g + grp * H + u0, lcg);
    ldf<V>(a.lnc_b + grp * H + u0, lcb);
    if constexpr (MOD == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            fold_slabs<V, DS>(rt[q], nr, g[q]);
            if (a.R_nslab > DS) add_slabs<V>(a.R + DS * a.R_slab + b * a.ld_R + q * H + u0, a.R_nslab - DS, a.R_slab, g[q]);
        }
    }

    // ---- LayerNorm statistics of the four gate blocks
    float s[8];
    if constexpr (MOD == 3) {
#pragma unroll
        for (int q = 0; q < 8; ++q) s[q] = 0.f;
        const float* gs = a.gstats + (int64_t)b * 4 * a.gstat_tiles * 2;
        for (int i = tid; i < 4 * a.gstat_tiles; i += NT) {
            const int gq = i / a.gstat_tiles;
            const float v0 = gs[2 * i], v1 = gs[2 * i + 1];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                s[q] += q == gq ? v0 : 0.f;
                s[4 + q] += q == gq ? v1 : 0.f;
            }
        }
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            s[q] = 0.f;
            s[4 + q] = 0.f;
#pragma unroll
            for (int j = 0; j < V; ++j) {
                s[q] += g[q][j];
                s[4 + q] += g[q][j] * g[q][j];
            }
        }
    }
    block_sum<8, NW>(s, lds);
    float rs[4], xs[4][V];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float mean = s[q] * invH;
        const float var = fmaxf(s[4 + q] * invH - mean * mean, 0.f);
        rs[q] = rsqrtf(var + kLnEps);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            xs[q][j] = (g[q][j] - mean) * rs[q];
            g[q][j] = xs[q][j] * lg[q][j] + lb[q][j];
        }
    }
    // ---- cell
    float cn[V], og[V], s2[2] = {0.f, 0.f};
#pragma unroll
    for (int j = 0; j < V; ++j) {
        const float i = cell_sig(g[0][j]);
        const float tj = cell_tanh(g[1][j]);
        const float f = cell_sig(g[2][j] + a.forget_bias);
        og[j] = cell_sig(g[3][j]);
        const float m = dropout_mult(keep_on, key, ro + j, a.keep);
        cn[j] = cp[j] * f + i * tj * m;
        s2[0] += cn[j];
        s2[1] += cn[j] * cn[j];
    }
    block_sum<2, NW>(s2, lds);
    const float mean = s2[0] * invH;
    const float var = fmaxf(s2[1] * invH - mean * mean, 0.f);
    const float rc = rsqrtf(var + kLnEps);
    float ch[V], h[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
        ch[j] = (cn[j] - mean) * rc;
        h[j] = cell_tanh(ch[j] * lcg[j] + lcb[j]) * og[j];
    }
    // ---- stores
    if (save) {
        if (tid < 4) a.rstd[b * 5 + tid] = pick<4>(rs, tid);
        if (tid == 0) a.rstd[b * 5 + 4] = rc;
        st_sv<V>(a.chat, ro, a.save_lp, ch);
#pragma unroll
        for (int q = 0; q < 4; ++q) st_sv<V>(a.xhat, (int64_t)b * 4 * H + q * H + u0, a.save_lp, xs[q]);
    }
    stf<V>(a.h_out + ro, h);
    if (a.h_carry != nullptr) stf<V>(a.h_carry + ro, h);
    if (a.c_out != nullptr) stf<V>(a.c_out + ro, cn);
    stf<V>(a.c_carry + ro, cn);
    if (a.lp_kind == 1) stb<V>((__hip_bfloat16*)a.h_lp + b * a.ld_lp + u0, h);
    else stf<V>((float*)a.h_lp + b * a.ld_lp + u0, h);
}

template <int NT, int V, bool MOD, int DO>
__global__ __launch_bounds__(NT) void row_bwd(const BwdArgs a) {
    row_bwd_body<NT, V, MOD, DO>(a, blockIdx.x);
}

// ---- dispatch --------------------------------------------------------------------------
template <typename A>
using KernelT = void (*)(const A);


// Units per thread: 4 (rows up to 2048 units: <= 512 threads, no AGPR spill
// in the backward), 8 for wider rows.
int pick_v(int H) { return H > 2048 ? 8 : 4; }

#define SKR_ROW_GEOMS(X) X(64, 4) X(128, 4) X(256, 4) X(512, 4) X(256, 8) X(512, 8)

template <int MOD, int DS>
KernelT<FwdArgs> fwd_kernel(int nt, int v) {
#define SKR_ROW_CASE(NT_, V_) if (nt == NT_ && v == V_) return row_fwd<NT_, V_, MOD, DS>;
    SKR_ROW_GEOMS(SKR_ROW_CASE)
#undef SKR_ROW_CASE
    return nullptr;
}
template <bool MOD, int DO>
KernelT<BwdArgs> bwd_kernel(int nt, int v) {
#define SKR_ROW_CASE(NT_, V_) if (nt == NT_ && v == V_) return row_bwd<NT_, V_, MOD, DO>;
    SKR_ROW_GEOMS(SKR_ROW_CASE)
#undef SKR_ROW_CASE
    return nullptr;
}

}  // namespace

// Shape / layout support of the row kernels for a row of H units: 0 if
// supported, else the code the launchers return.
SKR_API int skr_row_supported(int H) {
    if (H < 256 || H % 256 != 0) return -2;
    const int v = pick_v(H), nt = H / v;
    return nt <= 512 ? 0 : -2;   // (1024-thread variants would spill at their 128-VGPR cap)
}

// Forward step. mod 0: g = xp + sum of R slabs; 3: precomputed g + per-tile
// statistics (csrc/hyper_mod.hip). LayerNorm cells only, no resets, bf16 or
// fp32 next-step operand (lp_kind 1 / 2); every pointer 16-byte aligned and
// every stride a multiple of 8 elements.
SKR_API int skr_row_fwd_step(const FwdArgs* args, int mod, hipStream_t s) {
    const FwdArgs& a = *args;
    if (a.B <= 0) return 0;
    if (skr_row_supported(a.H) != 0) return -2;
    if (a.reset != nullptr || (mod != 0 && mod != 3) || (a.lp_kind != 1 && a.lp_kind != 2)) return -3;
    if (mod == 3 && (a.gpre == nullptr || a.gstats == nullptr || a.gstat_tiles < 1)) return -3;
    if (mod == 0 && (a.xp == nullptr || a.R == nullptr || a.R_nslab < 1)) return -3;
    if (!al16(a.xp) || !al16(a.R) || !al16(a.gpre) || !al16(a.c_prev) || !al16(a.h_out) || !al16(a.c_carry) ||
        !al16(a.h_lp) || !al16(a.xhat) || !al16(a.chat) || !al16(a.c_out) || !al16(a.h_carry) || !al16(a.ln_g) ||
        !al16(a.ln_b) || !al16(a.lnc_g) || !al16(a.lnc_b))
        return -4;
    if (!mul8(a.ld_xp) || !mul8(a.ld_R) || !mul8(a.R_slab) || !mul8(a.ld_lp)) return -4;
    const int v = pick_v(a.H), nt = a.H / v;
    KernelT<FwdArgs> k = nullptr;
    if (mod == 3) k = fwd_kernel<3, 1>(nt, v);
    else if (a.R_nslab <= 1) k = fwd_kernel<0, 1>(nt, v);
    else if (a.R_nslab <= 2) k = fwd_kernel<0, 2>(nt, v);
    else if (a.R_nslab <= 4) k = fwd_kernel<0, 4>(nt, v);
    else k = fwd_kernel<0, 8>(nt, v);
    if (k == nullptr) return -2;
    hipLaunchKernelGGL(k, dim3(a.B), dim3(nt), 0, s, a);
    return SKR_CHECK_LAUNCH();
}

// Backward step. mod 0: LN-LSTM / hyper cell; 2: HyperLSTM main cell (bf16
// vec, bf16 R copy r_lp, bf16 dxp / dvec; vec_bias may be null = zero).
SKR_API int skr_row_bwd_step(const BwdArgs* args, int mod, hipStream_t s) {
    const BwdArgs& a = *args;
    if (a.B <= 0) return 0;
    if (skr_row_supported(a.H) != 0) return -2;
    const int rc = row_bwd_check(a, mod);
    if (rc) return rc;
    const int v = pick_v(a.H), nt = a.H / v;
    const bool wide = a.dh_out != nullptr && a.dho_nslab > 1;   // split-K dh_out (the hyper cell's dvec path)
    KernelT<BwdArgs> k = mod == 2 ? (wide ? bwd_kernel<true, 32>(nt, v) : bwd_kernel<true, 1>(nt, v))
                                  : (wide ? bwd_kernel<false, 32>(nt, v) : bwd_kernel<false, 1>(nt, v));
    if (k == nullptr) return -2;
    hipLaunchKernelGGL(k, dim3(a.B), dim3(nt), 0, s, a);
    return SKR_CHECK_LAUNCH();
}
