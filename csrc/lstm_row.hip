// Fused LSTM-family cell step (forward + backward) for gfx950.
//
// One workgroup owns one batch row; NT threads (NT = 64..1024, a power of
// two chosen from H) each own UPT = ceil(H / NT) hidden units and all four
// gates (i, j, f, o) of each. Wide workgroups (16 waves at H = 2048) keep
// enough loads in flight per row: the step is latency-bound at B ~ 100 rows.
// Everything between the recurrent GEMM and the next step's GEMM is fused
// into one launch per step:
//
//   g      = xp + R                              (plain / LN-LSTM)
//          = xh*ax + R*ah + bh + bias            (HyperLSTM main cell, MOD;
//                                                 a/b = vec + vec_bias per gate)
//   y      = LN_all(g)*gamma + beta              (LN: per gate block over H)
//   c'     = c*sig(y_f + fb) + sig(y_i)*tanh(y_j)*mask
//   h'     = tanh(LN(c')*gc + bc)*sig(y_o)  |  tanh(c')*sig(y_o)
//   carry  = reset[b] ? init : (h', c')          (reference eoc reset)
//
// plus the saves the backward needs and a bf16 copy of the carried h written
// straight into the next GEMM's A operand (which may be a column slice of a
// concatenated [h | h_hyper] buffer, hence the explicit row stride).
// Rows can be split into parameter groups (grp_rows): the two directions of
// the bidirectional encoder run as 2B rows of one launch with their own
// LayerNorm parameters.
// The recurrent dropout mask is regenerated from a stateless hash of
// (seed, stream, step, b*H + u) in both passes -- never stored.
//
// Reference semantics: model.py:19-23 (BasicLSTMCell), model.py:82-92 (eoc
// reset); LayerNorm-/Hyper-LSTM semantics: sketch_rnn_amd/models/cells.py.
#include "lstm_args.h"

namespace {

using namespace skr;

template <int NT, int UPT, bool LN, bool MOD>
__global__ __launch_bounds__(NT) void lstm_fwd_kernel(const FwdArgs a) {
    constexpr int NW = NT / 64;
    __shared__ float lds[NW * 8];
    const int b = blockIdx.x, tid = threadIdx.x, H = a.H;
    const int grp = a.grp_rows > 0 ? b / a.grp_rows : 0;
    const float* ln_g = a.ln_g ? a.ln_g + grp * 4 * H : nullptr;
    const float* ln_b = a.ln_b ? a.ln_b + grp * 4 * H : nullptr;
    const float* lnc_g = a.lnc_g ? a.lnc_g + grp * H : nullptr;
    const float* lnc_b = a.lnc_b ? a.lnc_b + grp * H : nullptr;
    const bool keep_on = a.keep < 1.0f;
    const uint32_t key = keep_on ? skr::hash_key(*a.seed, a.stream, a.step) : 0u;
    float g[UPT][4];
    bool act_u[UPT];
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
        const int u = tid + k * NT;
        act_u[k] = u < H;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float v = 0.f;
            if (act_u[k]) {
                const float xv = a.xp[b * a.ld_xp + q * H + u];
                const float rv = ld_slabs(a.R, b * a.ld_R + q * H + u, a.R_nslab, a.R_slab);
                if (MOD) {
                    v = xv * vec_at(a.vec, a.vec_bias, a.vec_gs, a.vec_ld, q, b, u, H) +
                        rv * vec_at(a.vec, a.vec_bias, a.vec_gs, a.vec_ld, 4 + q, b, u, H) +
                        vec_at(a.vec, a.vec_bias, a.vec_gs, a.vec_ld, 8 + q, b, u, H) + a.bias[q * H + u];
                } else {
                    v = xv + rv;
                }
            }
            g[k][q] = v;
        }
    }
    if (LN) {
        float mean[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float s = 0.f;
#pragma unroll
            for (int k = 0; k < UPT; ++k) s += g[k][q];
            mean[q] = s;
        }
        skr::block_sum<4, NW>(mean, lds);
        float var[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            mean[q] /= (float)H;
            float s = 0.f;
#pragma unroll
            for (int k = 0; k < UPT; ++k) {
                const float d = act_u[k] ? g[k][q] - mean[q] : 0.f;
                s += d * d;
            }
            var[q] = s;
        }
        skr::block_sum<4, NW>(var, lds);
        float rs[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) rs[q] = rsqrtf(var[q] / (float)H + kLnEps);
#pragma unroll
        for (int k = 0; k < UPT; ++k) {
            const int u = tid + k * NT;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float xh = (g[k][q] - mean[q]) * rs[q];
                if (act_u[k]) {
                    a.xhat[(int64_t)b * 4 * H + q * H + u] = xh;
                    g[k][q] = xh * ln_g[q * H + u] + ln_b[q * H + u];
                }
            }
        }
        if (tid < 4) a.rstd[b * 5 + tid] = rs[tid];
    }
    float c[UPT], o_[UPT];
    float csum = 0.f;
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
        const int u = tid + k * NT;
        const int64_t ro = (int64_t)b * H + u;
        const float i = skr::sigmoidf_(g[k][0]);
        const float tj = tanhf(g[k][1]);
        const float f = skr::sigmoidf_(g[k][2] + a.forget_bias);
        const float o = skr::sigmoidf_(g[k][3]);
        float m = 1.f;
        if (keep_on) m = skr::hash_uniform(key, (uint32_t)ro) < a.keep ? 1.0f / a.keep : 0.f;
        float cn = 0.f;
        if (act_u[k]) {
            cn = a.c_prev[ro] * f + i * tj * m;
            float* ap = a.act + (int64_t)b * 4 * H + u;
            ap[0] = i;
            ap[H] = tj;
            ap[2 * H] = f;
            ap[3 * H] = o;
            a.c_out[ro] = cn;
        }
        c[k] = cn;
        o_[k] = o;
        csum += cn;
    }
    float th[UPT];
    if (LN) {
        float s1[1] = {csum};
        skr::block_sum<1, NW>(s1, lds);
        const float mc = s1[0] / (float)H;
        float s2[1] = {0.f};
#pragma unroll
        for (int k = 0; k < UPT; ++k) {
            const float d = act_u[k] ? c[k] - mc : 0.f;
            s2[0] += d * d;
        }
        skr::block_sum<1, NW>(s2, lds);
        const float rc = rsqrtf(s2[0] / (float)H + kLnEps);
        if (tid == 0) a.rstd[b * 5 + 4] = rc;
#pragma unroll
        for (int k = 0; k < UPT; ++k) {
            const int u = tid + k * NT;
            const float ch = (c[k] - mc) * rc;
            float t = 0.f;
            if (act_u[k]) {
                a.chat[(int64_t)b * H + u] = ch;
                t = tanhf(ch * lnc_g[u] + lnc_b[u]);
            }
            th[k] = t;
        }
    } else {
#pragma unroll
        for (int k = 0; k < UPT; ++k) th[k] = tanhf(c[k]);
    }
    const bool r = a.reset != nullptr && a.reset[b] != 0.f;
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
        if (!act_u[k]) continue;
        const int u = tid + k * NT;
        const int64_t ro = (int64_t)b * H + u;
        const float h = th[k] * o_[k];
        a.h_out[ro] = h;
        const float hc = r ? a.init_h[ro] : h;
        const float cc = r ? a.init_c[ro] : c[k];
        a.h_carry[ro] = hc;
        a.c_carry[ro] = cc;
        if (a.lp_kind == 1) ((__hip_bfloat16*)a.h_lp)[b * a.ld_lp + u] = skr::to_bf16(hc);
        else if (a.lp_kind == 2) ((float*)a.h_lp)[b * a.ld_lp + u] = hc;
    }
}

template <int NT, int UPT, bool LN, bool MOD>
__global__ __launch_bounds__(NT) void lstm_bwd_kernel(const BwdArgs a) {
    constexpr int NW = NT / 64;
    __shared__ float lds[NW * 8];
    const int b = blockIdx.x, tid = threadIdx.x, H = a.H;
    const int grp = a.grp_rows > 0 ? b / a.grp_rows : 0;
    const float* ln_g = a.ln_g ? a.ln_g + grp * 4 * H : nullptr;
    const float* lnc_g = a.lnc_g ? a.lnc_g + grp * H : nullptr;
    const float* lnc_b = a.lnc_b ? a.lnc_b + grp * H : nullptr;
    const bool keep_on = a.keep < 1.0f;
    const uint32_t key = keep_on ? skr::hash_key(*a.seed, a.stream, a.step) : 0u;
    const bool r = a.reset != nullptr && a.reset[b] != 0.f;
    bool act_u[UPT];
    float dc[UPT], dout[UPT], dch[UPT], ch_[UPT];
    float s1 = 0.f, s2 = 0.f;
    // ---- output: h' = th * o ------------------------------------------------
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
        const int u = tid + k * NT;
        act_u[k] = u < H;
        const int64_t ro = (int64_t)b * H + u;
        float dcv = 0.f, dov = 0.f, dchv = 0.f, chv = 0.f;
        if (act_u[k]) {
            const float dhc = a.dh_rec ? ld_slabs(a.dh_rec, b * a.ld_dh_rec + u, a.dhr_nslab, a.dhr_slab) : 0.f;
            const float dcc = a.dc_rec[ro];
            const float dh = (a.dh_out ? ld_slabs(a.dh_out, ro, a.dho_nslab, a.dho_slab) : 0.f) + (r ? 0.f : dhc);
            dcv = r ? 0.f : dcc;
            if (r && a.dinit_h) {
                a.dinit_h[ro] += dhc;
                a.dinit_c[ro] += dcc;
            }
            const float o = a.act[(int64_t)b * 4 * H + 3 * H + u];
            float t;
            if (LN) {
                chv = a.chat[ro];
                t = tanhf(chv * lnc_g[u] + lnc_b[u]);
            } else {
                t = tanhf(a.c_new[ro]);
            }
            dov = dh * t;
            const float dcn = dh * o * (1.f - t * t);
            if (LN) {
                a.dlncy[ro] = dcn;
                dchv = dcn * lnc_g[u];
                s1 += dchv;
                s2 += dchv * chv;
            } else {
                dcv += dcn;
            }
        }
        dc[k] = dcv;
        dout[k] = dov;
        dch[k] = dchv;
        ch_[k] = chv;
    }
    if (LN) {
        float s[2] = {s1, s2};
        skr::block_sum<2, NW>(s, lds);
        const float m1 = s[0] / (float)H, m2 = s[1] / (float)H;
        const float rc = a.rstd[b * 5 + 4];
#pragma unroll
        for (int k = 0; k < UPT; ++k) dc[k] += rc * (dch[k] - m1 - ch_[k] * m2);
    }
    // ---- cell: c' = c*f + i*tj*m ---------------------------------------------
    float dy[UPT][4];
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
        const int u = tid + k * NT;
        const int64_t ro = (int64_t)b * H + u;
        dy[k][0] = dy[k][1] = dy[k][2] = dy[k][3] = 0.f;
        if (!act_u[k]) continue;
        const float* ap = a.act + (int64_t)b * 4 * H + u;
        const float i = ap[0], tj = ap[H], f = ap[2 * H], o = ap[3 * H];
        float m = 1.f;
        if (keep_on) m = skr::hash_uniform(key, (uint32_t)ro) < a.keep ? 1.0f / a.keep : 0.f;
        const float cp = a.c_prev[ro];
        const float d = dc[k];
        dy[k][0] = d * tj * m * i * (1.f - i);
        dy[k][1] = d * i * m * (1.f - tj * tj);
        dy[k][2] = d * cp * f * (1.f - f);
        dy[k][3] = dout[k] * o * (1.f - o);
        a.dc_rec[ro] = d * f;
    }
    // ---- layer norm over each gate block -----------------------------------------
    if (LN) {
        float acc[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] = 0.f;
        float xh[UPT][4];
#pragma unroll
        for (int k = 0; k < UPT; ++k) {
            const int u = tid + k * NT;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float x = 0.f;
                if (act_u[k]) {
                    const int64_t gi = (int64_t)b * 4 * H + q * H + u;
                    x = a.xhat[gi];
                    a.dlny[gi] = dy[k][q];
                    const float dg = dy[k][q] * ln_g[q * H + u];
                    dy[k][q] = dg;
                    acc[q] += dg;
                    acc[4 + q] += dg * x;
                }
                xh[k][q] = x;
            }
        }
        skr::block_sum<8, NW>(acc, lds);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float rs = a.rstd[b * 5 + q];
            const float m1 = acc[q] / (float)H, m2 = acc[4 + q] / (float)H;
#pragma unroll
            for (int k = 0; k < UPT; ++k) dy[k][q] = rs * (dy[k][q] - m1 - xh[k][q] * m2);
        }
    }
    // ---- outputs ------------------------------------------------------------------
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
        if (!act_u[k]) continue;
        const int u = tid + k * NT;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float dg = dy[k][q];
            float dr = dg;
            if (MOD) {
                const float xv = a.xp[b * a.ld_xp + q * H + u];
                const float rv = ld_slabs(a.R, b * a.ld_R + q * H + u, a.R_nslab, a.R_slab);
                a.dxp[b * a.ld_dxp + q * H + u] = dg * vec_at(a.vec, a.vec_bias, a.vec_gs, a.vec_ld, q, b, u, H);
                dr = dg * vec_at(a.vec, a.vec_bias, a.vec_gs, a.vec_ld, 4 + q, b, u, H);
                const int64_t o0 = (int64_t)b * a.vec_ld + u;
                const float d3[3] = {dg * xv, dg * rv, dg};
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const int64_t oi = (4 * j + q) * a.vec_gs + o0;
                    if (a.dvec_kind == 1) ((__hip_bfloat16*)a.dvec)[oi] = skr::to_bf16(d3[j]);
                    else ((float*)a.dvec)[oi] = d3[j];
                }
            }
            a.dG[b * a.ld_dG + q * H + u] = dr;
            if (a.dG_lp_kind == 1) ((__hip_bfloat16*)a.dG_lp)[b * a.ld_dG_lp + q * H + u] = skr::to_bf16(dr);
        }
    }
}

template <int NT, int UPT>
int launch(const FwdArgs& a, bool ln, bool mod, hipStream_t s) {
    if (mod) hipLaunchKernelGGL((lstm_fwd_kernel<NT, UPT, true, true>), dim3(a.B), dim3(NT), 0, s, a);
    else if (ln) hipLaunchKernelGGL((lstm_fwd_kernel<NT, UPT, true, false>), dim3(a.B), dim3(NT), 0, s, a);
    else hipLaunchKernelGGL((lstm_fwd_kernel<NT, UPT, false, false>), dim3(a.B), dim3(NT), 0, s, a);
    return SKR_CHECK_LAUNCH();
}
template <int NT, int UPT>
int launch(const BwdArgs& a, bool ln, bool mod, hipStream_t s) {
    if (mod) hipLaunchKernelGGL((lstm_bwd_kernel<NT, UPT, true, true>), dim3(a.B), dim3(NT), 0, s, a);
    else if (ln) hipLaunchKernelGGL((lstm_bwd_kernel<NT, UPT, true, false>), dim3(a.B), dim3(NT), 0, s, a);
    else hipLaunchKernelGGL((lstm_bwd_kernel<NT, UPT, false, false>), dim3(a.B), dim3(NT), 0, s, a);
    return SKR_CHECK_LAUNCH();
}

// Workgroup shape from H: NT = next power of two >= H (64..1024), one unit
// per thread; beyond 1024 units, 1024 threads with 2 or 4 units each.
template <typename A>
int dispatch(const A& a, bool ln, bool mod, hipStream_t s) {
    if (mod && !ln) return -3;
    if (a.B <= 0) return 0;
    const int H = a.H;
    if (H <= 64) return launch<64, 1>(a, ln, mod, s);
    if (H <= 128) return launch<128, 1>(a, ln, mod, s);
    if (H <= 256) return launch<256, 1>(a, ln, mod, s);
    if (H <= 512) return launch<512, 1>(a, ln, mod, s);
    if (H <= 1024) return launch<1024, 1>(a, ln, mod, s);
    if (H <= 2048) return launch<1024, 2>(a, ln, mod, s);
    if (H <= 4096) return launch<1024, 4>(a, ln, mod, s);
    return -2;
}

}  // namespace

// Host entry points: argument structs are passed by pointer from Python (ctypes
// mirrors of FwdArgs / BwdArgs in sketch_rnn_amd/ops/_hipapi.py).
SKR_API int skr_lstm_fwd_step(const FwdArgs* args, int ln, int mod, hipStream_t s) {
    if (args->cluster > 1) return skr::launch_cluster(*args, ln != 0, mod != 0, s);
    return dispatch(*args, ln != 0, mod != 0, s);
}

SKR_API int skr_lstm_bwd_step(const BwdArgs* args, int ln, int mod, hipStream_t s) {
    if (args->cluster > 1) return skr::launch_cluster(*args, ln != 0, mod != 0, s);
    return dispatch(*args, ln != 0, mod != 0, s);
}

SKR_API int skr_lstm_fwd_args_size() { return (int)sizeof(FwdArgs); }
SKR_API int skr_lstm_bwd_args_size() { return (int)sizeof(BwdArgs); }
