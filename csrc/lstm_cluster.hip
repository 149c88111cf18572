// Clustered LSTM-family cell step: one batch row split over C workgroups.
//
// Why: the per-step cell update is memory-bound (~100-300 KB per row at
// H = 2048) but has only B ~ 100 rows; one workgroup per row leaves 60 % of
// the 256 CUs idle and funnels each row through one CU's load path. Here a
// row is split over C = ceil(H / 256) workgroups (grid C x B, one hidden
// unit x 4 gates per thread). Without LayerNorm the step is purely
// elementwise. With LayerNorm the C workgroups of a row exchange partial
// statistics inside the launch:
//
//   each workgroup: local (mean, M2) per gate block  (two-pass, in registers)
//   publish: 8 floats with write-through (sc1) agent stores, drain vmcnt,
//            one relaxed agent atomic add on the row's arrival counter
//   wait:    one lane polls the counter (relaxed, s_sleep backoff, bounded)
//   read:    every partial loaded with sc1 (agent) loads after the poll
//   combine: Chan's parallel formula -> exact mean / variance of the row
//
// This is the write-through / drained-flag hand-off of the CDNA4 guide
// (Guideline 16 R1; "Valid forms" row 1: one lane per storing workgroup,
// agent atomic add, sc1 loads), so no acquire fence is needed. Counters are
// per (step, row, phase) and zeroed by one memset per sequence; a wait that
// exceeds the spin bound sets *err (checked by the host) instead of hanging.
// All B*C workgroups must be co-resident (B*C <= ~4 per CU at 256 threads):
// the host only selects cluster mode when that holds.
//
// Math is identical to csrc/lstm_row.hip (same saves, same dropout hash).
#include "lstm_args.h"

namespace {

using namespace skr;

constexpr int NT = 256, NW = NT / 64;
constexpr int kMaxCluster = 16;          // H <= 4096
constexpr unsigned kSpinLimit = 1u << 21;
// Every arrival counter and every workgroup's partial slot owns a 128-byte
// line: agent-scope atomics and sc1 traffic on a shared line serialise at the
// memory side (CDNA4 guide, float-atomics contention row).
constexpr int kSyncStride = 32;   // ints
constexpr int kPartStride = 32;   // floats

// Publish `nv` floats of this workgroup (LDS `mine`), wait for the row's C
// workgroups, gather all C*nv values into LDS `all` ([C][nv]).
__device__ void cluster_allgather(float* part, int* cnt, int* err, int b, int c, int C, const float* mine, int nv,
                                  float* all) {
    __syncthreads();
    if (threadIdx.x == 0) {
        float* dst = part + ((int64_t)b * C + c) * kPartStride;
        for (int i = 0; i < nv; ++i) __hip_atomic_store(dst + i, mine[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned spins = 0;
        while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < C) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > kSpinLimit) {
                __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < C * nv; i += NT) {
        const int cc = i / nv, k = i - cc * nv;
        all[i] = __hip_atomic_load(part + ((int64_t)b * C + cc) * kPartStride + k, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
}

// Exact mean / variance of a row from per-workgroup (mean, M2) pairs.
__device__ __forceinline__ void chan_combine(const float* all, int C, int nv, int q, int H, float& mean, float& var) {
    float m = 0.f;
    for (int cc = 0; cc < C; ++cc) m += (float)min(NT, H - cc * NT) * all[cc * nv + q];
    m /= (float)H;
    float m2 = 0.f;
    for (int cc = 0; cc < C; ++cc) {
        const float n = (float)min(NT, H - cc * NT);
        const float d = all[cc * nv + q] - m;
        m2 += all[cc * nv + (nv / 2) + q] + n * d * d;
    }
    mean = m;
    var = m2 / (float)H;
}

template <bool LN, bool MOD>
__global__ __launch_bounds__(NT) void lstm_fwd_cluster(const FwdArgs a) {
    __shared__ float lds[NW * 8];
    __shared__ float mine[8];
    __shared__ float all[kMaxCluster * 8];
    const int c = blockIdx.x, b = blockIdx.y, C = gridDim.x, tid = threadIdx.x, H = a.H;
    const int u = c * NT + tid;
    const bool on = u < H;
    const int nloc = min(NT, H - c * NT);
    const int grp = a.grp_rows > 0 ? b / a.grp_rows : 0;
    const float* ln_g = a.ln_g ? a.ln_g + grp * 4 * H : nullptr;
    const float* ln_b = a.ln_b ? a.ln_b + grp * 4 * H : nullptr;
    const float* lnc_g = a.lnc_g ? a.lnc_g + grp * H : nullptr;
    const float* lnc_b = a.lnc_b ? a.lnc_b + grp * H : nullptr;
    const bool keep_on = a.keep < 1.0f;
    const uint32_t key = keep_on ? hash_key(*a.seed, a.stream, a.step) : 0u;
    const int64_t ro = (int64_t)b * H + u;
    float g[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        float v = 0.f;
        if (on) {
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
        g[q] = v;
    }
    if (LN) {
        float s[4] = {g[0], g[1], g[2], g[3]};
        block_sum<4, NW>(s, lds);
        float ml[4], m2[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            ml[q] = s[q] / (float)nloc;
            const float d = on ? g[q] - ml[q] : 0.f;
            m2[q] = d * d;
        }
        block_sum<4, NW>(m2, lds);
        if (tid == 0) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                mine[q] = ml[q];
                mine[4 + q] = m2[q];
            }
        }
        cluster_allgather(a.part, a.sync + b * kSyncStride, a.err, b, c, C, mine, 8, all);
        float rs[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float mean, var;
            chan_combine(all, C, 8, q, H, mean, var);
            rs[q] = rsqrtf(var + kLnEps);
            const float xh = (g[q] - mean) * rs[q];
            if (on) {
                a.xhat[(int64_t)b * 4 * H + q * H + u] = xh;
                g[q] = xh * ln_g[q * H + u] + ln_b[q * H + u];
            }
        }
        if (c == 0 && tid < 4) a.rstd[b * 5 + tid] = rs[tid];
    }
    const float i = sigmoidf_(g[0]);
    const float tj = tanhf(g[1]);
    const float f = sigmoidf_(g[2] + a.forget_bias);
    const float o = sigmoidf_(g[3]);
    const float m = dropout_mult(keep_on, key, ro, a.keep);
    float cn = 0.f;
    if (on) {
        cn = a.c_prev[ro] * f + i * tj * m;
        float* ap = a.act + (int64_t)b * 4 * H + u;
        ap[0] = i;
        ap[H] = tj;
        ap[2 * H] = f;
        ap[3 * H] = o;
        a.c_out[ro] = cn;
    }
    float th;
    if (LN) {
        float s1[1] = {cn};
        block_sum<1, NW>(s1, lds);
        const float ml = s1[0] / (float)nloc;
        const float d = on ? cn - ml : 0.f;
        float s2[1] = {d * d};
        block_sum<1, NW>(s2, lds);
        if (tid == 0) {
            mine[0] = ml;
            mine[1] = s2[0];
        }
        cluster_allgather(a.part + (int64_t)a.B * C * kPartStride, a.sync + (a.B + b) * kSyncStride, a.err, b, c, C, mine, 2, all);
        float mean, var;
        chan_combine(all, C, 2, 0, H, mean, var);
        const float rc = rsqrtf(var + kLnEps);
        if (c == 0 && tid == 0) a.rstd[b * 5 + 4] = rc;
        const float ch = (cn - mean) * rc;
        th = 0.f;
        if (on) {
            a.chat[ro] = ch;
            th = tanhf(ch * lnc_g[u] + lnc_b[u]);
        }
    } else {
        th = tanhf(cn);
    }
    if (!on) return;
    const bool r = a.reset != nullptr && a.reset[b] != 0.f;
    const float h = th * o;
    a.h_out[ro] = h;
    const float hc = r ? a.init_h[ro] : h;
    a.h_carry[ro] = hc;
    a.c_carry[ro] = r ? a.init_c[ro] : cn;
    if (a.lp_kind == 1) ((__hip_bfloat16*)a.h_lp)[b * a.ld_lp + u] = to_bf16(hc);
    else if (a.lp_kind == 2) ((float*)a.h_lp)[b * a.ld_lp + u] = hc;
}

template <bool LN, bool MOD>
__global__ __launch_bounds__(NT) void lstm_bwd_cluster(const BwdArgs a) {
    __shared__ float lds[NW * 8];
    __shared__ float mine[8];
    __shared__ float all[kMaxCluster * 8];
    const int c = blockIdx.x, b = blockIdx.y, C = gridDim.x, tid = threadIdx.x, H = a.H;
    const int u = c * NT + tid;
    const bool on = u < H;
    const int grp = a.grp_rows > 0 ? b / a.grp_rows : 0;
    const float* ln_g = a.ln_g ? a.ln_g + grp * 4 * H : nullptr;
    const float* lnc_g = a.lnc_g ? a.lnc_g + grp * H : nullptr;
    const float* lnc_b = a.lnc_b ? a.lnc_b + grp * H : nullptr;
    const bool keep_on = a.keep < 1.0f;
    const uint32_t key = keep_on ? hash_key(*a.seed, a.stream, a.step) : 0u;
    const bool r = a.reset != nullptr && a.reset[b] != 0.f;
    const int64_t ro = (int64_t)b * H + u;
    // ---- output: h' = th * o ----
    float dc = 0.f, dout = 0.f, dch = 0.f, ch = 0.f;
    if (on) {
        const float dhc = a.dh_rec ? ld_slabs(a.dh_rec, b * a.ld_dh_rec + u, a.dhr_nslab, a.dhr_slab) : 0.f;
        const float dcc = a.dc_rec[ro];
        const float dh = (a.dh_out ? ld_slabs(a.dh_out, ro, a.dho_nslab, a.dho_slab) : 0.f) + (r ? 0.f : dhc);
        dc = r ? 0.f : dcc;
        if (r && a.dinit_h) {
            a.dinit_h[ro] += dhc;
            a.dinit_c[ro] += dcc;
        }
        const float o = a.act[(int64_t)b * 4 * H + 3 * H + u];
        float t;
        if (LN) {
            ch = a.chat[ro];
            t = tanhf(ch * lnc_g[u] + lnc_b[u]);
        } else {
            t = tanhf(a.c_new[ro]);
        }
        dout = dh * t;
        const float dcn = dh * o * (1.f - t * t);
        if (LN) {
            a.dlncy[ro] = dcn;
            dch = dcn * lnc_g[u];
        } else {
            dc += dcn;
        }
    }
    if (LN) {
        float s[2] = {dch, dch * ch};
        block_sum<2, NW>(s, lds);
        if (tid == 0) {
            mine[0] = s[0];
            mine[1] = s[1];
        }
        cluster_allgather(a.part, a.sync + b * kSyncStride, a.err, b, c, C, mine, 2, all);
        float t0 = 0.f, t1 = 0.f;
        for (int cc = 0; cc < C; ++cc) {
            t0 += all[cc * 2];
            t1 += all[cc * 2 + 1];
        }
        const float rc = a.rstd[b * 5 + 4];
        dc += rc * (dch - t0 / (float)H - ch * t1 / (float)H);
    }
    // ---- cell ----
    float dy[4] = {0.f, 0.f, 0.f, 0.f};
    if (on) {
        const float* ap = a.act + (int64_t)b * 4 * H + u;
        const float i = ap[0], tj = ap[H], f = ap[2 * H], o = ap[3 * H];
        const float m = dropout_mult(keep_on, key, ro, a.keep);
        const float cp = a.c_prev[ro];
        dy[0] = dc * tj * m * i * (1.f - i);
        dy[1] = dc * i * m * (1.f - tj * tj);
        dy[2] = dc * cp * f * (1.f - f);
        dy[3] = dout * o * (1.f - o);
        a.dc_rec[ro] = dc * f;
    }
    if (LN) {
        float acc[8], xh[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            xh[q] = 0.f;
            acc[q] = acc[4 + q] = 0.f;
            if (on) {
                const int64_t gi = (int64_t)b * 4 * H + q * H + u;
                xh[q] = a.xhat[gi];
                a.dlny[gi] = dy[q];
                const float dg = dy[q] * ln_g[q * H + u];
                dy[q] = dg;
                acc[q] = dg;
                acc[4 + q] = dg * xh[q];
            }
        }
        block_sum<8, NW>(acc, lds);
        if (tid == 0) {
#pragma unroll
            for (int k = 0; k < 8; ++k) mine[k] = acc[k];
        }
        cluster_allgather(a.part + (int64_t)a.B * C * kPartStride, a.sync + (a.B + b) * kSyncStride, a.err, b, c, C, mine, 8, all);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float t0 = 0.f, t1 = 0.f;
            for (int cc = 0; cc < C; ++cc) {
                t0 += all[cc * 8 + q];
                t1 += all[cc * 8 + 4 + q];
            }
            dy[q] = a.rstd[b * 5 + q] * (dy[q] - t0 / (float)H - xh[q] * t1 / (float)H);
        }
    }
    if (!on) return;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float dg = dy[q];
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
                if (a.dvec_kind == 1) ((__hip_bfloat16*)a.dvec)[oi] = to_bf16(d3[j]);
                else ((float*)a.dvec)[oi] = d3[j];
            }
        }
        a.dG[b * a.ld_dG + q * H + u] = dr;
        if (a.dG_lp_kind == 1) ((__hip_bfloat16*)a.dG_lp)[b * a.ld_dG_lp + q * H + u] = to_bf16(dr);
    }
}

}  // namespace

namespace skr {

int launch_cluster(const FwdArgs& a, bool ln, bool mod, hipStream_t s) {
    const int C = (a.H + NT - 1) / NT;
    if (C != a.cluster || C > kMaxCluster || (mod && !ln)) return -5;
    const dim3 grid(C, a.B);
    if (mod) hipLaunchKernelGGL((lstm_fwd_cluster<true, true>), grid, dim3(NT), 0, s, a);
    else if (ln) hipLaunchKernelGGL((lstm_fwd_cluster<true, false>), grid, dim3(NT), 0, s, a);
    else hipLaunchKernelGGL((lstm_fwd_cluster<false, false>), grid, dim3(NT), 0, s, a);
    return SKR_CHECK_LAUNCH();
}

int launch_cluster(const BwdArgs& a, bool ln, bool mod, hipStream_t s) {
    const int C = (a.H + NT - 1) / NT;
    if (C != a.cluster || C > kMaxCluster || (mod && !ln)) return -5;
    const dim3 grid(C, a.B);
    if (mod) hipLaunchKernelGGL((lstm_bwd_cluster<true, true>), grid, dim3(NT), 0, s, a);
    else if (ln) hipLaunchKernelGGL((lstm_bwd_cluster<true, false>), grid, dim3(NT), 0, s, a);
    else hipLaunchKernelGGL((lstm_bwd_cluster<false, false>), grid, dim3(NT), 0, s, a);
    return SKR_CHECK_LAUNCH();
}

}  // namespace skr
