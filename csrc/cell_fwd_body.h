// Forward cell step of the LSTM-family cell kernels as a device function
// (csrc/lstm_cell.hip: workgroup (c, b) = (blockIdx.x, blockIdx.y)).
// Semantics and geometry: csrc/lstm_cell.hip header comment.
#pragma once
#include "lstm_args.h"

namespace {

using namespace skr;

constexpr int kMaxCluster = 16;
constexpr int kRecSlabs = 8;      // ceiling of the unrolled dh_rec / dh_rec2 slab loads
constexpr unsigned kSpinLimit = 1u << 21;
constexpr int kSlots = 16;        // 8-byte granules per workgroup slot (128 B)

// Diagnostic build only (-DSKR_TRACE_CELL; the round-3 cell bench, removed from the tree, defined it):
// s_memrealtime stamps per workgroup at entry / loads landed / after each
// LayerNorm exchange / stores drained.
#ifdef SKR_TRACE_CELL
__device__ uint64_t* g_cell_trace;
#define SKR_STAMP(i)                                                                              \
    do {                                                                                          \
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                          \
        if (g_cell_trace && threadIdx.x == 0)                                                     \
            g_cell_trace[((int64_t)b * C + c) * 8 + (i)] = __builtin_amdgcn_s_memrealtime();      \
    } while (0)
#else
#define SKR_STAMP(i) do {} while (0)
#endif

// Publish `nv` floats of this workgroup (LDS `mine`) as tagged granules and
// gather the row's C*nv values into LDS `all` ([C][nv]).
__device__ void cluster_allgather(uint64_t* part, int* err, int b, int c, int C, const float* mine, int nv,
                                  uint32_t tag, float* all) {
    lds_barrier();
    const int tid = threadIdx.x;
    uint64_t* row = part + (int64_t)b * C * kSlots;
    if (tid < nv) {
        const uint64_t w = ((uint64_t)tag << 32) | __float_as_uint(mine[tid]);
        __hip_atomic_store(row + c * kSlots + tid, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (tid < 64) {
        for (int i = tid; i < C * nv; i += 64) {
            const int cc = i / nv, k = i - cc * nv;
            uint64_t w = __hip_atomic_load(row + cc * kSlots + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            unsigned spins = 0;
            while ((uint32_t)(w >> 32) != tag) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > kSpinLimit) {
                    __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                w = __hip_atomic_load(row + cc * kSlots + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            all[i] = __uint_as_float((uint32_t)w);
        }
    }
    lds_barrier();
}

// Row-wide sums of N per-thread values: block reduction, then (C > 1) the
// in-launch exchange. `slot` selects the (counter, partial) pair of this phase.
template <int N, int NW>
__device__ __forceinline__ void row_sum(float (&v)[N], float* lds, float* mine, float* all, uint64_t* part,
                                        int* err, uint32_t tag, int b, int c, int C) {
    block_sum<N, NW>(v, lds);
    if (C <= 1) return;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < N; ++i) mine[i] = v[i];
    }
    cluster_allgather(part, err, b, c, C, mine, N, tag, all);
#pragma unroll
    for (int i = 0; i < N; ++i) {
        float s = 0.f;
        for (int cc = 0; cc < C; ++cc) s += all[cc * N + i];
        v[i] = s;
    }
}

// x5 / w5 (decode step, csrc/decode_step.hip): the x-projection is formed
// here from the row's 5 stroke values, xp[b] + sum_k x5[k] w5[k][col] (the
// summation order of skr_bproj_fwd, csrc/inproj.hip); null: xp is complete.
template <int NT, int UPT, int NS, bool LN, int MOD>
__device__ __forceinline__ void cell_fwd_body(const FwdArgs& a, const int c, const int b, const int C,
                                              const float* x5 = nullptr, const float* w5 = nullptr,
                                              int64_t ldw5 = 0) {
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
    // saves for the backward (null pointers at inference): LN layers save
    // xhat / rstd / chat only -- the backward recomputes the gate activations
    // from xhat -- plain layers save act
    const bool save = LN ? a.xhat != nullptr : a.act != nullptr;
    SKR_STAMP(0);

    // ---- every load up front (clamped indices; results of u >= H discarded)
    float g[UPT][4], cp[UPT], lg[UPT][4], lb[UPT][4], lcg[UPT], lcb[UPT];
    float rsv[UPT][4];   // MOD: summed R (saved in bf16 for the backward when r_lp is set)
    bool on[UPT];
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
        const int u = base + k * NT + tid;
        on[k] = u < H;
        const int uc = min(u, H - 1);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if constexpr (MOD == 3) {   // precomputed pre-activations (csrc/hyper_mod.hip)
                g[k][q] = a.gpre[(int64_t)b * 4 * H + q * H + uc];
                rsv[k][q] = 0.f;
                if (LN) {
                    lg[k][q] = ln_g[q * H + uc];
                    lb[k][q] = ln_b[q * H + uc];
                }
                continue;
            }
            float xv = a.xp[b * a.ld_xp + q * H + uc];
            if (x5 != nullptr) {
#pragma unroll
                for (int i = 0; i < 5; ++i) xv += x5[i] * w5[i * ldw5 + q * H + uc];
            }
            const float rv = slab_sum<NS>(a.R, b * a.ld_R + q * H + uc, a.R_nslab, a.R_slab);
            if (MOD) {
                const int64_t vo = (int64_t)b * a.vec_ld + uc;
                const float ax = ldvec<MOD>(a.vec, q * a.vec_gs + vo) + a.vec_bias[q * H + uc];
                const float ah = ldvec<MOD>(a.vec, (4 + q) * a.vec_gs + vo) + a.vec_bias[(4 + q) * H + uc];
                const float bh = ldvec<MOD>(a.vec, (8 + q) * a.vec_gs + vo) + a.vec_bias[(8 + q) * H + uc];
                g[k][q] = xv * ax + rv * ah + bh + a.bias[q * H + uc];
                rsv[k][q] = rv;
            } else {
                g[k][q] = xv + rv;
            }
            if (LN) {
                lg[k][q] = ln_g[q * H + uc];
                lb[k][q] = ln_b[q * H + uc];
            }
        }
        cp[k] = a.c_prev[(int64_t)b * H + uc];
        if (LN) {
            lcg[k] = lnc_g[uc];
            lcb[k] = lnc_b[uc];
        }
    }
    // ---- LayerNorm over each gate block of the row: sums and sums of
    // squares in ONE row reduction (var = E[g^2] - mean^2 in fp32, clamped).
    // The saves (xhat, bf16 R, c') are stored only after the second
    // exchange: stores queued on a CU delay its in-launch hand-offs.
    float xs[UPT][4];   // xhat (LN)
    SKR_STAMP(1);
    if (LN) {
        float s[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            s[q] = 0.f;
            s[4 + q] = 0.f;
#pragma unroll
            for (int k = 0; k < UPT; ++k) {
                const float v = on[k] ? g[k][q] : 0.f;
                s[q] += v;
                s[4 + q] += v * v;
            }
        }
        if constexpr (MOD == 3) {   // the row's statistics: sum of the per-tile partials
#pragma unroll
            for (int q = 0; q < 8; ++q) s[q] = 0.f;
            const float* gs = a.gstats + (int64_t)b * 4 * a.gstat_tiles * 2;
            for (int i = tid; i < 4 * a.gstat_tiles; i += NT) {
                const int gq = i / a.gstat_tiles;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (q == gq) {
                        s[q] += gs[2 * i];
                        s[4 + q] += gs[2 * i + 1];
                    }
                }
            }
            block_sum<8, NW>(s, lds);
        } else {
            row_sum<8, NW>(s, lds, mine, all, a.part, a.err, a.step + 1, b, c, C);
        }
        SKR_STAMP(2);
        float mean[4], var[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            mean[q] = s[q] / (float)H;
            var[q] = fmaxf(s[4 + q] / (float)H - mean[q] * mean[q], 0.f);
        }
        float rs[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) rs[q] = rsqrtf(var[q] + kLnEps);
#pragma unroll
        for (int k = 0; k < UPT; ++k) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                xs[k][q] = (g[k][q] - mean[q]) * rs[q];
                g[k][q] = xs[k][q] * lg[k][q] + lb[k][q];
            }
        }
        if (save && c == 0 && tid < 4) a.rstd[b * 5 + tid] = rs[tid];
    }
    // ---- cell
    float cn[UPT], og[UPT];
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
        const int u = base + k * NT + tid;
        const int64_t ro = (int64_t)b * H + u;
        const float i = cell_sig(g[k][0]);
        const float tj = cell_tanh(g[k][1]);
        const float f = cell_sig(g[k][2] + a.forget_bias);
        const float o = cell_sig(g[k][3]);
        const float m = dropout_mult(keep_on, key, ro, a.keep);
        cn[k] = on[k] ? cp[k] * f + i * tj * m : 0.f;
        og[k] = o;
        if (!LN && save && on[k]) {
            float* ap = a.act + (int64_t)b * 4 * H + u;
            ap[0] = i;
            ap[H] = tj;
            ap[2 * H] = f;
            ap[3 * H] = o;
        }
        if (!LN) {
            if (a.c_out != nullptr && on[k]) a.c_out[ro] = cn[k];
        }
    }
    float th[UPT];
    if (LN) {
        float s2[2] = {0.f, 0.f};
#pragma unroll
        for (int k = 0; k < UPT; ++k) {
            s2[0] += cn[k];          // cn == 0 for units past H
            s2[1] += cn[k] * cn[k];
        }
        row_sum<2, NW>(s2, lds, mine, all, a.part + (int64_t)a.B * C * kSlots, a.err, a.step + 1, b, c, C);
        SKR_STAMP(3);
        const float mean = s2[0] / (float)H;
        const float var = fmaxf(s2[1] / (float)H - mean * mean, 0.f);
        const float rc = rsqrtf(var + kLnEps);
        if (save && c == 0 && tid == 0) a.rstd[b * 5 + 4] = rc;
#pragma unroll
        for (int k = 0; k < UPT; ++k) {
            const int u = base + k * NT + tid;
            const int64_t ro = (int64_t)b * H + u;
            const float ch = (cn[k] - mean) * rc;
            th[k] = cell_tanh(ch * lcg[k] + lcb[k]);
            if (!on[k]) continue;
            if (save) {
                st_save(a.chat, ro, ch, a.save_lp);
#pragma unroll
                for (int q = 0; q < 4; ++q) st_save(a.xhat, (int64_t)b * 4 * H + q * H + u, xs[k][q], a.save_lp);
            }
            if (a.c_out != nullptr) a.c_out[ro] = cn[k];
            if (MOD && a.r_lp != nullptr) {
#pragma unroll
                for (int q = 0; q < 4; ++q) a.r_lp[b * a.ld_R + q * H + u] = to_bf16(rsv[k][q]);
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < UPT; ++k) th[k] = cell_tanh(cn[k]);
    }
    // ---- MX-fp8 copy of the carried h (FwdArgs::h_q8): 32 consecutive units
    // are 32 consecutive lanes, so each block's amax is 5 xor shuffles; every
    // lane takes part (units past H count as 0)
    if (a.h_q8 != nullptr) {
#pragma unroll
        for (int k = 0; k < UPT; ++k) {
            const int u = base + k * NT + tid;
            const int64_t ro = (int64_t)b * H + min(u, H - 1);
            const float hc = !on[k] ? 0.f : (r ? a.init_h[ro] : th[k] * og[k]);
            float m = fabsf(hc);
#pragma unroll
            for (int o = 1; o < 32; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
            const int X = min(max((int)((__float_as_uint(m) >> 23) & 0xff) - 7, 0), 254);
            const float q = hc * __uint_as_float((uint32_t)(254 - X) << 23);
            if (on[k]) {
                a.h_q8[(int64_t)b * a.ld_q8 + u] = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(q, 0.f, 0, false) & 0xff);
                if ((tid & 31) == 0) {
                    const int blk = u >> 5;
                    a.h_qs[(int64_t)b * (H / 32) + (blk & 3) * (H / 128) + (blk >> 2)] = (uint8_t)X;
                }
            }
        }
    }
    // ---- outputs + carry (reference eoc reset)
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
        const int u = base + k * NT + tid;
        if (!on[k]) continue;
        const int64_t ro = (int64_t)b * H + u;
        const float h = th[k] * og[k];
        a.h_out[ro] = h;
        if constexpr (!LN && MOD != 0 && MOD != 3) {   // (the LN path stores it after its exchanges)
            if (a.r_lp != nullptr) {
#pragma unroll
                for (int q = 0; q < 4; ++q) a.r_lp[b * a.ld_R + q * H + u] = to_bf16(rsv[k][q]);
            }
        }
        const float hc = r ? a.init_h[ro] : h;
        if (a.h_carry != nullptr) a.h_carry[ro] = hc;   // (== h_out without resets: callers skip it)
        a.c_carry[ro] = r ? a.init_c[ro] : cn[k];
        if (a.lp_kind == 1) ((__hip_bfloat16*)a.h_lp)[b * a.ld_lp + u] = to_bf16(hc);
        else if (a.lp_kind == 2) ((float*)a.h_lp)[b * a.ld_lp + u] = hc;
    }
    SKR_STAMP(4);
}

}  // namespace
