// Row-per-workgroup LayerNorm-LSTM cell helpers and the backward step body
// (csrc/row_cell.hip: one workgroup per batch row; csrc/chain_step.hip: the
// same body as the waiting rows of a chained launch). Design and semantics:
// csrc/row_cell.hip header comment.
#pragma once
#include "cell_fwd_body.h"
#include "handoff.h"

namespace {

using namespace skr;

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// ---- vector loads / stores of V contiguous values (V = 4 or 8) -------------------------
template <int V>
__device__ __forceinline__ void ldf(const float* p, float (&o)[V]) {
#pragma unroll
    for (int j = 0; j < V; j += 4) {
        const f32x4 t = *(const f32x4*)(p + j);
        o[j] = t[0];
        o[j + 1] = t[1];
        o[j + 2] = t[2];
        o[j + 3] = t[3];
    }
}
__device__ __forceinline__ void unpack2(uint32_t w, float& lo, float& hi) {
    lo = __uint_as_float(w << 16);
    hi = __uint_as_float(w & 0xffff0000u);
}
template <int V>
__device__ __forceinline__ void ldb(const void* p, float (&o)[V]) {
    if constexpr (V == 4) {
        const u32x2 w = *(const u32x2*)p;
        unpack2(w[0], o[0], o[1]);
        unpack2(w[1], o[2], o[3]);
    } else {
#pragma unroll
        for (int j = 0; j < V; j += 8) {
            const u32x4 w = *(const u32x4*)((const char*)p + 2 * j);
#pragma unroll
            for (int i = 0; i < 4; ++i) unpack2(w[i], o[j + 2 * i], o[j + 2 * i + 1]);
        }
    }
}
// LN saves: bf16 (lp) or fp32
template <int V>
__device__ __forceinline__ void ld_sv(const void* p, int64_t i, bool lp, float (&o)[V]) {
    if (lp) ldb<V>((const __hip_bfloat16*)p + i, o);
    else ldf<V>((const float*)p + i, o);
}
template <int V>
__device__ __forceinline__ void stf(float* p, const float (&v)[V]) {
#pragma unroll
    for (int j = 0; j < V; j += 4) *(f32x4*)(p + j) = f32x4{v[j], v[j + 1], v[j + 2], v[j + 3]};
}
__device__ __forceinline__ uint32_t pack2(float a, float b) {
    return (uint32_t)__bfloat16_as_ushort(__float2bfloat16(a)) |
           ((uint32_t)__bfloat16_as_ushort(__float2bfloat16(b)) << 16);
}
template <int V>
__device__ __forceinline__ void stb(void* p, const float (&v)[V]) {
    if constexpr (V == 4) {
        *(u32x2*)p = u32x2{pack2(v[0], v[1]), pack2(v[2], v[3])};
    } else {
#pragma unroll
        for (int j = 0; j < V; j += 8)
            *(u32x4*)((char*)p + 2 * j) = u32x4{pack2(v[j], v[j + 1]), pack2(v[j + 2], v[j + 3]),
                                                pack2(v[j + 4], v[j + 5]), pack2(v[j + 6], v[j + 7])};
    }
}
template <int V>
__device__ __forceinline__ void st_sv(void* p, int64_t i, bool lp, const float (&v)[V]) {
    if (lp) stb<V>((__hip_bfloat16*)p + i, v);
    else stf<V>((float*)p + i, v);
}
// Split-K slab sums. load_slabs issues all D loads of up to D slabs into
// distinct registers (clamped addresses: slabs past n re-read slab n-1, the
// same lines) before fold_slabs adds the first n -- an accumulate-as-you-load
// loop reuses one destination and serialises every load behind the last.
// add_slabs handles counts past a ceiling (batches of 8, each waited on).
template <int V, int D>
__device__ __forceinline__ void load_slabs(const float* p, int n, int64_t slab, float (&t)[D][V]) {
#pragma unroll
    for (int k = 0; k < D; ++k) ldf<V>(p + (int64_t)min(k, n - 1) * slab, t[k]);
}
template <int V, int D>
__device__ __forceinline__ void fold_slabs(const float (&t)[D][V], int n, float (&o)[V]) {
#pragma unroll
    for (int k = 0; k < D; ++k)
#pragma unroll
        for (int j = 0; j < V; ++j) o[j] += k < n ? t[k][j] : 0.f;
}
template <int V>
__device__ __forceinline__ void add_slabs(const float* p, int n, int64_t slab, float (&o)[V]) {
    for (int s0 = 0; s0 < n; s0 += 8) {
        float t[8][V];
        load_slabs<V, 8>(p + s0 * slab, n - s0, slab, t);
        fold_slabs<V, 8>(t, n - s0, o);
    }
}
template <int N>
__device__ __forceinline__ float pick(const float (&v)[N], int i) {
    float r = v[0];
#pragma unroll
    for (int k = 1; k < N; ++k) r = i == k ? v[k] : r;
    return r;
}

// Row sums of a row split over C workgroups: each workgroup's block sums
// (already in every thread) published and the C partials added in part order.
template <int N>
__device__ __forceinline__ void row_exchange(float (&v)[N], float* mine, float* all, uint64_t* part, int* err,
                                             uint32_t tag, int b, int c, int C) {
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

// ---- forward -------------------------------------------------------------------------
// (the step kernels: csrc/row_cell.hip row_fwd)
// MOD 0: g = xp + sum of the R slabs (LN-LSTM / hyper cell; DS = compile-time
// slab ceiling); MOD 3: g = gpre with the gate statistics summed from gstats
// (HyperLSTM main cell).
// CHAIN (csrc/chain_step.hip, MOD 0): the R slabs are produced by tiles of
// the SAME launch -- every other load is issued first, then the row waits on
// the launch's arrival counter and reads the slabs with sc1 loads.
// HSC1 (csrc/hyper_mod.hip hyper_cell_mod): the bf16 next-step operand h_lp
// is read by workgroups of the SAME launch after the row's arrival, so it is
// stored write-through (8-byte relaxed agent-scope stores, lp_kind 1 only).
template <int NT, int V, int MOD, int DS, bool CHAIN = false, bool HSC1 = false>
__device__ __forceinline__ void row_fwd_body(const FwdArgs& a, const int b, const uint32_t* chain_cnt = nullptr,
                                             uint32_t chain_target = 0, int* chain_err = nullptr, const int tid0 = 0) {
    static_assert(!CHAIN || (V == 4 && MOD == 0), "chained forward row: MOD 0, 16-byte slab loads");
    static_assert(!HSC1 || V == 4, "write-through h_lp: 8-byte stores");
    constexpr int NW = NT / 64;
    __shared__ float lds[NW * 8];
    const int tid = threadIdx.x - tid0, H = a.H, u0 = tid * V;   // tid0: first thread of the row (one-wave rows)
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
            if constexpr (!CHAIN) load_slabs<V, DS>(a.R + b * a.ld_R + q * H + u0, nr, a.R_slab, rt[q]);
        }
        ldf<V>(ln_g + q * H + u0, lg[q]);
        ldf<V>(ln_b + q * H + u0, lb[q]);
    }
    ldf<V>(a.c_prev + ro, cp);
    ldf<V>(a.lnc_g + grp * H + u0, lcg);
    ldf<V>(a.lnc_b + grp * H + u0, lcb);
    if constexpr (CHAIN) {
        chain_wait<1>(chain_cnt, chain_target, chain_err);
        const __amdgpu_buffer_rsrc_t r = rsrc(a.R, 0x7fffffff);
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int k = 0; k < DS; ++k) {
                const f32x4 v = ld_sc1_f32x4(r, (uint32_t)(((int64_t)min(k, nr - 1) * a.R_slab + b * a.ld_R + q * H + u0) * 4));
#pragma unroll
                for (int jj = 0; jj < V; ++jj) rt[q][k][jj] = v[jj];
            }
    }
    if constexpr (MOD == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            fold_slabs<V, DS>(rt[q], nr, g[q]);
            if (!CHAIN && a.R_nslab > DS)
                add_slabs<V>(a.R + DS * a.R_slab + b * a.ld_R + q * H + u0, a.R_nslab - DS, a.R_slab, g[q]);
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
    if constexpr (HSC1) {
        const uint64_t w = (uint64_t)pack2(h[0], h[1]) | ((uint64_t)pack2(h[2], h[3]) << 32);
        __hip_atomic_store((uint64_t*)((__hip_bfloat16*)a.h_lp + b * a.ld_lp + u0), w, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    } else if (a.lp_kind == 1) {
        stb<V>((__hip_bfloat16*)a.h_lp + b * a.ld_lp + u0, h);
    } else {
        stf<V>((float*)a.h_lp + b * a.ld_lp + u0, h);
    }
}

// ---- backward ------------------------------------------------------------------------
// MOD: HyperLSTM main cell (bf16 modulation vectors, bf16 R copy; writes
// dxh = dg*ax, dvec = [dg*xh | dg*R | dg] and dR = dg*ah); otherwise dG = dg.
// DO: compile-time ceiling of the dh_out slab count (1 or 32); dh_rec /
// dh_rec2 slabs are loaded 8 at a time.
// CHAIN (csrc/chain_step.hip): the dh_rec slabs are produced by tiles of
// the SAME launch -- every other load is issued first, then the row waits on
// the launch's arrival counter and reads them with sc1 loads (16-byte
// buffer loads); the arithmetic is unchanged.
// DVSC1 (csrc/chain_step.hip, three-stage launch): dvec is read by GEMM tiles
// of the SAME launch after the rows' arrival counter, so its stores are
// write-through (sc1, 8-byte relaxed agent-scope atomic stores).
template <int V>
__device__ __forceinline__ void stb_sc1(void* p, const float (&v)[V]) {
    static_assert(V == 4, "8-byte sc1 stores");
    const uint64_t w = (uint64_t)pack2(v[0], v[1]) | ((uint64_t)pack2(v[2], v[3]) << 32);
    __hip_atomic_store((uint64_t*)p, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// CL > 1: the row is split over CL workgroups (part c of CL owns units
// [c H / CL, (c + 1) H / CL), NT V == H / CL), and its two LayerNorm-backward
// row sums are exchanged between them in-launch as tagged granules
// (cluster_allgather, csrc/cell_fwd_body.h; a.part / a.err, tag = step + 1).
template <int NT, int V, bool MOD, int DO, bool CHAIN = false, bool DVSC1 = false, int POLL = 1, int CL = 1>
__device__ __forceinline__ void row_bwd_body(const BwdArgs& a, const int b, const uint32_t* chain_cnt = nullptr,
                                             uint32_t chain_target = 0, int* chain_err = nullptr, const int c = 0) {
    static_assert(!CHAIN || V == 4, "chained row: 16-byte slab loads");
    constexpr int NW = NT / 64;
    __shared__ float lds[NW * 8];
    __shared__ float mine[8];
    __shared__ float all[kMaxCluster * 8];
    const int tid = threadIdx.x, H = a.H, u0 = c * (H / CL) + tid * V;
    const int grp = a.grp_rows > 0 ? b / a.grp_rows : 0;
    const float* ln_g = a.ln_g + grp * 4 * H;
    const float* ln_b = a.ln_b + grp * 4 * H;
    const int64_t ro = (int64_t)b * H + u0;
    const float invH = 1.0f / (float)H;
    const bool keep_on = a.keep < 1.0f;
    const uint32_t key = keep_on ? hash_key(*a.seed, a.stream, a.step) : 0u;

    // ---- every load up front
    float dh[V], dcc[V], cp[V], cx[V], lcg[V], lcb[V];
    float xh[4][V], lg[4][V], lb[4][V], xv[4][V], rv[4][V], ax[4][V], ah[4][V];
    float t0[DO][V], t1[8][V], t2[8][V];
    const int n0 = a.dh_out ? min(a.dho_nslab, DO) : 0;
    const int n1 = a.dh_rec ? min(a.dhr_nslab, 8) : 0;
    const int n2 = a.dh_rec2 ? min(a.dhr2_nslab, 8) : 0;
    if (n0) load_slabs<V, DO>(a.dh_out + ro, n0, a.dho_slab, t0);
    if (!CHAIN && n1) load_slabs<V, 8>(a.dh_rec + b * a.ld_dh_rec + u0, n1, a.dhr_slab, t1);
    if (n2) load_slabs<V, 8>(a.dh_rec2 + b * a.ld_dh_rec2 + u0, n2, a.dhr2_slab, t2);
    ldf<V>(a.dc_rec + ro, dcc);
    ldf<V>(a.c_prev + ro, cp);
    ld_sv<V>(a.chat, ro, a.save_lp, cx);
    ldf<V>(a.lnc_g + grp * H + u0, lcg);
    ldf<V>(a.lnc_b + grp * H + u0, lcb);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        ld_sv<V>(a.xhat, (int64_t)b * 4 * H + q * H + u0, a.save_lp, xh[q]);
        ldf<V>(ln_g + q * H + u0, lg[q]);
        ldf<V>(ln_b + q * H + u0, lb[q]);
        if constexpr (MOD) {
            const int64_t vo = (int64_t)b * a.vec_ld + u0;
            if (a.xp_lp) ldb<V>((const __hip_bfloat16*)a.xp + b * a.ld_xp + q * H + u0, xv[q]);
            else ldf<V>(a.xp + b * a.ld_xp + q * H + u0, xv[q]);
            ldb<V>(a.r_lp + b * a.ld_R + q * H + u0, rv[q]);
            ldb<V>((const __hip_bfloat16*)a.vec + q * a.vec_gs + vo, ax[q]);
            ldb<V>((const __hip_bfloat16*)a.vec + (4 + q) * a.vec_gs + vo, ah[q]);
        }
    }
    if constexpr (CHAIN) {
        chain_wait<POLL>(chain_cnt, chain_target, chain_err);
        if (n1) {
            const __amdgpu_buffer_rsrc_t r = rsrc(a.dh_rec, 0x7fffffff);
            const int64_t base = (int64_t)b * a.ld_dh_rec + u0;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const f32x4 v = ld_sc1_f32x4(r, (uint32_t)(((int64_t)min(k, n1 - 1) * a.dhr_slab + base) * 4));
#pragma unroll
                for (int j = 0; j < V; ++j) t1[k][j] = v[j];
            }
        }
    }
#pragma unroll
    for (int j = 0; j < V; ++j) dh[j] = 0.f;
    if (n0) fold_slabs<V, DO>(t0, n0, dh);
    if (n1) fold_slabs<V, 8>(t1, n1, dh);
    if (n2) fold_slabs<V, 8>(t2, n2, dh);
    if (a.dh_out && a.dho_nslab > DO) add_slabs<V>(a.dh_out + DO * a.dho_slab + ro, a.dho_nslab - DO, a.dho_slab, dh);
    if (a.dh_rec && a.dhr_nslab > 8)
        add_slabs<V>(a.dh_rec + 8 * a.dhr_slab + b * a.ld_dh_rec + u0, a.dhr_nslab - 8, a.dhr_slab, dh);
    if (a.dh_rec2 && a.dhr2_nslab > 8)
        add_slabs<V>(a.dh_rec2 + 8 * a.dhr2_slab + b * a.ld_dh_rec2 + u0, a.dhr2_nslab - 8, a.dhr2_slab, dh);
    if constexpr (MOD) {
        if (a.vec_bias != nullptr) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float e0[V], e1[V];
                ldf<V>(a.vec_bias + q * H + u0, e0);
                ldf<V>(a.vec_bias + (4 + q) * H + u0, e1);
#pragma unroll
                for (int j = 0; j < V; ++j) {
                    ax[q][j] += e0[j];
                    ah[q][j] += e1[j];
                }
            }
        }
    }
    // ---- gate activations from xhat (as the forward)
    float ac[4][V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
        ac[0][j] = cell_sig(xh[0][j] * lg[0][j] + lb[0][j]);
        ac[1][j] = cell_tanh(xh[1][j] * lg[1][j] + lb[1][j]);
        ac[2][j] = cell_sig(xh[2][j] * lg[2][j] + lb[2][j] + a.forget_bias);
        ac[3][j] = cell_sig(xh[3][j] * lg[3][j] + lb[3][j]);
    }
    // ---- h' = o * tanh(LN(c')): back through the c LayerNorm
    float dout[V], dch[V], dlc[V], s2[2] = {0.f, 0.f};
#pragma unroll
    for (int j = 0; j < V; ++j) {
        const float t = cell_tanh(cx[j] * lcg[j] + lcb[j]);
        dout[j] = dh[j] * t;
        const float dcn = dh[j] * ac[3][j] * (1.f - t * t);
        dlc[j] = dcn;
        dch[j] = dcn * lcg[j];
        s2[0] += dch[j];
        s2[1] += dch[j] * cx[j];
    }
    block_sum<2, NW>(s2, lds);
    if constexpr (CL > 1) row_exchange<2>(s2, mine, all, a.part, a.err, a.step + 1, b, c, CL);
    const float rc = a.rstd[b * 5 + 4];
    const float m1 = s2[0] * invH, m2 = s2[1] * invH;
    // ---- c' = c*f + i*tj*m
    float dy[4][V], dcr[V], acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = 0.f;
#pragma unroll
    for (int j = 0; j < V; ++j) {
        const float dc = dcc[j] + rc * (dch[j] - m1 - cx[j] * m2);
        const float i = ac[0][j], tj = ac[1][j], f = ac[2][j], o = ac[3][j];
        const float m = dropout_mult(keep_on, key, ro + j, a.keep);
        dy[0][j] = dc * tj * m * i * (1.f - i);
        dy[1][j] = dc * i * m * (1.f - tj * tj);
        dy[2][j] = dc * cp[j] * f * (1.f - f);
        dy[3][j] = dout[j] * o * (1.f - o);
        dcr[j] = dc * f;
    }
    // ---- back through the gate LayerNorms
    float dg[4][V];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int j = 0; j < V; ++j) {
            dg[q][j] = dy[q][j] * lg[q][j];
            acc[q] += dg[q][j];
            acc[4 + q] += dg[q][j] * xh[q][j];
        }
    block_sum<8, NW>(acc, lds);
    if constexpr (CL > 1) row_exchange<8>(acc, mine, all, a.part + (int64_t)a.B * CL * kSlots, a.err, a.step + 1, b, c, CL);
    st_sv<V>(a.dlncy, ro, a.save_lp, dlc);
    stf<V>(a.dc_rec + ro, dcr);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        st_sv<V>(a.dlny, (int64_t)b * 4 * H + q * H + u0, a.save_lp, dy[q]);
        const float rs = a.rstd[b * 5 + q];
        const float a1 = acc[q] * invH, a2 = acc[4 + q] * invH;
#pragma unroll
        for (int j = 0; j < V; ++j) dg[q][j] = rs * (dg[q][j] - a1 - xh[q][j] * a2);
    }
    // ---- outputs
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        float dr[V];
        if constexpr (MOD) {
            float t[V];
            const int64_t o0 = (int64_t)b * a.vec_ld + u0;
#pragma unroll
            for (int j = 0; j < V; ++j) t[j] = dg[q][j] * ax[q][j];
            stb<V>((__hip_bfloat16*)a.dxp + b * a.ld_dxp + q * H + u0, t);
#pragma unroll
            for (int j = 0; j < V; ++j) t[j] = dg[q][j] * xv[q][j];
            if constexpr (DVSC1) stb_sc1<V>((__hip_bfloat16*)a.dvec + q * a.vec_gs + o0, t);
            else stb<V>((__hip_bfloat16*)a.dvec + q * a.vec_gs + o0, t);
#pragma unroll
            for (int j = 0; j < V; ++j) t[j] = dg[q][j] * rv[q][j];
            if constexpr (DVSC1) {
                stb_sc1<V>((__hip_bfloat16*)a.dvec + (4 + q) * a.vec_gs + o0, t);
                stb_sc1<V>((__hip_bfloat16*)a.dvec + (8 + q) * a.vec_gs + o0, dg[q]);
            } else {
                stb<V>((__hip_bfloat16*)a.dvec + (4 + q) * a.vec_gs + o0, t);
                stb<V>((__hip_bfloat16*)a.dvec + (8 + q) * a.vec_gs + o0, dg[q]);
            }
#pragma unroll
            for (int j = 0; j < V; ++j) dr[j] = dg[q][j] * ah[q][j];
        } else {
#pragma unroll
            for (int j = 0; j < V; ++j) dr[j] = dg[q][j];
        }
        if (a.dG != nullptr) stf<V>(a.dG + b * a.ld_dG + q * H + u0, dr);
        if (a.dG_lp_kind == 1) stb<V>((__hip_bfloat16*)a.dG_lp + b * a.ld_dG_lp + q * H + u0, dr);
    }
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
inline bool mul8(int64_t v) { return (v & 7) == 0; }

// Operand / layout checks of a backward row step (mod 0: LN-LSTM / hyper
// cell; 2: HyperLSTM main cell): 0 if the row kernels take it.
inline int row_bwd_check(const BwdArgs& a, int mod) {
    if (a.reset != nullptr || (mod != 0 && mod != 2) || a.xhat == nullptr || a.dlny == nullptr) return -3;
    if (mod == 2 && (a.r_lp == nullptr || a.xp == nullptr || a.vec == nullptr || a.dxp_kind != 1 ||
                     a.dvec_kind != 1 || a.dxp == nullptr || a.dvec == nullptr))
        return -3;
    if ((a.dh_out && a.dho_nslab < 1) || (a.dh_rec && a.dhr_nslab < 1) || (a.dh_rec2 && a.dhr2_nslab < 1)) return -3;
    if (!al16(a.dh_out) || !al16(a.dh_rec) || !al16(a.dh_rec2) || !al16(a.dc_rec) || !al16(a.c_prev) ||
        !al16(a.xhat) || !al16(a.chat) || !al16(a.xp) || !al16(a.r_lp) || !al16(a.vec) || !al16(a.vec_bias) ||
        !al16(a.dG) || !al16(a.dG_lp) || !al16(a.dxp) || !al16(a.dvec) || !al16(a.dlny) || !al16(a.dlncy) ||
        !al16(a.ln_g) || !al16(a.ln_b) || !al16(a.lnc_g) || !al16(a.lnc_b))
        return -4;
    if (!mul8(a.dho_slab) || !mul8(a.ld_dh_rec) || !mul8(a.dhr_slab) || !mul8(a.ld_dh_rec2) || !mul8(a.dhr2_slab) ||
        !mul8(a.ld_xp) || !mul8(a.ld_R) || !mul8(a.vec_gs) || !mul8(a.vec_ld) || !mul8(a.ld_dG) ||
        !mul8(a.ld_dG_lp) || !mul8(a.ld_dxp))
        return -4;
    return 0;
}

// Operand / layout checks of a forward row step (mod 0: xp + R slabs; 3:
// precomputed g + tile statistics): 0 if the row kernels take it.
inline int row_fwd_check(const FwdArgs& a, int mod) {
    if (a.reset != nullptr || (mod != 0 && mod != 3) || (a.lp_kind != 1 && a.lp_kind != 2)) return -3;
    if (mod == 3 && (a.gpre == nullptr || a.gstats == nullptr || a.gstat_tiles < 1)) return -3;
    if (mod == 0 && (a.xp == nullptr || a.R == nullptr || a.R_nslab < 1)) return -3;
    if (!al16(a.xp) || !al16(a.R) || !al16(a.gpre) || !al16(a.c_prev) || !al16(a.h_out) || !al16(a.c_carry) ||
        !al16(a.h_lp) || !al16(a.xhat) || !al16(a.chat) || !al16(a.c_out) || !al16(a.h_carry) || !al16(a.ln_g) ||
        !al16(a.ln_b) || !al16(a.lnc_g) || !al16(a.lnc_b))
        return -4;
    if (!mul8(a.ld_xp) || !mul8(a.ld_R) || !mul8(a.R_slab) || !mul8(a.ld_lp)) return -4;
    return 0;
}

}  // namespace
