// HyperLSTM forward time step, everything but the main LayerNorm cell in ONE
// launch (the main cell follows as csrc/lstm_cell.hip MOD 3):
//
//   R_hyp = [h | hh]_{t-1} @ W_y        split-K tiles, fp32 partial slabs
//   hh_t  = hyper LN-LSTM cell(x W_x^hyp + R_hyp)        one workgroup per row
//   R     = h_{t-1} @ W_h                 split-K (2) tiles; the halves are
//                                          exchanged between the two splits
//   zd    = hh_t @ W_z                     (per tile, MFMA, W_z slice in LDS)
//   vec   = bf16(zd) @ W_a + q            (q = b_z @ W_a; + main bias on the
//                                          shift blocks) -> bf16
//   g     = xh * vec_x + R * vec_h + vec_b,  per-(row, gate, 64-unit tile)
//                                          sums of g and g^2 for the main LN
//
// Reference recurrence: /root/reference model.py:66-95 (static unroll of the
// decoder cell); HyperLSTM semantics: sketch_rnn_amd/models/cells.py
// hyper_lstm_step (the oracle computes vec exactly this unfolded way).
//
// Why one launch: per step the hyper chain (R_hyp -> hyper cell -> vec) and
// the 32 MB weight stream of h @ W_h are independent until the gate
// epilogue. As separate launches (round 3: grouped GEMM 12.5 us -> hyper cell
// 4.8 -> modulation GEMM 10.2, profiles/r3/vae_large_kernel_summary.txt) the
// chain ran AFTER the stream; here it runs beside it, R never leaves the
// registers of the tile that computed it (only the split partner's half
// crosses, 12.8 KB per tile), and the modulation reads W_z (L2-resident,
// 48 KB per gate) + W_a (1.5 MB) instead of the 12.6 MB folded P = W_z W_a.
//
// Roles by blockIdx.x (256 threads; 72 KB dynamic LDS = the GEMM ring, so at
// most 2 workgroups per CU and the whole grid -- 64 + B + 256 workgroups at
// vae_large -- is co-resident; every wait is on a LOWER block index or on the
// split partner, and every spin is bounded: a timeout sets *err and the grid
// drains):
//   [0, nY)            R_hyp tiles (tile n, split s): slab rows stored sc1,
//                      then one agent atomic add on sync[0]
//   [nY, nY + B)       hyper cell rows: wait sync[0] >= (t+1) nY, sc1 slab
//                      loads, hh_t -> A_next[:, H:] as 16-byte sc1 stores, one
//                      add on sync[1]
//   [nY + B, ...)      main tiles: r = 16 g + 8 s + m -> tile 8 g + m, split s
//                      (the two splits of a tile are blocks b and b + 8: one
//                      XCD under round-robin placement -- speed only)
// Hand-offs follow the CDNA4 guide's first measured row (sc1 payload stores,
// vmcnt(0) of every storing wave, barrier, one lane signals; consumers poll
// with sc1 loads and read the payload with sc1 buffer loads only).
#include "glds_mma.h"
#include "handoff.h"
#include "lstm_args.h"

namespace {

using namespace skr;
typedef bf16x8_t bf16x8;
typedef f32x4_t f32x4;
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));

constexpr int kBN = 64, kNS = 3;                 // main / hyper GEMM tiles: 64 columns, 3-stage ring
constexpr int kEP = 32;                          // embedding padded to one MFMA K step
constexpr int kZS = 3 * kEP + 8;                 // sZ row stride (bf16): conflict-free 16-byte reads
constexpr int kLds = glds_lds_bytes<kBN, kNS>(); // 73,728 B (the backward launch)
// forward launch: the main tiles' epilogue (W_z slice 48 KB + four [32][kZS] z tiles) outgrows the ring
constexpr int kLdsF = 96 * 256 * 2 + 4 * 32 * kZS * 2 > kLds ? 96 * 256 * 2 + 4 * 32 * kZS * 2 : kLds;

// Diagnostic build only (scripts/build_native.py --variant trace_hstep,
// scripts/hstep_trace.py): s_memrealtime stamps (100 MHz) per workgroup at
// the phase boundaries, [block][8] of the last launch.
#ifdef SKR_TRACE_HSTEP
__device__ uint64_t* g_hstep_trace;
#define HS_STAMP(i)                                                                               \
    do {                                                                                          \
        if (g_hstep_trace && threadIdx.x == 0)                                                    \
            g_hstep_trace[(int64_t)blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime();      \
    } while (0)
#else
#define HS_STAMP(i) do {} while (0)
#endif

struct HypFwdArgs {
    int B, H, Hh, S_y;
    uint32_t step;
    const __hip_bfloat16* A;      // [B][K] this step's operand [h_{t-1} | hh_{t-1}], K = H + Hh
    const __hip_bfloat16* WhT;    // [4H][H]
    const __hip_bfloat16* WyT;    // [4Hh][K]
    const float* XH;              // [B][4H] main x-projection (no bias)
    const float* XHY;             // [B][4Hh] hyper x-projection
    const float* hc_prev;         // [B][Hh]
    const float* hln_g; const float* hln_b; const float* hlnc_g; const float* hlnc_b;
    const __hip_bfloat16* WzT;    // [12 * kEP][Hh] (embedding rows past E are zero)
    const __hip_bfloat16* WaT;    // [12][H][kEP] (embedding columns past E are zero)
    const float* qb;              // [12H] b_z @ W_a (+ the main bias on blocks 8..11)
    float forget_bias, hkeep;
    const int64_t* seed; uint32_t hstream;
    float* RY;                    // [S_y][4Hh/64] fragment-native slab tiles (8192 floats each) in-launch
    __hip_bfloat16* A_next;       // [B][K]: hh_t written into columns H..
    float* HH;                    // [B][Hh]
    float* hc_out;                // [B][Hh]
    void* hxhat; float* hrstd; void* hchat;   // hyper LN saves (null at inference)
    float* GP;                    // [B][4H]
    float* GS;                    // [B][4][H/32][2]
    __hip_bfloat16* VEC;          // [B][12H] (blocks 0..7 written) or null
    __hip_bfloat16* RLP;          // [B][4H] or null
    uint32_t* sync;               // [2], zeroed per sequence
    int* err;
    int save_lp;
};

__device__ __forceinline__ u32x4v as_u4(f32x4 v) { return __builtin_bit_cast(u32x4v, v); }

// One wave of every workgroup polls (the others wait at the barrier);
// returns false (uniformly) when the wait timed out or another did.
__device__ __forceinline__ bool wg_wait(const uint32_t* c, uint32_t target, int* err) {
    __shared__ int s_ok;
    if (threadIdx.x < 64) {
        const bool ok = wait_flags(c, 1, target, err);
        if (threadIdx.x == 0) s_ok = ok ? 1 : 0;
    }
    __syncthreads();
    return s_ok != 0;
}

// Every wave drains its (sc1) stores, then one lane adds 1 to the counter.
__device__ __forceinline__ void wg_arrive(uint32_t* c) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Split-K slabs handed over inside a launch are stored fragment-native: each
// lane's f32x4 accumulator (4 consecutive rows of one column) as ONE 16-byte
// write-through store -- 4-byte sc1 stores (one fabric write each) took
// 4-6 us per tile under the weight stream (scripts/hstep_trace.py). Layout per
// slab tile: [4 waves][2 row tiles][4 col tiles][64 lanes][4 rows] floats
// (8192 floats for 128 rows x 64 columns); frag_idx maps (row, column).
__device__ __forceinline__ int64_t frag_idx(int64_t tile, int row, int c) {
    const int w = row >> 5, i = (row >> 4) & 1, fq = (row >> 2) & 3, e = row & 3, j = c >> 4, fr = c & 15;
    return (((((tile * 4 + w) * 2 + i) * 4 + j) * 64 + fq * 16 + fr) << 2) + e;
}

__device__ __forceinline__ void st_frag_tile(__amdgpu_buffer_rsrc_t r, int64_t tile, const f32x4 (&acc)[2][4]) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            st_sc1(r, (uint32_t)((((((tile * 4 + w) * 2 + i) * 4 + j) * 64 + lane) * 16)), as_u4(acc[i][j]));
}

// ---- role 1: R_hyp split-K tile ---------------------------------------------------------
__device__ void rhyp_tile(const HypFwdArgs& a, int id, __hip_bfloat16* smem) {
    const int K = a.H + a.Hh, Gh = 4 * a.Hh, ntY = Gh / kBN;
    const int nt = id % ntY, s = id / ntY, ksl = K / a.S_y;
    f32x4 acc[2][kBN / 16];
    HS_STAMP(0);
    glds_mma<kBN, kNS>(a.A, K, a.WyT, K, a.B, nt * kBN, (int64_t)s * ksl, ksl, smem, acc);
    HS_STAMP(1);
    st_frag_tile(rsrc(a.RY, (int64_t)a.S_y * ntY * 8192 * 4), (int64_t)s * ntY + nt, acc);
    wg_arrive(&a.sync[0]);
    HS_STAMP(2);
}

// ---- role 2: hyper LayerNorm-LSTM cell, one row ------------------------------------------
// The hand-off (hh_t, 16-byte sc1 stores) is published first; the saves for
// the backward and the fp32 outputs (read by later launches) are stored after
// the arrival, off the chain.
__device__ void hyper_row(const HypFwdArgs& a, int b, int nY) {
    HS_STAMP(0);
    if (!wg_wait(&a.sync[0], (a.step + 1) * (uint32_t)nY, a.err)) return;
    HS_STAMP(1);
    __shared__ float lds[4 * 8];
    __shared__ __attribute__((aligned(16))) __hip_bfloat16 hrow[256];
    const int tid = threadIdx.x, Hh = a.Hh, Gh = 4 * Hh, K = a.H + Hh, ntY = Gh / kBN;
    const bool on = tid < Hh;
    const int u = on ? tid : Hh - 1;
    const auto ry = rsrc(a.RY, (int64_t)a.S_y * ntY * 8192 * 4);
    float g[4], lg[4], lb[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        float rs[8];
        const int col = q * Hh + u;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const int ss = min(s, a.S_y - 1);
            rs[s] = ld_sc1_f32(ry, (uint32_t)(frag_idx((int64_t)ss * ntY + (col >> 6), b, col & 63) * 4));
        }
        g[q] = a.XHY[(int64_t)b * Gh + col] + slab_fold<8>(rs, a.S_y);
        lg[q] = a.hln_g[col];
        lb[q] = a.hln_b[col];
    }
    const float cp = a.hc_prev[(int64_t)b * Hh + u];
    const float lcg = a.hlnc_g[u], lcb = a.hlnc_b[u];
    float s[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float v = on ? g[q] : 0.f;
        s[q] = v;
        s[4 + q] = v * v;
    }
    block_sum<8, 4>(s, lds);
    float rs[4], xs[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float mean = s[q] / (float)Hh;
        const float var = fmaxf(s[4 + q] / (float)Hh - mean * mean, 0.f);
        rs[q] = rsqrtf(var + kLnEps);
        xs[q] = (g[q] - mean) * rs[q];
        g[q] = xs[q] * lg[q] + lb[q];
    }
    const int64_t ro = (int64_t)b * Hh + u;
    const bool keep_on = a.hkeep < 1.0f;
    const uint32_t key = keep_on ? hash_key(*a.seed, a.hstream, a.step) : 0u;
    const float ig = cell_sig(g[0]), tj = cell_tanh(g[1]), fg = cell_sig(g[2] + a.forget_bias), og = cell_sig(g[3]);
    const float m = dropout_mult(keep_on, key, ro, a.hkeep);
    const float cn = on ? cp * fg + ig * tj * m : 0.f;
    float s2[2] = {cn, cn * cn};
    block_sum<2, 4>(s2, lds);
    const float mean = s2[0] / (float)Hh;
    const float var = fmaxf(s2[1] / (float)Hh - mean * mean, 0.f);
    const float rc = rsqrtf(var + kLnEps);
    const float ch = (cn - mean) * rc;
    const float h = cell_tanh(ch * lcg + lcb) * og;
    if (on) hrow[tid] = to_bf16(h);
    lds_barrier();
    // hh_t into the next operand, 16-byte write-through stores (read in this launch)
    if (tid < Hh / 8) {
        const auto an = rsrc(a.A_next, (int64_t)a.B * K * 2);
        st_sc1(an, (uint32_t)(((int64_t)b * K + a.H + 8 * tid) * 2), *(const u32x4v*)&hrow[8 * tid]);
    }
    wg_arrive(&a.sync[1]);
    HS_STAMP(2);
    const bool save = a.hxhat != nullptr;
    if (save && tid < 4) a.hrstd[b * 5 + tid] = rs[tid];
    if (save && tid == 0) a.hrstd[b * 5 + 4] = rc;
    if (on) {
        a.HH[ro] = h;
        a.hc_out[ro] = cn;
        if (save) {
            st_save(a.hchat, ro, ch, a.save_lp);
#pragma unroll
            for (int q = 0; q < 4; ++q) st_save(a.hxhat, (int64_t)b * Gh + q * Hh + tid, xs[q], a.save_lp);
        }
    }
}

// ---- role 3: main tile (R = h W_h over the full K, modulation, gate pre-activations) ----
// 32 columns (units u0 .. u0 + 31 of gate q) x all rows, no split-K: nothing
// to exchange between workgroups (a split-K pair's partial exchange cost
// 8.5 us under the stream, scripts/hstep_trace.py).
constexpr int kBNm = 32, kGSm = kBNm + 4;

template <int HHC>   // 16-byte chunks per W_z row (Hh / 8)
__device__ void main_tile(const HypFwdArgs& a, int nt, __hip_bfloat16* smem) {
    constexpr int NJ = kBNm / 16;
    const int H = a.H, Hh = a.Hh, G = 4 * H, K = H + Hh, NV = 12 * H;
    const int n0 = nt * kBNm, q = n0 / H, u0 = n0 - q * H;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, fq = lane >> 4;
    const bool rows_on = 32 * w < a.B;

    f32x4 acc[2][NJ];
    HS_STAMP(0);
    glds_mma<kBNm, kNS>(a.A, K, a.WhT, H, a.B, n0, 0, H, smem, acc);
    HS_STAMP(1);

    // ---- prefetch what does not depend on this launch: x-projection, W_a
    // fragments, q; the W_z slice of gate q into LDS (the ring is free)
    float xv[2][NJ][4];
    bf16x8 waf[3][NJ];
    float qv[3][NJ];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = min(32 * w + 16 * i + 4 * fq + e, a.B - 1);
                xv[i][j][e] = a.XH[(int64_t)row * G + n0 + 16 * j + fr];
            }
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int64_t col = (int64_t)(q + 4 * k) * H + u0 + 16 * j + fr;
            waf[k][j] = *(const bf16x8*)(a.WaT + col * kEP + 8 * fq);
            qv[k][j] = a.qb[col];
        }
    __syncthreads();                                // every wave is past the ring
    constexpr int SWM = (HHC < 16 ? HHC : 16) - 1;
    __hip_bfloat16* sWz = smem;                     // [96][Hh], 16-byte chunks XOR-swizzled by row
    __hip_bfloat16* sZ = smem + 96 * HHC * 8 + w * (32 * kZS);   // this wave's [32][kZS]
    for (int c = tid; c < 96 * HHC; c += 256) {
        const int row = c / HHC, ch = c - row * HHC, kb = q + 4 * (row >> 5), e = row & 31;
        const bf16x8 v = *(const bf16x8*)(a.WzT + ((int64_t)kb * kEP + e) * Hh + 8 * ch);
        *(bf16x8*)(sWz + row * Hh + ((ch ^ (row & SWM)) << 3)) = v;
    }
    HS_STAMP(2);
    // ---- wait for every hyper row (hh_t); the barrier also publishes the W_z slice
    if (!wg_wait(&a.sync[1], (a.step + 1) * (uint32_t)a.B, a.err) || !rows_on) return;
    HS_STAMP(3);

    // zd = hh_t @ W_z (cols: 3 blocks x 32 embeddings), rows 32w .. 32w + 31
    const auto an = rsrc(a.A_next, (int64_t)a.B * K * 2);
    constexpr int KS = HHC / 4;                      // MFMA K steps over Hh
    f32x4 za[2][6];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int c = 0; c < 6; ++c) za[i][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 hf[2][KS];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int row = 32 * w + 16 * i + fr;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
            hf[i][ks] = row < a.B ? ld_sc1(an, (uint32_t)(((int64_t)row * K + H + 32 * ks + 8 * fq) * 2)) : bf16x8{};
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
        for (int c = 0; c < 6; ++c) {
            const int row = (c >> 1) * 32 + 16 * (c & 1) + fr, ch = 4 * ks + fq;
            const bf16x8 bf = *(const bf16x8*)(sWz + row * Hh + ((ch ^ (row & SWM)) << 3));
#pragma unroll
            for (int i = 0; i < 2; ++i) za[i][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hf[i][ks], bf, za[i][c], 0, 0, 0);
        }
    }
    // bf16(zd) -> LDS [row][3 x 32], read back as the A operand of vec = zd @ W_a
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int c = 0; c < 6; ++c)
#pragma unroll
            for (int e = 0; e < 4; ++e)
                sZ[(16 * i + 4 * fq + e) * kZS + (c >> 1) * 32 + 16 * (c & 1) + fr] = to_bf16(za[i][c][e]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bf16x8 zf[2][3];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int k = 0; k < 3; ++k) zf[i][k] = *(const bf16x8*)(sZ + (16 * i + fr) * kZS + 32 * k + 8 * fq);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    float* sG = (float*)sZ;                          // the wave's z region, free again: [16][kGSm] stage
    HS_STAMP(4);

    const bool save = a.VEC != nullptr;
    const int tile = u0 / kBNm, ntile = H / kBNm;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        float gv[NJ][4], vx[NJ][4], vh[NJ][4];
        float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            f32x4 v[3];
#pragma unroll
            for (int k = 0; k < 3; ++k)
                v[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(zf[i][k], waf[k][j], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                // the bf16-rounded vectors are what the backward reads: g uses them too
                const float x = __bfloat162float(to_bf16(v[0][e] + qv[0][j]));
                const float hm = __bfloat162float(to_bf16(v[1][e] + qv[1][j]));
                const float bm = __bfloat162float(to_bf16(v[2][e] + qv[2][j]));
                const float gg = xv[i][j][e] * x + acc[i][j][e] * hm + bm;
                gv[j][e] = gg;
                vx[j][e] = x;
                vh[j][e] = hm;
                s1[e] += gg;
                s2[e] += gg * gg;
            }
        }
        // per-row sums over the tile's 32 units: 16-lane DPP row reductions
#pragma unroll
        for (int e = 0; e < 4; ++e) {
#define SKR_ROWSUM(x) x += dpp_f32<0xB1>(x); x += dpp_f32<0x4E>(x); x += dpp_f32<0x141>(x); x += dpp_f32<0x140>(x);
            SKR_ROWSUM(s1[e])
            SKR_ROWSUM(s2[e])
#undef SKR_ROWSUM
        }
        const int rbase = 32 * w + 16 * i;
        if (fr == 0) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = rbase + 4 * fq + e;
                if (row < a.B) {
                    float* sp = a.GS + (((int64_t)row * 4 + q) * ntile + tile) * 2;
                    *(u32x2v*)sp = u32x2v{__float_as_uint(s1[e]), __float_as_uint(s2[e])};
                }
            }
        }
        // row-contiguous 16-byte stores through the wave's LDS stage: g (fp32),
        // then R and the x / h modulation vectors (bf16) for the backward
        auto stage_store = [&](auto&& val, int kind) {
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) sG[(4 * fq + e) * kGSm + 16 * j + fr] = val(j, e);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                const int rr = (lane >> 3) + 8 * p, c4 = lane & 7, row = rbase + rr;
                const f32x4 v4 = *(const f32x4*)(sG + rr * kGSm + 4 * c4);
                if (row < a.B) {
                    if (kind == 0) {
                        *(f32x4*)(a.GP + (int64_t)row * G + n0 + 4 * c4) = v4;
                    } else {
                        const u32x2v pk{(uint32_t)__bfloat16_as_ushort(to_bf16(v4[0])) |
                                            ((uint32_t)__bfloat16_as_ushort(to_bf16(v4[1])) << 16),
                                        (uint32_t)__bfloat16_as_ushort(to_bf16(v4[2])) |
                                            ((uint32_t)__bfloat16_as_ushort(to_bf16(v4[3])) << 16)};
                        __hip_bfloat16* dst = kind == 1 ? a.RLP + (int64_t)row * G + n0
                                            : a.VEC + (int64_t)row * NV + (kind == 2 ? q : 4 + q) * H + u0;
                        *(u32x2v*)(dst + 4 * c4) = pk;
                    }
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        };
        stage_store([&](int j, int e) { return gv[j][e]; }, 0);
        if (a.RLP != nullptr) stage_store([&](int j, int e) { return acc[i][j][e]; }, 1);
        if (save) {
            stage_store([&](int j, int e) { return vx[j][e]; }, 2);
            stage_store([&](int j, int e) { return vh[j][e]; }, 3);
        }
    }
    HS_STAMP(5);
}

template <int HHC>
__global__ __launch_bounds__(256, 2) void hyper_fwd_step(const HypFwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) __hip_bfloat16 smem[];
    const int nY = (4 * a.Hh / kBN) * a.S_y;
    const int id = blockIdx.x;
    if (id < nY) {
        rhyp_tile(a, id, smem);
    } else if (id < nY + a.B) {
        hyper_row(a, id - nY, nY);
    } else {
        main_tile<HHC>(a, id - nY - a.B, smem);
    }
}

// ===========================================================================
// Backward time step (after the main cell's backward, csrc/row_cell.hip), ONE
// launch for the rest of the step:
//
//   dhh_v  = dvec @ P^T                  split-K tiles -> DHZ slabs (in-launch)
//   hyper cell backward, one row each     dh = sum DHZ + the hh part of DAY
//                                          (previous launch) -> dR_hyp (bf16,
//                                          16-byte sc1 stores, in-launch)
//   d[h|hh] = dR_hyp @ W_y^T              split-K tiles -> DAY slabs: the W_y
//                                          slice is in LDS before the wait
//   dh      = dR_main @ W_h^T             split-K tiles -> DAM slabs, beside
//                                          the whole chain (no dependency)
//
// Round 3 ran these as three launches ([dvec P^T] -> [hyper cell + dR_main
// W_h^T] -> [dR_hyp W_y^T], 6.5 + 14.2 + 6.5 us per step): the 32 MB dR_main
// stream sat in front of the last product of the chain. Here the chain runs
// beside it.
//
// Roles by blockIdx.x: [dvec tiles | dR_main tiles | hyper rows | dR_hyp
// tiles]. Only the hyper rows (wait for every dvec tile) and the dR_hyp tiles
// (wait for every hyper row) wait, and each waits only on roles earlier in
// the grid. Those waiting workgroups (B + (K/64) S_ay) are fewer than the
// device holds at once, so whatever the dispatch order a free slot always
// remains for a producer: the launcher checks that bound.
struct HypBwdArgs {
    int B, H, Hh, S_h, S_am, S_ay;
    uint32_t epoch, step;         // epoch = T - t (counters), step = t (dropout hash)
    const __hip_bfloat16* dVEC;   // [B][12H]
    const __hip_bfloat16* Pl;     // [Hh][12H]
    const __hip_bfloat16* dRM;    // [B][4H]
    const __hip_bfloat16* Whl;    // [H][4H]
    const __hip_bfloat16* Wyl;    // [K][4Hh]
    float* DHZ;                   // [S_h][Hh/64] fragment-native slab tiles (8192 floats each) in-launch
    float* DAM;                   // [S_am][B][H]
    float* DAY;                   // [S_ay][B][K]: read (hh part, previous launch) then written
    int dhr_on;                   // 0: no carried-h source this step (first step, no final-state grads)
    float* dhc_rec;               // [B][Hh] in: grad into carried hc_t; out: into hc_{t-1}
    const float* hc_prev;         // [B][Hh]
    const void* hchat; const void* hxhat; const float* hrstd;
    const float* hln_g; const float* hln_b; const float* hlnc_g; const float* hlnc_b;
    float forget_bias, hkeep;
    const int64_t* seed; uint32_t hstream;
    __hip_bfloat16* dRY;          // [B][4Hh] in-launch
    void* hdlny; void* hdlncy;    // LN saves for the parameter gradients
    uint32_t* sync;               // [2], zeroed per sequence
    int* err;
    int save_lp;
};

__device__ void dvec_tile(const HypBwdArgs& a, int id, __hip_bfloat16* smem) {
    const int NV = 12 * a.H, ntV = a.Hh / kBN;
    const int nt = id % ntV, s = id / ntV, ksl = NV / a.S_h;
    f32x4 acc[2][kBN / 16];
    HS_STAMP(0);
    glds_mma<kBN, kNS>(a.dVEC, NV, a.Pl, NV, a.B, nt * kBN, (int64_t)s * ksl, ksl, smem, acc);
    HS_STAMP(1);
    st_frag_tile(rsrc(a.DHZ, (int64_t)a.S_h * ntV * 8192 * 4), (int64_t)s * ntV + nt, acc);
    wg_arrive(&a.sync[0]);
    HS_STAMP(2);
}

__device__ void drm_tile(const HypBwdArgs& a, int id, __hip_bfloat16* smem) {
    const int G = 4 * a.H, ntM = a.H / kBN;
    const int nt = id % ntM, s = id / ntM, ksl = G / a.S_am;
    f32x4 acc[2][kBN / 16];
    HS_STAMP(0);
    glds_mma<kBN, kNS>(a.dRM, G, a.Whl, G, a.B, nt * kBN, (int64_t)s * ksl, ksl, smem, acc);
    HS_STAMP(1);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fq = lane >> 4;
    float* C = a.DAM + (int64_t)s * a.B * a.H;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < kBN / 16; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = 32 * w + 16 * i + 4 * fq + e;
                if (row < a.B) C[(int64_t)row * a.H + nt * kBN + 16 * j + fr] = acc[i][j][e];
            }
    HS_STAMP(2);
}

// hyper LayerNorm-LSTM cell backward, one row (csrc/cell_bwd_body.h semantics:
// LN, no modulation, no resets, one workgroup per row); DHS: compile-time
// ceiling of the dvec-path slab count
template <int DHS>
__device__ void hyper_row_bwd(const HypBwdArgs& a, int b, int nV) {
    HS_STAMP(0);
    if (!wg_wait(&a.sync[0], a.epoch * (uint32_t)nV, a.err)) return;
    HS_STAMP(1);
    __shared__ float lds[4 * 8];
    __shared__ __attribute__((aligned(16))) __hip_bfloat16 drow[4 * 256];
    const int tid = threadIdx.x, Hh = a.Hh, Gh = 4 * Hh, K = a.H + Hh, ntV = Hh / kBN;
    const bool on = tid < Hh;
    const int u = on ? tid : Hh - 1;
    const int64_t ro = (int64_t)b * Hh + u;
    // dh from the vec path (this launch, sc1) + the carried-h path (previous launch)
    const auto dz = rsrc(a.DHZ, (int64_t)a.S_h * ntV * 8192 * 4);
    float t3[DHS];
#pragma unroll
    for (int s = 0; s < DHS; ++s) {
        const int ss = min(s, a.S_h - 1);
        t3[s] = ld_sc1_f32(dz, (uint32_t)(frag_idx((int64_t)ss * ntV + (u >> 6), b, u & 63) * 4));
    }
    float t1[8];
    if (a.dhr_on) {
#pragma unroll
        for (int s = 0; s < 8; ++s) t1[s] = a.DAY[(int64_t)min(s, a.S_ay - 1) * a.B * K + (int64_t)b * K + a.H + u];
    } else {
#pragma unroll
        for (int s = 0; s < 8; ++s) t1[s] = 0.f;
    }
    const float dcc = a.dhc_rec[ro], cp = a.hc_prev[ro];
    const float cx = ld_save(a.hchat, ro, a.save_lp), lcg = a.hlnc_g[u], lcb = a.hlnc_b[u];
    float xh[4], lg[4], lb[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        xh[q] = ld_save(a.hxhat, (int64_t)b * Gh + q * Hh + u, a.save_lp);
        lg[q] = a.hln_g[q * Hh + u];
        lb[q] = a.hln_b[q * Hh + u];
    }
    const float dhc = slab_fold<8>(t1, a.S_ay);
    const float dho = slab_fold<DHS>(t3, a.S_h);
    const float ig = cell_sig(xh[0] * lg[0] + lb[0]);
    const float tj = cell_tanh(xh[1] * lg[1] + lb[1]);
    const float fg = cell_sig(xh[2] * lg[2] + lb[2] + a.forget_bias);
    const float og = cell_sig(xh[3] * lg[3] + lb[3]);
    const float dh = dho + dhc;
    float dc = dcc;
    const float th = cell_tanh(cx * lcg + lcb);
    const float dout = dh * th;
    const float dcn = dh * og * (1.f - th * th);
    const float dch = on ? dcn * lcg : 0.f;
    float s2[2] = {dch, dch * cx};
    block_sum<2, 4>(s2, lds);
    const float rc = a.hrstd[b * 5 + 4];
    dc += rc * (dch - s2[0] / (float)Hh - cx * s2[1] / (float)Hh);
    const bool keep_on = a.hkeep < 1.0f;
    const uint32_t key = keep_on ? hash_key(*a.seed, a.hstream, a.step) : 0u;
    const float m = dropout_mult(keep_on, key, ro, a.hkeep);
    float dy[4], dly[4], acc[8];
    dy[0] = dc * tj * m * ig * (1.f - ig);
    dy[1] = dc * ig * m * (1.f - tj * tj);
    dy[2] = dc * cp * fg * (1.f - fg);
    dy[3] = dout * og * (1.f - og);
    const float dcr = dc * fg;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        dly[q] = dy[q];
        const float dg = on ? dy[q] * lg[q] : 0.f;
        dy[q] = dg;
        acc[q] = dg;
        acc[4 + q] = dg * xh[q];
    }
    float rsq[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) rsq[q] = a.hrstd[b * 5 + q];
    block_sum<8, 4>(acc, lds);
    if (on) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
            drow[q * Hh + tid] = to_bf16(rsq[q] * (dy[q] - acc[q] / (float)Hh - xh[q] * acc[4 + q] / (float)Hh));
    }
    lds_barrier();
    if (tid < Gh / 8) {   // dR_hyp row, 16-byte write-through stores (read in this launch)
        const auto dr = rsrc(a.dRY, (int64_t)a.B * Gh * 2);
        st_sc1(dr, (uint32_t)(((int64_t)b * Gh + 8 * tid) * 2), *(const u32x4v*)&drow[8 * tid]);
    }
    wg_arrive(&a.sync[1]);
    HS_STAMP(2);
    if (on) {   // saves for the parameter gradients and the carried-c gradient: after the hand-off
        st_save(a.hdlncy, ro, dcn, a.save_lp);
        a.dhc_rec[ro] = dcr;
#pragma unroll
        for (int q = 0; q < 4; ++q) st_save(a.hdlny, (int64_t)b * Gh + q * Hh + u, dly[q], a.save_lp);
    }
}

// d[h | hh] slab = dR_hyp[:, ks] @ W_y[n-tile, ks]^T; the weight slice is
// staged in LDS before the wait, dR_hyp is read after it (sc1, to registers)
template <int KSL>
__device__ void dry_tile(const HypBwdArgs& a, int id, __hip_bfloat16* smem) {
    constexpr int NCH = KSL / 8, SWM = (NCH < 16 ? NCH : 16) - 1, KS = KSL / 32;
    constexpr int PER = kBN * NCH / 256;          // 16-byte pieces per thread
    const int K = a.H + a.Hh, Gh = 4 * a.Hh, ntY = K / kBN;
    const int nt = id % ntY, s = id / ntY, k0 = s * KSL, n0 = nt * kBN;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, fq = lane >> 4;
    bf16x8 wv[PER];
    HS_STAMP(0);
#pragma unroll
    for (int p = 0; p < PER; ++p) {
        const int c = tid + 256 * p, row = c / NCH, ch = c - row * NCH;
        wv[p] = *(const bf16x8*)(a.Wyl + (int64_t)(n0 + row) * Gh + k0 + 8 * ch);
    }
#pragma unroll
    for (int p = 0; p < PER; ++p) {
        const int c = tid + 256 * p, row = c / NCH, ch = c - row * NCH;
        *(bf16x8*)(smem + row * KSL + ((ch ^ (row & SWM)) << 3)) = wv[p];
    }
    HS_STAMP(1);
    if (!wg_wait(&a.sync[1], a.epoch * (uint32_t)a.B, a.err)) return;   // (its barrier also publishes the slice)
    HS_STAMP(2);
    const auto dr = rsrc(a.dRY, (int64_t)a.B * Gh * 2);
    bf16x8 af[2][KS];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int row = 32 * w + 16 * i + fr;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
            af[i][ks] = row < a.B ? ld_sc1(dr, (uint32_t)(((int64_t)row * Gh + k0 + 32 * ks + 8 * fq) * 2)) : bf16x8{};
    }
    f32x4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = 16 * j + fr, ch = 4 * ks + fq;
            const bf16x8 bf = *(const bf16x8*)(smem + row * KSL + ((ch ^ (row & SWM)) << 3));
#pragma unroll
            for (int i = 0; i < 2; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][ks], bf, acc[i][j], 0, 0, 0);
        }
    float* C = a.DAY + (int64_t)s * a.B * K;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = 32 * w + 16 * i + 4 * fq + e;
                if (row < a.B) C[(int64_t)row * K + n0 + 16 * j + fr] = acc[i][j][e];
            }
    HS_STAMP(3);
}

template <int KSL, int DHS>
__global__ __launch_bounds__(256, 2) void hyper_bwd_step(const HypBwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) __hip_bfloat16 smem[];
    const int nV = (a.Hh / kBN) * a.S_h, nM = (a.H / kBN) * a.S_am;
    const int id = blockIdx.x;
    if (id < nV) dvec_tile(a, id, smem);
    else if (id < nV + nM) drm_tile(a, id - nV, smem);
    else if (id < nV + nM + a.B) hyper_row_bwd<DHS>(a, id - nV - nM, nV);
    else dry_tile<KSL>(a, id - nV - nM - a.B, smem);
}

}  // namespace

// One forward time step of the HyperLSTM (see the header); the main LayerNorm
// cell runs next as skr_lstm_fwd_step MOD 3 on GP / GS (gstat_tiles = H / 64).
// Shapes: B <= 128, H % 128 == 0 (so 4H / 64 tiles pair up in blocks of 16),
// Hh in {64, 128, 256}, (4 Hh / 64) * S_y tiles with (H + Hh) / S_y % 64 == 0,
// S_y <= 8.
SKR_API int skr_hyper_fwd_step(const HypFwdArgs* args, hipStream_t s) {
    const HypFwdArgs& a = *args;
    if (a.B < 1 || a.B > BM || a.H % 64 != 0 || (a.Hh != 64 && a.Hh != 128 && a.Hh != 256)) return -2;
    if (a.S_y < 1 || a.S_y > 8 || ((a.H + a.Hh) / a.S_y) % BK != 0 || (a.H + a.Hh) % a.S_y != 0) return -3;
    if (!a.A || !a.WhT || !a.WyT || !a.XH || !a.XHY || !a.hc_prev || !a.WzT || !a.WaT || !a.qb || !a.RY ||
        !a.A_next || !a.HH || !a.hc_out || !a.GP || !a.GS || !a.sync || !a.err || !a.seed)
        return -4;
    if (((uintptr_t)a.A | (uintptr_t)a.WhT | (uintptr_t)a.WyT | (uintptr_t)a.WzT | (uintptr_t)a.WaT |
         (uintptr_t)a.A_next | (uintptr_t)a.GP | (uintptr_t)a.RY) & 15)
        return -4;
    const int nY = (4 * a.Hh / kBN) * a.S_y, nR = 4 * a.H / kBNm;
    const int grid = nY + a.B + nR, waiting = a.B + nR;
    auto launch = [&](auto kern) {
        static bool attr = false;
        if (!attr) {
            (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsF);
            attr = true;
        }
        // the waiting workgroups (hyper rows, main tiles) must leave at least
        // one slot for a producer, whatever the dispatch order (2 per CU by LDS)
        if (!grid_fits((const void*)kern, 256, kLdsF, waiting + 1, 2)) return -8;
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), kLdsF, s, a);
        return SKR_CHECK_LAUNCH();
    };
    switch (a.Hh) {
        case 64: return launch(hyper_fwd_step<8>);
        case 128: return launch(hyper_fwd_step<16>);
        default: return launch(hyper_fwd_step<32>);
    }
}

SKR_API int skr_hyper_fwd_args_size() { return (int)sizeof(HypFwdArgs); }

// One backward time step after the main cell (see hyper_bwd_step above).
// Shapes: B <= 128, H % 64 == 0, Hh in {64, 128, 256}, 12H / S_h and 4H / S_am
// multiples of 64, S_h <= 64, S_ay <= 8 with 4 Hh / S_ay in {64, 128, 256}.
SKR_API int skr_hyper_bwd_step(const HypBwdArgs* args, hipStream_t s) {
    const HypBwdArgs& a = *args;
    if (a.B < 1 || a.B > BM || a.H % 64 != 0 || (a.Hh != 64 && a.Hh != 128 && a.Hh != 256)) return -2;
    const int NV = 12 * a.H, G = 4 * a.H, Gh = 4 * a.Hh, K = a.H + a.Hh;
    if (a.S_h < 1 || a.S_h > 64 || NV % a.S_h || (NV / a.S_h) % BK || a.S_am < 1 || G % a.S_am ||
        (G / a.S_am) % BK || a.S_ay < 1 || a.S_ay > 8 || Gh % a.S_ay || K % kBN)
        return -3;
    const int ksl = Gh / a.S_ay;
    if (ksl != 64 && ksl != 128 && ksl != 256) return -3;
    if (!a.dVEC || !a.Pl || !a.dRM || !a.Whl || !a.Wyl || !a.DHZ || !a.DAM || !a.DAY || !a.dhc_rec || !a.hc_prev ||
        !a.hchat || !a.hxhat || !a.hrstd || !a.dRY || !a.hdlny || !a.hdlncy || !a.sync || !a.err || !a.seed)
        return -4;
    if (((uintptr_t)a.dVEC | (uintptr_t)a.Pl | (uintptr_t)a.dRM | (uintptr_t)a.Whl | (uintptr_t)a.Wyl |
         (uintptr_t)a.dRY) & 15)
        return -4;
    const int nV = (a.Hh / kBN) * a.S_h, nM = (a.H / kBN) * a.S_am, nY = (K / kBN) * a.S_ay;
    const int grid = nV + nM + a.B + nY, waiting = a.B + nY;
    auto launch = [&](auto kern) {
        static bool attr = false;
        if (!attr) {
            (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
            attr = true;
        }
        // the waiting workgroups must leave at least one slot for a producer
        if (!grid_fits((const void*)kern, 256, kLds, waiting + 1, 2)) return -8;
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), kLds, s, a);
        return SKR_CHECK_LAUNCH();
    };
    const int dhs = a.S_h <= 8 ? 8 : a.S_h <= 32 ? 32 : 64;
#define SKR_HB(K_)                                                          \
    do {                                                                    \
        if (dhs == 8) return launch(hyper_bwd_step<K_, 8>);                 \
        if (dhs == 32) return launch(hyper_bwd_step<K_, 32>);               \
        return launch(hyper_bwd_step<K_, 64>);                              \
    } while (0)
    switch (ksl) {
        case 64: SKR_HB(64);
        case 128: SKR_HB(128);
        default: SKR_HB(256);
    }
#undef SKR_HB
}

SKR_API int skr_hyper_bwd_args_size() { return (int)sizeof(HypBwdArgs); }

// Diagnostic build: point the phase stamps at a device buffer ([grid][8] uint64; null: off).
SKR_API int skr_hstep_trace(void* buf) {
#ifdef SKR_TRACE_HSTEP
    uint64_t* p = (uint64_t*)buf;
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_hstep_trace), &p, sizeof(p));
#else
    (void)buf;
    return -1;
#endif
}
