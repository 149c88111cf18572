// EXPERIMENT (not built into libskrnn_hip.so; measured slower than the
// per-step launch chain, kept as the record of the design):
//   vae_large scan, B 100, T 250, bf16, one MI355X (scripts/bench_hyper.py):
//   forward 45.6 us/step persistent vs 36.5 us/step for the launch chain.
//   The in-kernel trace (profiles/r3/hyper_persist_trace.txt) shows every
//   dependency level -- poll + payload load + compute + write-through drain
//   -- costing 5-8 us, the same as a kernel boundary + ramp + drain of the
//   chain, while the recurrence needs six levels per step either way (R
//   partials, hyper cell, modulation vectors, main cell, two LayerNorm
//   exchanges). Only the weight stream is saved, and the R_main MFMA work
//   (~3.8 GFLOP per step) then sits on every workgroup's critical path.
//   To try it: build this file into the library and route _HyperSeq.forward
//   to skr_hyper_persist_fwd (see git history, round 3).
//
// Persistent HyperLSTM forward (the vae_large decoder: H = 2048 main units,
// Hh = 256 hyper units, LayerNorm in both cells) -- ONE launch runs every
// time step of the recurrence. Reference recurrence: /root/reference
// model.py:66-95 (the static unroll; sketch-rnn's HyperLSTM cell semantics are
// the oracle in sketch_rnn_amd/models/cells.py hyper_lstm_step).
//
// Why: as a per-step launch chain (grouped GEMM, hyper cell, modulation GEMM,
// main cell) every step re-streams 50 MB of bf16 weights and pays four
// kernel ramps/drains (~40 us per step at B = 100). Here every weight a step
// needs lives on chip for the whole sequence and only activations move:
//
//   grid: 256 workgroups x 512 threads, one per CU (all co-resident; the
//   launcher checks). Workgroup g = 8 j + x: x = "slice" (0..7; blocks g and
//   g + 8 share an XCD under round-robin placement, so a slice's 32 workgroups
//   usually sit on one XCD -- speed only, never correctness), j = 0..31.
//   Slice x owns the hidden units U_x = [256 x, 256 x + 256).
//
//   VGPR-resident weights (loaded once):
//     W_h[U_x (K rows), column group j] -- 256 x 256 bf16 = 128 KB per WG,
//       column group j = gate q = j / 8, units U_(j % 8): MFMA B fragments,
//       16 per wave (2 column tiles x 8 k-steps) = 64 VGPRs;
//     P[:, 96 modulation columns] (vec = hh @ P + q, P = W_z W_a folded;
//       slice x's units, k-blocks 6 (j / 16) .. + 5, units 16 (j % 16)..+15),
//       8 fragments for waves 0-5.
//   LDS: h_{t-1}[:, U_x] and hh staging (56 KB each, XOR-swizzled), the
//   workgroup's W_y slice (hyper gates 32 j..32 j + 31 over K rows U_x and hh
//   rows 32 x..32 x + 31; 18 KB).
//
// Per step t, four phases, every dependency a point-to-point in-launch
// hand-off (write-through sc1 payload, drained, one flag per producer; the
// consumer polls with sc1 loads and reads with sc1 loads only: CDNA4 guide
// Guideline 16, first row of the measured sc1 table):
//   A (column owner, every WG): wait for h_{t-1}[:, U_x] (the 32 WGs of slice
//     x), stage it in LDS, MFMA the partial R_main = h[:, U_x] @ W_h[U_x, grp j]
//     and the partial R_hyp = [h | hh] @ W_y (K rows U_x + hh rows 32x..),
//     publish both (bf16 R_main partial rows through an LDS transpose).
//   B (hyper row owner, WG 8 j + x = row b < B): wait for every phase-A
//     flag, sum the 8 slices' R_hyp partials, LayerNorm-LSTM hyper cell
//     (c in registers across steps), publish hh_t (bf16).
//   C (modulation, every WG): wait for all hh_t, vec = hh_t @ P + q for the
//     WG's 96 columns on MFMA, publish (bf16; also the backward's save).
//   D (main row owner: rows j, j + 32, j + 64, j + 96 of slice x): sum the 8
//     K-slice partials of R_main, g = xh * vx + R * vh + vb, LayerNorm over
//     each gate (row statistics exchanged between the 8 slices of the row as
//     data-tagged 8-byte granules), cell update (c in registers), LayerNorm
//     over c (second exchange), h = tanh(LN c) * sig(o) -> publish h_t.
// The saves are exactly those of the per-step cell kernels (xhat, rstd,
// chat, bf16 R, vec, carried c / h), so the existing reverse-time kernels
// (csrc/lstm_cell.hip, csrc/skinny_gemm.hip) run the backward unchanged.
// Every wait is bounded (a timeout sets *err; every later wait then returns
// at once, so the grid always drains and the host raises).
#include "common.h"

namespace {

using namespace skr;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int H = 2048, HH = 256, G = 4 * H, GH = 4 * HH, K = H + HH, NV = 12 * H;
constexpr int NX = 8, NJ = 32, NWG = NX * NJ;
constexpr int NTH = 512, NW = NTH / 64;
constexpr int MAXB = 112, NRT = MAXB / 16;       // row tiles of 16
constexpr int WYK = 288, WYLD = 296;             // W_y slice: 256 + 32 k per row, padded row (conflict-free)
constexpr int PLD = 264;                         // P slice row: 256 k + 8 pad (conflict-free fragment reads)
// LDS carve (bf16 elements): X [MAXB][256] (phase A: h slice + R_main
// transpose; C: hh_t; D: gate activations), hh chunk [MAXB][32], vec
// transpose [6][MAXB][16], W_y slice [32][WYLD], P slice [96][PLD]
constexpr int L_X = 0, L_HC = MAXB * 256, L_V = L_HC + MAXB * 32, L_WY = L_V + 6 * MAXB * 16,
              L_P = L_WY + 32 * WYLD, L_END = L_P + 96 * PLD;
constexpr int kSc1 = 16;
constexpr unsigned kSpin = 1u << 22;
constexpr float kEps = 1e-3f;

}  // namespace

struct HPArgs {
    int T, B;
    const __hip_bfloat16* WhT;     // [G][H]   B^T of h @ W_h
    const __hip_bfloat16* WyT;     // [GH][K]  B^T of [h | hh] @ W_y
    const __hip_bfloat16* PlT;     // [NV][HH] B^T of hh @ P
    const float* qb;               // [NV] q (+ the main bias folded into blocks 8..11)
    const float* XH;               // [T][B][G]   x-projection of the main gates
    const float* XHY;              // [T][B][GH]  x-projection of the hyper gates
    const float* ln_g; const float* ln_b; const float* lnc_g; const float* lnc_b;
    const float* hln_g; const float* hln_b; const float* hlnc_g; const float* hlnc_b;
    const float* c0;               // [B][H]
    const float* hc0;              // [B][HH]
    float forget_bias, keep, hkeep;
    const int64_t* seed; uint32_t stream;
    __hip_bfloat16* A;             // [T+1][B][K]: A[0] = (h0 | hh0) preset; A[t+1] written
    __hip_bfloat16* PM;            // [2][NX][B][G] R_main partials
    float* PY;                     // [2][NX][NJ][NRT][2][64][4] R_hyp partials (MFMA fragment order)
    __hip_bfloat16* VEC;           // [T][B][NV]
    float* Hout;                   // [T][B][H]
    float* CC;                     // [T+1][B][H]  (CC[0] preset = c0)
    float* HCC;                    // [T+1][B][HH] (HCC[0] preset = hc0)
    float* HH_out;                 // [T][B][HH]
    float* XHAT; float* RSTD; float* CHAT; __hip_bfloat16* RLP;   // main saves (null: inference)
    float* HXHAT; float* HRSTD; float* HCHAT;                      // hyper saves
    uint32_t* flags;               // [4][256] zeroed by the launcher
    uint64_t* part;                // [2][MAXB][NX][8] LN granules, zeroed by the launcher
    int* err;
    uint64_t* trace;               // diagnostic [T][256][16] s_memrealtime stamps (wave 0), or null
};

namespace {

__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk_rsrc(const void* p, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)(bytes > 0x7fffffff ? 0x7fffffff : bytes),
                                             0x00020000);
}
__device__ __forceinline__ u32x4 ld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kSc1);
}
__device__ __forceinline__ uint32_t ld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, kSc1);
}
__device__ __forceinline__ void st16(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kSc1);
}
__device__ __forceinline__ void st8(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x2 v) {
    __builtin_amdgcn_raw_buffer_store_b64(v, r, off, 0, kSc1);
}
__device__ __forceinline__ float bf_lo(uint32_t v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float bf_hi(uint32_t v) { return __uint_as_float(v & 0xffff0000u); }
__device__ __forceinline__ uint32_t pack_bf(float a, float b) {
    const uint32_t lo = __bfloat16_as_ushort(__float2bfloat16(a));
    const uint32_t hi = __bfloat16_as_ushort(__float2bfloat16(b));
    return lo | (hi << 16);
}
__device__ __forceinline__ float tanh_(float x) { return tanhf(x); }
__device__ __forceinline__ float dropout_mult_(bool on, uint32_t key, int64_t idx, float keep) {
    if (!on) return 1.f;
    return hash_uniform(key, (uint32_t)idx) < keep ? 1.0f / keep : 0.f;
}

__global__ void zero_words(uint32_t* a, int na, uint32_t* b, int nb) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < na) a[i] = 0u;
    else if (i < na + nb) b[i - na] = 0u;
}

// One wave: wait until flags[idx(i)] >= epoch for i < n (each lane polls
// n / 64 rounded up). Bounded; on a timeout or an earlier error returns false.
template <typename F>
__device__ bool wave_wait(const uint32_t* flags, int n, F idx, uint32_t epoch, int* err) {
    const int lane = threadIdx.x & 63;
    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return false;
    for (unsigned spins = 0;; ++spins) {
        bool ok = true;
        for (int i = lane; i < n; i += 64)
            ok &= __hip_atomic_load(flags + idx(i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= epoch;
        if (__all(ok)) break;
        if ((spins & 255) == 255) {
            if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return false;
            if (spins > kSpin) {
                if (lane == 0) __hip_atomic_store(err, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return false;
            }
        }
        __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler barrier: payload loads stay below
    return true;
}

__device__ __forceinline__ void publish(uint32_t* f, uint32_t epoch) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(f, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Swizzled [row][256] bf16 LDS tile: 16-byte chunk c of row r at chunk c ^ (r & 15).
__device__ __forceinline__ int sw(int row, int chunk) { return row * 256 + ((chunk ^ (row & 15)) << 3); }
// Swizzled [row][32] bf16 tile (the hh chunk): chunk c (0..3) of row r at c ^ ((r >> 2) & 3).
__device__ __forceinline__ int swc(int row, int chunk) { return row * 32 + ((chunk ^ ((row >> 2) & 3)) << 3); }

// Block sum of N values over all 8 waves (every thread calls it).
template <int N>
__device__ __forceinline__ void bsum(float (&v)[N], float* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = wave_sum(v[i]);
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < N; ++i) red[w * N + i] = v[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < N; ++i) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < NW; ++k) s += red[k * N + i];
        v[i] = s;
    }
    __syncthreads();
}

// Sum over the 32 lanes of this lane's half-wave (every lane active).
__device__ __forceinline__ float half_sum(float v) {
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 8, 64);
    v += __shfl_xor(v, 16, 64);
    return v;
}

#define HP_STAMP(i)                                                                          \
    do {                                                                                     \
        if (a.trace != nullptr && threadIdx.x == 0)                                          \
            a.trace[((int64_t)t * NWG + g) * 16 + (i)] = __builtin_amdgcn_s_memrealtime();   \
    } while (0)

template <bool SAVE>
__global__ __launch_bounds__(NTH) void hyper_persist_fwd(const HPArgs a) {
    extern __shared__ __attribute__((aligned(16))) __hip_bfloat16 smem[];
    __hip_bfloat16* sH = smem + L_X;                    // [MAXB][256] h slice / transpose / hh_t
    __hip_bfloat16* sHc = smem + L_HC;                  // [MAXB][32] hh chunk x (R_hyp's hh rows)
    __hip_bfloat16* sV = smem + L_V;                    // [6][MAXB][16] vec transpose
    __hip_bfloat16* sWy = smem + L_WY;                  // [32][WYLD]
    __hip_bfloat16* sP = smem + L_P;                    // [96][PLD]
    float* red = (float*)(smem + L_END);                // [NW * 8]
    float* sAct = (float*)sH;                           // phase D: [4 rows][4 gates][256] (aliases sH)

    const int g = blockIdx.x, x = g & 7, j = g >> 3;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const int T = a.T, B = a.B;
    uint32_t* flagA = a.flags;
    uint32_t* flagB = a.flags + 256;
    uint32_t* flagC = a.flags + 512;
    uint32_t* flagD = a.flags + 768;
    uint64_t* part1 = a.part;
    uint64_t* part2 = a.part + MAXB * NX * 8;
    int* err = a.err;

    const auto rA = mk_rsrc(a.A, (int64_t)(T + 1) * B * K * 2);
    const auto rPM = mk_rsrc(a.PM, (int64_t)2 * NX * B * G * 2);
    const auto rPY = mk_rsrc(a.PY, (int64_t)2 * NX * NJ * NRT * 2 * 64 * 4 * 4);
    const auto rV = mk_rsrc(a.VEC, (int64_t)T * B * NV * 2);

    // ---------------- one-time setup ----------------
    // W_h fragments: wave w owns column tiles (2w, 2w+1) of group j over K rows U_x
    const int qj = j >> 3, uj = 256 * (j & 7);          // column group j = gate qj, units uj..uj+255
    bf16x8 wh[2][8];
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            const int n = qj * H + uj + 32 * w + 16 * ct + fr;
            wh[ct][ks] = *(const bf16x8*)(a.WhT + (int64_t)n * H + 256 * x + 32 * ks + 8 * fq);
        }
    // P slice -> LDS: row c = 16 wv + u (wv = k-block 6 (j / 16) + wv, unit uv + u)
    const int uv = 256 * x + 16 * (j & 15);
    for (int i = tid; i < 96 * 32; i += NTH) {
        const int c = i >> 5, ch = i & 31;
        const int n = (6 * (j >> 4) + (c >> 4)) * H + uv + (c & 15);
        *(bf16x8*)(sP + c * PLD + 8 * ch) = *(const bf16x8*)(a.PlT + (int64_t)n * HH + 8 * ch);
    }
    const float qbv = w < 6 ? a.qb[(6 * (j >> 4) + w) * H + uv + fr] : 0.f;
    // W_y slice -> LDS: row c = hyper gate column 32 j + c; k 0..255 = U_x, 256..287 = hh rows 32x..
    for (int i = tid; i < 32 * (WYK / 8); i += NTH) {
        const int c = i / (WYK / 8), ch = i % (WYK / 8);
        const int64_t src = ch < 32 ? (int64_t)256 * x + 8 * ch : (int64_t)H + 32 * x + 8 * (ch - 32);
        *(bf16x8*)(sWy + c * WYLD + 8 * ch) = *(const bf16x8*)(a.WyT + (int64_t)(32 * j + c) * K + src);
    }
    // zero the staging tiles (rows >= B stay zero), stage chunk x of hh_{-1} = hh0
    for (int i = tid; i < (MAXB * 256 + MAXB * 32) / 8; i += NTH) *(u32x4*)(smem + 8 * i) = u32x4{0u, 0u, 0u, 0u};
    __syncthreads();
    for (int i = tid; i < B * 4; i += NTH) {
        const int r = i >> 2, ch = i & 3;
        *(bf16x8*)(sHc + swc(r, ch)) = *(const bf16x8*)(a.A + (int64_t)r * K + H + 32 * x + 8 * ch);
    }
    // phase-D thread roles (recomputed per step): row slot r = w / 2 (rows
    // j + 32 r), gate q, 8 units; cell roles: even waves, row w / 2, 4 units per lane
    const int cb0 = j + 32 * (w >> 1);
    const bool crow0 = (w & 1) == 0 && cb0 < B;
    float cst[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) cst[i] = crow0 ? a.c0[(int64_t)cb0 * H + 256 * x + 4 * lane + i] : 0.f;
    // hyper row owner (phase B): row hb = 8 j + x, thread u = tid < 256
    const int hb = 8 * j + x;
    float hcst = (hb < B && tid < HH) ? a.hc0[(int64_t)hb * HH + tid] : 0.f;
    __syncthreads();

    for (int t = 0; t < T; ++t) {
        const uint32_t ep = t + 1;
        // per-thread index math is redone every step from a laundered thread
        // id: hoisted out of the loop it would pin ~100 address registers
        int tl = tid;
        asm volatile("" : "+v"(tl));
        const int lane = tl & 63, w = __builtin_amdgcn_readfirstlane(tl >> 6);
        const int fr = lane & 15, fq = lane >> 4;
        const int dr = w >> 1, dq = (tl >> 5) & 3, dc8 = tl & 31;
        const int db = j + 32 * dr;
        const bool drow = db < B;
        const int du = 256 * x + 8 * dc8;
        const int cr = w >> 1, cb = j + 32 * cr;
        const bool crow = (w & 1) == 0 && cb < B;
        const int cu = 256 * x + 4 * lane;
        const int hu = tl & (HH - 1);
        const bool hrow = hb < B && tl < HH;
        // ================= A: column owner =================
        HP_STAMP(0);
        if (t > 0 && w == 0) wave_wait(flagD, NJ, [&](int i) { return 8 * i + x; }, (uint32_t)t, err);
        HP_STAMP(1);
        __syncthreads();
        for (int i = tid; i < B * 32; i += NTH) {
            const int r = i >> 5, ch = i & 31;
            const u32x4 v = ld16(rA, (uint32_t)((((int64_t)t * B + r) * K + 256 * x + 8 * ch) * 2));
            *(u32x4*)(sH + sw(r, ch)) = v;
        }
        __syncthreads();
        f32x4 acc[NRT][2];
#pragma unroll
        for (int rt = 0; rt < NRT; ++rt) acc[rt][0] = acc[rt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
#pragma unroll
            for (int rt = 0; rt < NRT; ++rt) {
                const bf16x8 af = *(const bf16x8*)(sH + sw(16 * rt + fr, 4 * ks + fq));
                acc[rt][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, wh[0][ks], acc[rt][0], 0, 0, 0);
                acc[rt][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, wh[1][ks], acc[rt][1], 0, 0, 0);
            }
        }
        // R_hyp partial: wave w -> column tile (w & 1), row tiles w/2 and w/2 + 4
        const int hct = w & 1, hr0 = w >> 1, hr1 = (w >> 1) + 4;
        f32x4 hy0 = f32x4{0.f, 0.f, 0.f, 0.f}, hy1 = hy0;
#pragma unroll
        for (int ks = 0; ks < 9; ++ks) {
            const bf16x8 bw = *(const bf16x8*)(sWy + (16 * hct + fr) * WYLD + 32 * ks + 8 * fq);
            const bf16x8 a0 = ks < 8 ? *(const bf16x8*)(sH + sw(16 * hr0 + fr, 4 * ks + fq))
                                     : *(const bf16x8*)(sHc + swc(16 * hr0 + fr, fq));
            hy0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bw, hy0, 0, 0, 0);
            if (hr1 < NRT) {
                const bf16x8 a1 = ks < 8 ? *(const bf16x8*)(sH + sw(16 * hr1 + fr, 4 * ks + fq))
                                         : *(const bf16x8*)(sHc + swc(16 * hr1 + fr, fq));
                hy1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bw, hy1, 0, 0, 0);
            }
        }
        {
            const uint32_t base = (uint32_t)(((((t & 1) * NX + x) * NJ + j) * NRT) * 2);
            st16(rPY, ((base + hr0 * 2 + hct) * 64 + lane) * 16, __builtin_bit_cast(u32x4, hy0));
            if (hr1 < NRT) st16(rPY, ((base + hr1 * 2 + hct) * 64 + lane) * 16, __builtin_bit_cast(u32x4, hy1));
        }
        HP_STAMP(2);
        __syncthreads();   // every wave done reading sH
        // R_main partial -> bf16 rows in LDS (transpose) -> 16-byte write-through row stores
#pragma unroll
        for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int row = 16 * rt + 4 * fq + i, col = 32 * w + 16 * ct + fr;
                    sH[sw(row, col >> 3) + (col & 7)] = __float2bfloat16(acc[rt][ct][i]);
                }
        __syncthreads();
        for (int i = tid; i < B * 32; i += NTH) {
            const int r = i >> 5, ch = i & 31;
            const u32x4 v = *(const u32x4*)(sH + sw(r, ch));
            st16(rPM, (uint32_t)(((((int64_t)(t & 1) * NX + x) * B + r) * G + qj * H + uj + 8 * ch) * 2), v);
        }
        publish(flagA + g, ep);
        HP_STAMP(3);

        // ================= B: hyper row owner =================
        if (hb < B) {
            if (w == 0) wave_wait(flagA, NWG, [](int i) { return i; }, ep, err);
            HP_STAMP(4);
            __syncthreads();
            float gq[4];
            if (tid < HH) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int hc = q * HH + hu, jj = hc >> 5, ct = (hc >> 4) & 1;
                    const int ln = 16 * ((hb & 15) >> 2) + (hc & 15), e = hb & 3, rt = hb >> 4;
                    float s = a.XHY[((int64_t)t * B + hb) * GH + hc];
                    float p[NX];
#pragma unroll
                    for (int xs = 0; xs < NX; ++xs) {
                        const uint32_t idx = ((((((t & 1) * NX + xs) * NJ + jj) * NRT + rt) * 2 + ct) * 64 + ln) * 4 + e;
                        p[xs] = __uint_as_float(ld4(rPY, idx * 4));
                    }
#pragma unroll
                    for (int xs = 0; xs < NX; ++xs) s += p[xs];
                    gq[q] = s;
                }
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) gq[q] = 0.f;
            }
            float st[8];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                st[q] = gq[q];
                st[4 + q] = gq[q] * gq[q];
            }
            bsum<8>(st, red);
            float hx[4], hrs[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float mean = st[q] / (float)HH;
                const float var = fmaxf(st[4 + q] / (float)HH - mean * mean, 0.f);
                hrs[q] = rsqrtf(var + kEps);
                hx[q] = (gq[q] - mean) * hrs[q];
            }
            const float yi = hx[0] * a.hln_g[hu] + a.hln_b[hu];
            const float yj = hx[1] * a.hln_g[HH + hu] + a.hln_b[HH + hu];
            const float yf = hx[2] * a.hln_g[2 * HH + hu] + a.hln_b[2 * HH + hu];
            const float yo = hx[3] * a.hln_g[3 * HH + hu] + a.hln_b[3 * HH + hu];
            const bool hkon = a.hkeep < 1.f;
            const uint32_t hkey = hkon ? hash_key(*a.seed, a.stream + 1, t) : 0u;
            const float hm = hrow ? dropout_mult_(hkon, hkey, (int64_t)hb * HH + hu, a.hkeep) : 0.f;
            const float hcn = hrow ? hcst * sigmoidf_(yf + a.forget_bias) + sigmoidf_(yi) * tanh_(yj) * hm : 0.f;
            float s2[2] = {hcn, hcn * hcn};
            bsum<2>(s2, red);
            const float cm = s2[0] / (float)HH;
            const float crs = rsqrtf(fmaxf(s2[1] / (float)HH - cm * cm, 0.f) + kEps);
            const float chh = (hcn - cm) * crs;
            const float hhv = tanh_(chh * a.hlnc_g[hu] + a.hlnc_b[hu]) * sigmoidf_(yo);
            // hh_t -> bf16 via LDS (16-byte write-through stores)
            __hip_bfloat16* sO = (__hip_bfloat16*)(red + NW * 8);   // 512 B scratch after the reduction words
            if (tid < HH) sO[hu] = __float2bfloat16(hhv);
            __syncthreads();
            if (tid < HH / 8)
                st16(rA, (uint32_t)((((int64_t)(t + 1) * B + hb) * K + H + 8 * tid) * 2), *(const u32x4*)(sO + 8 * tid));
            publish(flagB + hb, ep);
            HP_STAMP(5);
            if (hrow) {
                hcst = hcn;
                const int64_t ro = (int64_t)t * B + hb;
                a.HH_out[ro * HH + hu] = hhv;
                a.HCC[(ro + B) * HH + hu] = hcn;
                if (SAVE) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) a.HXHAT[ro * GH + q * HH + hu] = hx[q];
                    a.HCHAT[ro * HH + hu] = chh;
                    if (hu == 0) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) a.HRSTD[ro * 5 + q] = hrs[q];
                        a.HRSTD[ro * 5 + 4] = crs;
                    }
                }
            }
        }

        // ================= C: modulation vectors =================
        if (w == 0) wave_wait(flagB, B, [](int i) { return i; }, ep, err);
        HP_STAMP(6);
        __syncthreads();
        for (int i = tid; i < B * 32; i += NTH) {
            const int r = i >> 5, ch = i & 31;
            const u32x4 v = ld16(rA, (uint32_t)((((int64_t)(t + 1) * B + r) * K + H + 8 * ch) * 2));
            *(u32x4*)(sH + sw(r, ch)) = v;
            if ((ch >> 2) == x) *(u32x4*)(sHc + swc(r, ch & 3)) = v;   // next step's R_hyp hh rows
        }
        __syncthreads();
        if (w < 6) {
            f32x4 vacc[NRT];
#pragma unroll
            for (int rt = 0; rt < NRT; ++rt) vacc[rt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 8; ++ks)
#pragma unroll
                for (int rt = 0; rt < NRT; ++rt) {
                    const bf16x8 af = *(const bf16x8*)(sH + sw(16 * rt + fr, 4 * ks + fq));
                    const bf16x8 bp = *(const bf16x8*)(sP + (16 * w + fr) * PLD + 32 * ks + 8 * fq);
                    vacc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bp, vacc[rt], 0, 0, 0);
                }
#pragma unroll
            for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
                for (int i = 0; i < 4; ++i) sV[(w * MAXB + 16 * rt + 4 * fq + i) * 16 + fr] = __float2bfloat16(vacc[rt][i] + qbv);
        }
        __syncthreads();
        for (int i = tid; i < 6 * B * 2; i += NTH) {
            const int wv = i / (2 * B), rem = i - wv * 2 * B, r = rem >> 1, hf = rem & 1;
            const int kbw = 6 * (j >> 4) + wv;
            st16(rV, (uint32_t)((((int64_t)t * B + r) * NV + kbw * H + uv + 8 * hf) * 2),
                 *(const u32x4*)(sV + (wv * MAXB + r) * 16 + 8 * hf));
        }
        publish(flagC + g, ep);
        HP_STAMP(7);

        // ================= D: main row owner =================
        // loads of this thread's 8 units of gate dq for row db
        float xh[8], rs8[8], vx[8], vh[8], vb[8];
        if (drow) {
            const float* xp = a.XH + ((int64_t)t * B + db) * G + dq * H + du;
            const f32x4 x0 = *(const f32x4*)xp, x1 = *(const f32x4*)(xp + 4);
#pragma unroll
            for (int i = 0; i < 4; ++i) { xh[i] = x0[i]; xh[4 + i] = x1[i]; }
        }
        // the R_main partials of gate dq, units U_x: column groups j' = 8 dq + x of every slice
        wave_wait(flagA, 2 * NX, [&](int i) { return 8 * (8 * ((w & 1) * 2 + (i >> 3)) + x) + (i & 7); }, ep, err);
        if (drow) {
            u32x4 pv[NX];
#pragma unroll
            for (int xs = 0; xs < NX; ++xs)
                pv[xs] = ld16(rPM, (uint32_t)(((((int64_t)(t & 1) * NX + xs) * B + db) * G + dq * H + du) * 2));
#pragma unroll
            for (int i = 0; i < 8; ++i) rs8[i] = 0.f;
#pragma unroll
            for (int xs = 0; xs < NX; ++xs)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    rs8[2 * i] += bf_lo(pv[xs][i]);
                    rs8[2 * i + 1] += bf_hi(pv[xs][i]);
                }
        }
        HP_STAMP(8);
        wave_wait(flagC, NJ, [&](int i) { return 8 * i + x; }, ep, err);
        HP_STAMP(9);
        if (drow) {
            const uint32_t vo = (uint32_t)(((int64_t)t * B + db) * NV + du);
            const u32x4 ax = ld16(rV, (vo + dq * H) * 2), ah = ld16(rV, (vo + (4 + dq) * H) * 2),
                        ab = ld16(rV, (vo + (8 + dq) * H) * 2);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                vx[2 * i] = bf_lo(ax[i]); vx[2 * i + 1] = bf_hi(ax[i]);
                vh[2 * i] = bf_lo(ah[i]); vh[2 * i + 1] = bf_hi(ah[i]);
                vb[2 * i] = bf_lo(ab[i]); vb[2 * i + 1] = bf_hi(ab[i]);
            }
        }
        float gv[8], s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            gv[i] = drow ? xh[i] * vx[i] + rs8[i] * vh[i] + vb[i] : 0.f;
            s1 += gv[i];
            s2 += gv[i] * gv[i];
        }
        s1 = half_sum(s1);
        s2 = half_sum(s2);
        HP_STAMP(10);
        // exchange 1: (sum, sum sq) of gate dq over U_x -> granules of row db, slice x
        if (drow && dc8 == 0) {
            uint64_t* gp = part1 + ((int64_t)db * NX + x) * 8 + 2 * dq;
            __hip_atomic_store(gp, ((uint64_t)ep << 32) | __float_as_uint(s1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(gp + 1, ((uint64_t)ep << 32) | __float_as_uint(s2), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        float tot = 0.f;
        if (drow) {   // wave-uniform (a wave holds one row)
            const uint64_t* gp = part1 + ((int64_t)db * NX + (lane >> 3)) * 8 + (lane & 7);
            uint64_t v = 0;
            for (unsigned spins = 0;; ++spins) {
                v = __hip_atomic_load(gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (__all((uint32_t)(v >> 32) == ep)) break;
                if ((spins & 255) == 0) {
                    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) break;
                    if (spins > kSpin) {
                        if (lane == 0) __hip_atomic_store(err, 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                }
                __builtin_amdgcn_s_sleep(1);
            }
            tot = __uint_as_float((uint32_t)v);
            tot += __shfl_xor(tot, 8, 64);
            tot += __shfl_xor(tot, 16, 64);
            tot += __shfl_xor(tot, 32, 64);   // lane s (< 8): total of stat s over the 8 slices
        }
        const float S1 = __shfl(tot, 2 * dq, 64), S2 = __shfl(tot, 2 * dq + 1, 64);
        const float mean = S1 / (float)H;
        const float rsd = rsqrtf(fmaxf(S2 / (float)H - mean * mean, 0.f) + kEps);
        float xs8[8];
        const bool kon = a.keep < 1.f;
        const uint32_t key = kon ? hash_key(*a.seed, a.stream, t) : 0u;
        HP_STAMP(11);
        __syncthreads();   // sAct (aliases sH) free: phase C's readers are done
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            xs8[i] = (gv[i] - mean) * rsd;
            const float y = xs8[i] * a.ln_g[dq * H + du + i] + a.ln_b[dq * H + du + i];
            float act;
            if (dq == 0) act = sigmoidf_(y);
            else if (dq == 1) act = tanh_(y) * dropout_mult_(kon, key, (int64_t)db * H + du + i, a.keep);
            else if (dq == 2) act = sigmoidf_(y + a.forget_bias);
            else act = sigmoidf_(y);
            sAct[(dr * 4 + dq) * 256 + 8 * dc8 + i] = act;
        }
        __syncthreads();
        float cn[4] = {0.f, 0.f, 0.f, 0.f}, og[4] = {0.f, 0.f, 0.f, 0.f};
        float ch[4], hv[4];
        float crsd = 0.f;
        if (crow) {
            const float* ap = sAct + cr * 4 * 256 + 4 * lane;
            const f32x4 ai = *(const f32x4*)ap, aj = *(const f32x4*)(ap + 256), af = *(const f32x4*)(ap + 512),
                        ao = *(const f32x4*)(ap + 768);
            float c1 = 0.f, c2 = 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                cn[i] = cst[i] * af[i] + ai[i] * aj[i];
                og[i] = ao[i];
                c1 += cn[i];
                c2 += cn[i] * cn[i];
            }
            c1 = wave_sum(c1);
            c2 = wave_sum(c2);
            uint64_t* gp = part2 + ((int64_t)cb * NX + x) * 8;
            if (lane == 0) {
                __hip_atomic_store(gp, ((uint64_t)ep << 32) | __float_as_uint(c1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(gp + 1, ((uint64_t)ep << 32) | __float_as_uint(c2), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
            const uint64_t* rp = part2 + ((int64_t)cb * NX + ((lane >> 1) & 7)) * 8 + (lane & 1);
            uint64_t v = 0;
            for (unsigned spins = 0;; ++spins) {
                v = __hip_atomic_load(rp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (__all((uint32_t)(v >> 32) == ep)) break;
                if ((spins & 255) == 0) {
                    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) break;
                    if (spins > kSpin) {
                        if (lane == 0) __hip_atomic_store(err, 6, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                }
                __builtin_amdgcn_s_sleep(1);
            }
            float tv = __uint_as_float((uint32_t)v);   // lanes 0..15: slice (lane >> 1), stat lane & 1
            tv += __shfl_xor(tv, 2, 64);
            tv += __shfl_xor(tv, 4, 64);
            tv += __shfl_xor(tv, 8, 64);
            HP_STAMP(12);
            const float C1 = __shfl(tv, 0, 64), C2 = __shfl(tv, 1, 64);
            const float cmean = C1 / (float)H;
            crsd = rsqrtf(fmaxf(C2 / (float)H - cmean * cmean, 0.f) + kEps);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                ch[i] = (cn[i] - cmean) * crsd;
                hv[i] = tanh_(ch[i] * a.lnc_g[cu + i] + a.lnc_b[cu + i]) * og[i];
            }
            st8(rA, (uint32_t)((((int64_t)(t + 1) * B + cb) * K + cu) * 2),
                u32x2{pack_bf(hv[0], hv[1]), pack_bf(hv[2], hv[3])});
        }
        publish(flagD + g, ep);
        HP_STAMP(13);
        // saves (plain stores, after the hand-off)
        if (crow) {
            const int64_t ro = ((int64_t)t * B + cb) * H + cu;
            *(f32x4*)(a.Hout + ro) = f32x4{hv[0], hv[1], hv[2], hv[3]};
            *(f32x4*)(a.CC + ro + (int64_t)B * H) = f32x4{cn[0], cn[1], cn[2], cn[3]};
#pragma unroll
            for (int i = 0; i < 4; ++i) cst[i] = cn[i];
            if (SAVE) {
                *(f32x4*)(a.CHAT + ro) = f32x4{ch[0], ch[1], ch[2], ch[3]};
                if (x == 0 && lane == 0) a.RSTD[((int64_t)t * B + cb) * 5 + 4] = crsd;
            }
        }
        if (SAVE && drow) {
            const int64_t ro = ((int64_t)t * B + db) * G + dq * H + du;
            *(f32x4*)(a.XHAT + ro) = f32x4{xs8[0], xs8[1], xs8[2], xs8[3]};
            *(f32x4*)(a.XHAT + ro + 4) = f32x4{xs8[4], xs8[5], xs8[6], xs8[7]};
            *(u32x4*)(a.RLP + ro) = u32x4{pack_bf(rs8[0], rs8[1]), pack_bf(rs8[2], rs8[3]), pack_bf(rs8[4], rs8[5]),
                                           pack_bf(rs8[6], rs8[7])};
            if (x == 0 && dc8 == 0) a.RSTD[((int64_t)t * B + db) * 5 + dq] = rsd;
        }
    }
}

}  // namespace

// Workgroup -> slice mapping needs exactly 256 co-resident workgroups.
SKR_API int skr_hyper_persist_flag_words() { return 4 * 256; }
SKR_API int skr_hyper_persist_part_words() { return 2 * MAXB * NX * 8; }
SKR_API int skr_hyper_persist_args_size() { return (int)sizeof(HPArgs); }

SKR_API int skr_hyper_persist_fwd(const HPArgs* a, hipStream_t s) {
    if (a->T <= 0) return 0;
    if (a->B < 1 || a->B > MAXB) return -2;
    if (((uintptr_t)a->A | (uintptr_t)a->PM | (uintptr_t)a->VEC | (uintptr_t)a->WhT | (uintptr_t)a->WyT |
         (uintptr_t)a->PlT | (uintptr_t)a->XH | (uintptr_t)a->Hout | (uintptr_t)a->CC) & 15)
        return -4;
    const bool save = a->XHAT != nullptr;
    if (save && (a->RSTD == nullptr || a->CHAT == nullptr || a->RLP == nullptr || a->HXHAT == nullptr ||
                 a->HRSTD == nullptr || a->HCHAT == nullptr))
        return -3;
    const size_t lds = (size_t)L_END * 2 + NW * 8 * 4 + 512;
    auto k = save ? hyper_persist_fwd<true> : hyper_persist_fwd<false>;
    static bool attr[2] = {false, false};
    if (!attr[save]) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr[save] = true;
    }
    // every workgroup waits on others: all 256 must be resident at once
    static int ok[2] = {-1, -1};
    if (ok[save] < 0) {
        int dev = 0, cus = 0, per = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)k, NTH, lds) != hipSuccess)
            return -8;
        ok[save] = (per >= 1 && cus * per >= NWG) ? 1 : 0;
    }
    if (!ok[save]) return -8;
    const int nz = 4 * 256 + 2 * (2 * MAXB * NX * 8);   // flags (u32) + granules (u64 = 2 words)
    hipLaunchKernelGGL(zero_words, dim3((nz + 255) / 256), dim3(256), 0, s, a->flags, 4 * 256, (uint32_t*)a->part,
                       2 * (2 * MAXB * NX * 8));
    hipLaunchKernelGGL(k, dim3(NWG), dim3(NTH), lds, s, *a);
    return SKR_CHECK_LAUNCH();
}
