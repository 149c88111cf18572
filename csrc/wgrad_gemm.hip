// Long-K weight-gradient GEMM: C = A^T . B over the T*B saved rows of a
// sequence (reference: /root/reference/model.py:182, tf.gradients over every
// Linear of the unrolled RNN).
//
//   A [K, M] bf16 (row stride lda)    B [K, N] bf16 (row stride ldb)
//   C [M, N] fp32 = sum_k A[k, :]^T B[k, :]        (+ optional colsum(B) [N])
//
// K = T*B = 25,000 rows for the headline decoder; M, N are weight dims
// (2048 x 8192, 256 x 24576, 2304 x 1024, 512 x 2048 per direction).
//
// Both operands arrive with K as the ROW index, so an MFMA fragment (8
// consecutive k of one output row/column) is a COLUMN of the staged tile.
// gfx950's ds_read_b64_tr_b16 delivers exactly that: per 16-lane group it
// reads a 4-row x 16-column block and hands lane i column i -- two reads
// make a v_mfma_f32_32x32x16_bf16 operand (lane l: k = 8 (l >> 5) .. +7 of
// row/column l & 31). No register transposes, no second LDS image.
//
// Tiling (one workgroup per CU, 512 threads = 8 waves):
//   * output tile 256 x 256, wave (wm, wn) = 4 x 2 owns 64 x 128 = 2 x 4
//     MFMA 32x32 tiles (128 fp32 accumulators per lane);
//   * K-step 32 rows: 16 KB of A + 16 KB of B per step, 4.2 MFLOP -- the
//     256 x 256 tile is what keeps the per-CU ingest (~75 GB/s at the MFMA
//     peak) inside what L2 feeds one CU;
//   * LDS-DMA ring (global_load_lds_dwordx4, 1 KiB per wave instruction = 2
//     tile rows), 4 stages x 32 KB, one counted vmcnt wait + one s_barrier per
//     K-step (the skinny GEMM's ring, csrc/skinny_gemm.hip);
//   * LDS rows of 512 B with the 16-byte chunk index XOR (row & 3) << 2
//     (applied on the per-lane GLOBAL address, since a DMA wave writes 1 KiB
//     linearly): the 32 lanes of a transposed read's half touch 4 rows x 4
//     chunks, which the XOR spreads over all 64 banks -- conflict-free;
//   * split-K over gridDim (S slabs of fp32 partials, summed by a second
//     deterministic pass) only when the output has too few tiles to fill the
//     chip; tile order is XCD-aware: workgroup id % 8 picks the XCD, and
//     consecutive tiles of one XCD form 4-row groups, so the A and B tiles a
//     K-step needs are shared in that XCD's L2;
//   * the K tail (K % 32 rows): clamped loads, then the invalid rows of the
//     last stage are zeroed in LDS before use.
// Measured (scripts/bench_wgrad.py, profiles/r3/wgrad_bench.jsonl): 804 /
// 471 / 143 / 130 us for the dW_h / dP+colsum / dW_y / encoder shapes
// against hipBLASLt's 837 / 700 / 174 / 168. A variant with fragments
// double-buffered across K-steps and a 5-stage ring was slower on dW_h (940).
// Round 5 (profiles/r5/wgrad_sweep.jsonl, one box): both k16 halves'
// fragment reads issued up front (DB) -- the second half's 12 transposed
// reads land under the first half's MFMAs -- dW_h 880 -> 785 us; dP + colsum
// at 5 splits (ops/gemm.py _wgrad_splits) 514 -> 438 us.
// Optional colsum(B) (the bias gradient folded into a projection's weight
// gradient: HyperLSTM dVEC): waves wm == 0 add their B fragments in fp32.
#include "common.h"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int TM = 256, TN = 256, BK = 32, NT = 512, NSTG = 4;
constexpr int ROWB = 512;                 // bytes per LDS tile row (256 bf16)
constexpr int OPB = BK * ROWB;            // 16 KB per operand per stage
constexpr int STGB = 2 * OPB;             // 32 KB per stage
constexpr int GPW = 4;                    // DMA instructions per wave per K-step

struct WgArgs {
    const __hip_bfloat16* A; int64_t lda, a_bs;
    const __hip_bfloat16* B; int64_t ldb, b_bs;
    float* C; int64_t c_bs;               // slab s of batch z at C + z * c_bs + s * M * N
    float* cs;                            // colsum slabs [batch][S][N] or null
    int64_t K; int M, N, S, kslice, tiles_m, tiles_n, total, per_xcd;
    int stride;                           // workgroups per XCD slot: tile j, j + stride, ... of one XCD's list
    int acc;                              // 1: C (and cs) += the product instead of =
};

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row & 3) << 2); }

template <int AHEAD_MAX>
__device__ __forceinline__ void wait_ahead(int ahead) {
    if constexpr (AHEAD_MAX >= 2) if (ahead >= 2) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GPW) : "memory"); return; }
    if (ahead == 1) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GPW) : "memory"); return; }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ds_read_b64_tr_b16 through inline asm: the compiler models the builtin's
// LDS read as aliasing every in-flight LDS-DMA write and drains the whole
// prefetch ring (s_waitcnt vmcnt(0)) in front of it. The asm read is opaque
// to the waitcnt pass, so the kernel waits for it explicitly (frag_wait) --
// tied to the destination registers, so no use can be scheduled above it.
__device__ __forceinline__ s16x4 tr_read(uint32_t addr) {
    s16x4 v;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(addr));
    return v;
}

struct Frags {
    s16x4 a[2][2], b[4][2];   // [tile][k half]: two transposed reads per MFMA operand
};

// wait until at most N LDS reads are outstanding (the younger fragment set's)
template <int N>
__device__ __forceinline__ void frag_wait(Frags& f) {
    asm volatile("s_waitcnt lgkmcnt(%12)"
                 : "+v"(f.a[0][0]), "+v"(f.a[0][1]), "+v"(f.a[1][0]), "+v"(f.a[1][1]), "+v"(f.b[0][0]),
                   "+v"(f.b[0][1]), "+v"(f.b[1][0]), "+v"(f.b[1][1]), "+v"(f.b[2][0]), "+v"(f.b[2][1]),
                   "+v"(f.b[3][0]), "+v"(f.b[3][1])
                 : "n"(N));
}

__device__ __forceinline__ bf16x8 join(const s16x4 (&h)[2]) {
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 v = {h[0][0], h[0][1], h[0][2], h[0][3], h[1][0], h[1][1], h[1][2], h[1][3]};
    return __builtin_bit_cast(bf16x8, v);
}

// DB: both k16 halves' fragment sets read up front, the second half's
// reads in flight under the first half's MFMAs (24 transposed reads per
// K-step in one batch instead of two exposed read -> wait -> MFMA rounds).
// BG: the bounded-grid form (several tiles per workgroup); otherwise one tile.
template <bool CS, bool DB, bool BG>
__global__ __launch_bounds__(NT) void wgrad_kernel(const WgArgs g) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // ---- workgroup -> (batch, split, tile): XCD-major linear order; a grid
    // smaller than the tile count (background launches) walks its XCD's list
    // with stride g.stride
    const int xcd = blockIdx.x & 7;
    for (int jx = blockIdx.x >> 3; jx < g.per_xcd; jx += g.stride) {
        const int lin = xcd * g.per_xcd + jx;
        if (lin >= g.total) return;                       // whole workgroup, before any barrier
        const int tiles = g.tiles_m * g.tiles_n;
        const int t = lin % tiles, zs = lin / tiles;      // zs = batch * S + split
        const int split = zs % g.S, z = zs / g.S;
        const int gsz = 4 * g.tiles_n, grp = t / gsz, fm = grp * 4;
        const int gm = min(g.tiles_m - fm, 4);
        const int tm = fm + (t % gsz) % gm, tn = (t % gsz) / gm;
        const int m0 = tm * TM, n0 = tn * TN;
        const int64_t k0 = (int64_t)split * g.kslice;
        const int64_t kend = min(g.K, k0 + g.kslice);
        const int nk = (int)((kend - k0 + BK - 1) / BK);
        const int tail = (int)(kend - k0) - (nk - 1) * BK;     // valid rows of the last K-step (1..32)
        const __hip_bfloat16* A = g.A + z * g.a_bs;
        const __hip_bfloat16* B = g.B + z * g.b_bs;

        const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
        // ---- DMA sources: wave w moves tile rows {2w, 2w+1} and {2w+16, 2w+17} of A and of B
        const int hr = lane >> 5, lc = lane & 31;
        const __hip_bfloat16* asrc[2];
        const __hip_bfloat16* bsrc[2];
        int rowk[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int R = 2 * w + 16 * i + hr;
            rowk[i] = R;
            const int c = swz(R, lc);
            asrc[i] = A + m0 + 8 * c;
            bsrc[i] = B + n0 + 8 * c;
        }
        auto issue = [&](int kt) {
            char* st = smem + (kt % NSTG) * STGB;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int64_t kr = min(k0 + (int64_t)kt * BK + rowk[i], kend - 1);   // clamped: finite data
                __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + kr * g.lda),
                                                 (__attribute__((address_space(3))) void*)(st + (2 * w + 16 * i) * ROWB),
                                                 16, 0, 0);
                __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + kr * g.ldb),
                                                 (__attribute__((address_space(3))) void*)(st + OPB + (2 * w + 16 * i) * ROWB),
                                                 16, 0, 0);
            }
        };

        // ---- fragment read offsets (bytes inside an operand tile), fixed across K-steps
        const int wm = w >> 1, wn = w & 1;
        const int G = lane >> 4, h = G >> 1, q = (lane >> 2) & 3, p = lane & 3;
        int aoff[2][2][2], boff[4][2][2];     // [tile][k16 half][read]
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int rd = 0; rd < 2; ++rd) {
                const int row = 16 * ks + 8 * h + 4 * rd + q;
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int col = 64 * wm + 32 * i + 16 * (G & 1) + 4 * p;
                    aoff[i][ks][rd] = row * ROWB + (swz(row, col >> 3) << 4) + 8 * (p & 1);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int col = 128 * wn + 32 * j + 16 * (G & 1) + 4 * p;
                    boff[j][ks][rd] = row * ROWB + (swz(row, col >> 3) << 4) + 8 * (p & 1);
                }
            }

        f32x16 acc[2][4];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
        float cs[4] = {0.f, 0.f, 0.f, 0.f};

        auto zero_tail = [&](char* st) {
            // rows past kend hold clamped (duplicate) data: zero them in both operands
            const int per = (BK - tail) * ROWB / 16;              // 16-byte pieces per operand
            for (int i = tid; i < 2 * per; i += NT) {
                const int op = i / per, r = i - op * per;
                *(int4*)(st + op * OPB + tail * ROWB + 16 * r) = int4{0, 0, 0, 0};
            }
            skr::lds_barrier();
        };
        const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
        // 12 transposed reads per fragment set (2 A tiles + 4 B tiles, 2 reads each)
        auto read_frags = [&](int stage, int ks, Frags& f) {
            const uint32_t st = lds0 + stage * STGB;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int rd = 0; rd < 2; ++rd) f.a[i][rd] = tr_read(st + aoff[i][ks][rd]);
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int rd = 0; rd < 2; ++rd) f.b[j][rd] = tr_read(st + OPB + boff[j][ks][rd]);
        };
        auto mfmas = [&](const Frags& f) {
            bf16x8 af[2], bfr[4];
#pragma unroll
            for (int i = 0; i < 2; ++i) af[i] = join(f.a[i]);
#pragma unroll
            for (int j = 0; j < 4; ++j) bfr[j] = join(f.b[j]);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
            if constexpr (CS) {
                if (wm == 0 && tm == 0) {   // (one tile row sums each column: several would race under acc)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
#pragma unroll
                        for (int e = 0; e < 8; ++e) cs[j] += (float)bfr[j][e];
                }
            }
        };

#pragma unroll
        for (int s = 0; s < NSTG - 1; ++s)
            if (s < nk) issue(s);
        for (int kt = 0; kt < nk; ++kt) {
            wait_ahead<NSTG - 2>(min(nk - 1 - kt, NSTG - 2));
            __builtin_amdgcn_s_barrier();     // stage kt landed for every wave; stage kt-1 is free
            if (kt + NSTG - 1 < nk) issue(kt + NSTG - 1);
            if (kt == nk - 1 && tail < BK) zero_tail(smem + (kt % NSTG) * STGB);
            if constexpr (DB) {
                Frags f0, f1;
                read_frags(kt % NSTG, 0, f0);
                read_frags(kt % NSTG, 1, f1);
                frag_wait<12>(f0);
                mfmas(f0);
                frag_wait<0>(f1);
                mfmas(f1);
            } else {
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    Frags f;
                    read_frags(kt % NSTG, ks, f);
                    frag_wait<0>(f);
                    mfmas(f);
                }
            }
        }
        // ---- epilogue: fp32 slab (lane: column r; registers: rows (e&3) + 8(e>>2) + 4h)
        float* C = g.C + z * g.c_bs + (int64_t)split * g.M * g.N;
        const int r = lane & 31;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int col = n0 + 128 * wn + 32 * j + r;
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int row = m0 + 64 * wm + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h;
                    float* c = C + (int64_t)row * g.N + col;
                    *c = g.acc ? *c + acc[i][j][e] : acc[i][j][e];
                }
            }
        if constexpr (CS) {
            if (wm == 0 && tm == 0) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float v = cs[j] + __shfl_xor(cs[j], 32, 64);
                    float* c = g.cs + (int64_t)zs * g.N + n0 + 128 * wn + 32 * j + r;
                    if (lane < 32) *c = g.acc ? *c + v : v;
                }
            }
        }
        if constexpr (!BG) break;
        __syncthreads();   // every wave's LDS reads of this tile are done before the next tile's DMA
    }
}

// ---- one wave per SIMD: 4 waves, each 128 x 128 of the 256 x 256 tile ------------------
// Variant 2 (skr_wgrad_set_variant): bit-identical to the 8-wave kernel and
// measured SLOWER on every shape of the step (profiles/r6/wgrad_variant_ab.jsonl:
// dW_h 836-869 vs 776-898 us, dP + colsum 452-456 vs 425-437, dW_y 138-140 vs
// 131, encoder 126-128 vs 116-117; step 23.97 / 23.99 vs 23.91 / 23.85 ms):
// a second wave per SIMD covers the LDS-read and barrier latencies better
// than the cross-K-step fragment pipeline of one wave does.
// (4 x 4 MFMA 32x32 tiles: 256 accumulators per lane; up to 512 registers per
// lane at one wave per SIMD). Fragments are software-pipelined across the
// K-step: half 1's transposed reads are in flight under half 0's MFMAs, and
// the NEXT K-step's half-0 reads under half 1's -- the ring's barrier sits
// between the two halves, so the MFMA pipe never waits on a barrier + first
// LDS read. Same staging (4-stage LDS-DMA ring, XOR-swizzled 512-byte rows),
// same fragment layout and k order per output element as wgrad_kernel.
constexpr int NT4 = 256, GPW4 = 8;

struct Frags4 {
    s16x4 a[4][2], b[4][2];   // [tile][read]: one k16 half
};

template <int N>
__device__ __forceinline__ void frag_wait4(Frags4& f) {
    asm volatile("s_waitcnt lgkmcnt(%16)"
                 : "+v"(f.a[0][0]), "+v"(f.a[0][1]), "+v"(f.a[1][0]), "+v"(f.a[1][1]), "+v"(f.a[2][0]),
                   "+v"(f.a[2][1]), "+v"(f.a[3][0]), "+v"(f.a[3][1]), "+v"(f.b[0][0]), "+v"(f.b[0][1]),
                   "+v"(f.b[1][0]), "+v"(f.b[1][1]), "+v"(f.b[2][0]), "+v"(f.b[2][1]), "+v"(f.b[3][0]),
                   "+v"(f.b[3][1])
                 : "n"(N));
}

// transposed read at base + a compile-time byte offset (the instruction's
// offset field: no address register per (k half, read) pair)
template <int OFF>
__device__ __forceinline__ s16x4 tr_read_at(uint32_t addr) {
    s16x4 v;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF));
    return v;
}

// the 8 reads of one operand for k16 half KS: tile i at base[i]; read rd at
// +4 rows (row = 16 KS + 8 h + 4 rd + q: the XOR swizzle depends on q only)
template <int KS>
__device__ __forceinline__ void read_op4(const uint32_t (&base)[4], s16x4 (&f)[4][2]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        f[i][0] = tr_read_at<KS * 16 * ROWB>(base[i]);
        f[i][1] = tr_read_at<KS * 16 * ROWB + 4 * ROWB>(base[i]);
    }
}

template <bool CS, bool BG>
__global__ __launch_bounds__(NT4) __attribute__((amdgpu_waves_per_eu(1, 1))) void wgrad_kernel4(const WgArgs g) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int xcd = blockIdx.x & 7;
    for (int jx = blockIdx.x >> 3; jx < g.per_xcd; jx += g.stride) {
        const int lin = xcd * g.per_xcd + jx;
        if (lin >= g.total) return;
        const int tiles = g.tiles_m * g.tiles_n;
        const int t = lin % tiles, zs = lin / tiles;
        const int split = zs % g.S, z = zs / g.S;
        const int gsz = 4 * g.tiles_n, grp = t / gsz, fm = grp * 4;
        const int gm = min(g.tiles_m - fm, 4);
        const int tm = fm + (t % gsz) % gm, tn = (t % gsz) / gm;
        const int m0 = tm * TM, n0 = tn * TN;
        const int64_t k0 = (int64_t)split * g.kslice;
        const int64_t kend = min(g.K, k0 + g.kslice);
        const int nk = (int)((kend - k0 + BK - 1) / BK);
        const int tail = (int)(kend - k0) - (nk - 1) * BK;
        const __hip_bfloat16* A = g.A + z * g.a_bs;
        const __hip_bfloat16* B = g.B + z * g.b_bs;

        const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
        // ---- DMA sources: wave w moves tile rows {2w + 8i, 2w + 8i + 1}, i < 4, of A and of B
        const int hr = lane >> 5, lc = lane & 31;
        const __hip_bfloat16* asrc[4];
        const __hip_bfloat16* bsrc[4];
        int rowk[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int R = 2 * w + 8 * i + hr;
            rowk[i] = R;
            const int c = swz(R, lc);
            asrc[i] = A + m0 + 8 * c;
            bsrc[i] = B + n0 + 8 * c;
        }
        auto issue = [&](int kt) {
            char* st = smem + (kt % NSTG) * STGB;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t kr = min(k0 + (int64_t)kt * BK + rowk[i], kend - 1);
                __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + kr * g.lda),
                                                 (__attribute__((address_space(3))) void*)(st + (2 * w + 8 * i) * ROWB),
                                                 16, 0, 0);
                __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + kr * g.ldb),
                                                 (__attribute__((address_space(3))) void*)(st + OPB + (2 * w + 8 * i) * ROWB),
                                                 16, 0, 0);
            }
        };
        // ---- fragment read offsets: wave (wm, wn) owns rows 128 wm.., columns
        // 128 wn..; per tile the (k half, read) pairs differ by whole rows (the
        // swizzle depends on row & 3 = q only), folded into the offset field
        const int wm = w >> 1, wn = w & 1;
        const int G = lane >> 4, h = G >> 1, q = (lane >> 2) & 3, p = lane & 3;
        int aoff[4], boff[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = 8 * h + q;
            const int ca = 128 * wm + 32 * i + 16 * (G & 1) + 4 * p;
            aoff[i] = row * ROWB + (swz(row, ca >> 3) << 4) + 8 * (p & 1);
            const int cb = 128 * wn + 32 * i + 16 * (G & 1) + 4 * p;
            boff[i] = OPB + row * ROWB + (swz(row, cb >> 3) << 4) + 8 * (p & 1);
        }
        f32x16 acc[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
        float cs[4] = {0.f, 0.f, 0.f, 0.f};
        const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
        // a half's 16 transposed reads in two groups of 8 (A, then B): the wait
        // for the previous set is issued between them, so no wait ever needs a
        // count above lgkmcnt's 4-bit field
        auto bases = [&](int kt, uint32_t (&ba)[4], uint32_t (&bb)[4]) {
            const uint32_t st = lds0 + (kt % NSTG) * STGB;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                ba[i] = st + aoff[i];
                bb[i] = st + boff[i];
            }
        };
        auto mfmas = [&](const Frags4& f) {
            bf16x8 af[4], bfr[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                af[i] = join(f.a[i]);
                bfr[i] = join(f.b[i]);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
            if constexpr (CS) {
                if (wm == 0 && tm == 0) {   // (one tile row sums each column: several would race under acc)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
#pragma unroll
                        for (int e = 0; e < 8; ++e) cs[j] += (float)bfr[j][e];
                }
            }
        };
        auto zero_tail = [&](char* st) {
            const int per = (BK - tail) * ROWB / 16;
            for (int i = tid; i < 2 * per; i += NT4) {
                const int op = i / per, r = i - op * per;
                *(int4*)(st + op * OPB + tail * ROWB + 16 * r) = int4{0, 0, 0, 0};
            }
        };
        auto wait_stage = [&](int ahead) {   // this wave's DMAs of the stage `ahead` steps before the newest landed
            if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GPW4) : "memory");
            else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GPW4) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        };
        // ---- prologue: stages 0 .. NSTG-2 in flight; stage 0 visible; its half 0 read
#pragma unroll
        for (int s = 0; s < NSTG - 1; ++s)
            if (s < nk) issue(s);
        wait_stage(min(nk - 1, NSTG - 2));   // stage 0 landed (stages 1, 2 may fly)
        __builtin_amdgcn_s_barrier();
        if (nk == 1 && tail < BK) {
            zero_tail(smem);
            skr::lds_barrier();
        }
        Frags4 f0, f1;
        uint32_t ba[4], bb[4];
        bases(0, ba, bb);
        read_op4<0>(ba, f0.a);
        read_op4<0>(bb, f0.b);
        for (int kt = 0; kt < nk; ++kt) {
            // stage kt is visible (barrier passed); f0 = its half 0 (in flight)
            read_op4<1>(ba, f1.a);
            frag_wait4<8>(f0);            // (LDS reads complete in order: f0 is older than these 8)
            read_op4<1>(bb, f1.b);
            mfmas(f0);
            // stage kt + 1: this wave's DMAs landed (stage kt + 2, if issued, may
            // still fly), then every wave's; every wave is past its reads of
            // stage kt - 1, whose buffer the next DMA refills
            if (kt + 1 < nk) {
                wait_stage(min(nk - 2 - kt, 1));
                __builtin_amdgcn_s_barrier();
                if (kt + NSTG - 1 < nk) issue(kt + NSTG - 1);
                if (kt + 1 == nk - 1 && tail < BK) {   // the last stage's rows past kend: zeroed before any read
                    zero_tail(smem + ((kt + 1) % NSTG) * STGB);
                    skr::lds_barrier();
                }
                bases(kt + 1, ba, bb);
                read_op4<0>(ba, f0.a);
                frag_wait4<8>(f1);
                read_op4<0>(bb, f0.b);
            } else {
                frag_wait4<0>(f1);
            }
            mfmas(f1);
        }
        // ---- epilogue (lane: column r; registers: rows (e&3) + 8(e>>2) + 4h)
        float* C = g.C + z * g.c_bs + (int64_t)split * g.M * g.N;
        const int r = lane & 31;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int col = n0 + 128 * wn + 32 * j + r;
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int row = m0 + 128 * wm + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h;
                    float* c = C + (int64_t)row * g.N + col;
                    *c = g.acc ? *c + acc[i][j][e] : acc[i][j][e];
                }
            }
        if constexpr (CS) {
            if (wm == 0 && tm == 0) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float v = cs[j] + __shfl_xor(cs[j], 32, 64);
                    float* c = g.cs + (int64_t)zs * g.N + n0 + 128 * wn + 32 * j + r;
                    if (lane < 32) *c = g.acc ? *c + v : v;
                }
            }
        }
        if constexpr (!BG) break;
        __syncthreads();
    }
}

// out[z][i] = sum_s slab[z][s][i] (i < n, n % 4 == 0), fixed order: deterministic
__global__ __launch_bounds__(256) void slab_sum_kernel(const float* __restrict__ src, int S, int64_t n, int nb,
                                                       float* __restrict__ out, int acc) {
    const int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (i4 >= n * nb) return;
    const int64_t z = i4 / n, i = i4 - z * n;
    const float* p = src + z * S * n + i;
    float4 a = *(const float4*)p;
    for (int s = 1; s < S; ++s) {
        const float4 b = *(const float4*)(p + s * n);
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    if (acc) {   // added to the destination last: the chunked (background) order of ops/gemm.py
        const float4 o = *(const float4*)(out + i4);
        a.x = o.x + a.x; a.y = o.y + a.y; a.z = o.z + a.z; a.w = o.w + a.w;
    }
    *(float4*)(out + i4) = a;
}

}  // namespace

static int g_wgrad_db = 1;   // fragment schedule (DB template argument), skr_wgrad_set_variant

// A/B hook: 1 = both k16 halves' fragments read up front (DB), 0 = per-half,
// 2 = the one-wave-per-SIMD kernel (wgrad_kernel4); < 0 = leave unchanged.
// Returns the schedule in force before the call.
SKR_API int skr_wgrad_set_variant(int db) {
    const int prev = g_wgrad_db;
    if (db >= 0) g_wgrad_db = db > 2 ? 1 : db;
    return prev;
}

// C[z] (+)= A[z]^T . B[z] (+ cs[z] (+)= colsum(B[z]) when cs != null) for z < nb.
// A [K, M] bf16 (lda, batch stride a_bs elements), B [K, N] bf16 (ldb, b_bs).
// S split-K slabs: slab s of batch z at work + (z * S + s) * M * N (fp32);
// with S == 1 the kernel writes C directly (work unused). cs_work [nb][S][N].
// Requirements: M % 256 == 0, N % 256 == 0, lda, ldb % 8 == 0, 16-byte
// aligned bases (returns -2 / -4 otherwise: callers use a library GEMM).
// acc: add into C / cs instead of overwriting them. max_grid > 0 (a multiple
// of 8): at most that many workgroups, each walking several tiles -- the
// background launches of ops/gemm.py that run beside the HyperLSTM backward
// scan on a second stream and must leave most CUs to it.
SKR_API int skr_wgrad2(const void* A, int64_t lda, int64_t a_bs, const void* B, int64_t ldb, int64_t b_bs,
                       int64_t K, int M, int N, int nb, int S, float* C, float* work, float* cs, float* cs_work,
                       int acc, int max_grid, hipStream_t s) {
    if (K <= 0 || M <= 0 || N <= 0 || nb <= 0 || max_grid < 0 || max_grid % 8) return -2;
    if (M % TM || N % TN || lda % 8 || ldb % 8 || a_bs % 8 || b_bs % 8 || S < 1) return -2;
    if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) & 15) return -4;
    if (S > 1 && work == nullptr) return -3;
    if (cs != nullptr && S > 1 && cs_work == nullptr) return -3;
    WgArgs g;
    g.A = (const __hip_bfloat16*)A; g.lda = lda; g.a_bs = a_bs;
    g.B = (const __hip_bfloat16*)B; g.ldb = ldb; g.b_bs = b_bs;
    g.C = S > 1 ? work : C;
    g.c_bs = (int64_t)S * M * N;
    g.cs = cs == nullptr ? nullptr : (S > 1 ? cs_work : cs);
    g.K = K; g.M = M; g.N = N; g.S = S;
    g.kslice = (int)(((K + S - 1) / S + BK - 1) / BK * BK);
    if ((int64_t)g.kslice * (S - 1) >= K) return -5;   // an empty split
    g.tiles_m = M / TM; g.tiles_n = N / TN;
    g.total = nb * S * g.tiles_m * g.tiles_n;
    g.per_xcd = (g.total + 7) / 8;
    g.stride = max_grid > 0 ? min(g.per_xcd, max_grid / 8) : g.per_xcd;
    g.acc = (acc != 0 && S == 1) ? 1 : 0;   // with split-K slabs the sum pass adds instead
    const int grid = 8 * g.stride;
    const size_t lds = (size_t)NSTG * STGB;
    static bool attr = false;
    if (!attr) {
        const void* ks[8] = {(const void*)wgrad_kernel<false, false, false>, (const void*)wgrad_kernel<true, false, false>,
                             (const void*)wgrad_kernel<false, true, false>, (const void*)wgrad_kernel<true, true, false>,
                             (const void*)wgrad_kernel<false, false, true>, (const void*)wgrad_kernel<true, false, true>,
                             (const void*)wgrad_kernel<false, true, true>, (const void*)wgrad_kernel<true, true, true>};
        for (const void* k : ks)
            if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return -6;
        const void* k4[4] = {(const void*)wgrad_kernel4<false, false>, (const void*)wgrad_kernel4<true, false>,
                             (const void*)wgrad_kernel4<false, true>, (const void*)wgrad_kernel4<true, true>};
        for (const void* k : k4)
            if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return -6;
        attr = true;
    }
    const bool cs_on = g.cs != nullptr, bg = g.stride < g.per_xcd;
    const dim3 gd(grid), bd(NT);
#define SKR_WG_LAUNCH(CS_, DB_)                                                                   \
    do {                                                                                          \
        if (bg) hipLaunchKernelGGL((wgrad_kernel<CS_, DB_, true>), gd, bd, lds, s, g);            \
        else hipLaunchKernelGGL((wgrad_kernel<CS_, DB_, false>), gd, bd, lds, s, g);              \
    } while (0)
    if (g_wgrad_db == 2) {   // one wave per SIMD, fragments pipelined across the K-step
        const dim3 bd4(NT4);
        if (bg) {
            if (cs_on) hipLaunchKernelGGL((wgrad_kernel4<true, true>), gd, bd4, lds, s, g);
            else hipLaunchKernelGGL((wgrad_kernel4<false, true>), gd, bd4, lds, s, g);
        } else {
            if (cs_on) hipLaunchKernelGGL((wgrad_kernel4<true, false>), gd, bd4, lds, s, g);
            else hipLaunchKernelGGL((wgrad_kernel4<false, false>), gd, bd4, lds, s, g);
        }
    } else if (g_wgrad_db) {
        if (cs_on) SKR_WG_LAUNCH(true, true);
        else SKR_WG_LAUNCH(false, true);
    } else {
        if (cs_on) SKR_WG_LAUNCH(true, false);
        else SKR_WG_LAUNCH(false, false);
    }
#undef SKR_WG_LAUNCH
    if (S > 1) {
        const int64_t n = (int64_t)M * N;
        hipLaunchKernelGGL(slab_sum_kernel, dim3((unsigned)((n * nb / 4 + 255) / 256)), dim3(256), 0, s, work, S, n, nb, C,
                           acc);
        if (cs != nullptr)
            hipLaunchKernelGGL(slab_sum_kernel, dim3((unsigned)((N * nb / 4 + 255) / 256)), dim3(256), 0, s, cs_work, S,
                               (int64_t)N, nb, cs, acc);
    }
    return SKR_CHECK_LAUNCH();
}

SKR_API int skr_wgrad(const void* A, int64_t lda, int64_t a_bs, const void* B, int64_t ldb, int64_t b_bs,
                      int64_t K, int M, int N, int nb, int S, float* C, float* work, float* cs, float* cs_work,
                      hipStream_t s) {
    return skr_wgrad2(A, lda, a_bs, B, ldb, b_bs, K, M, N, nb, S, C, work, cs, cs_work, 0, 0, s);
}
