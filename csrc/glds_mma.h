// Main loop of the skinny bf16 GEMM tiles (csrc/skinny_gemm.hip,
// csrc/hyper_step.hip): one [M <= 128, BN] tile of A . Bt^T over the K range
// [k0, k0 + kslice), accumulated in registers.
//
// LDS-DMA ring. Tiles move global -> LDS with global_load_lds_dwordx4
// (no staging registers, no ds_write), NS buffers deep: NS-1 K-tiles are in
// flight while one is multiplied. One counted `s_waitcnt vmcnt(N)` plus a raw
// s_barrier per K-tile (a __syncthreads() would drain every prefetch, CDNA4
// guide "Pipelining across barriers"). LDS rows are 128 B (BK = 64 bf16) with
// the 16-byte chunk index XOR-swizzled by (row >> 1) & 7 -- applied on the
// per-lane GLOBAL address, since an LDS-DMA wave writes 1 KiB linearly -- so
// the 16 rows of a ds_read_b128 fragment read hit 16 distinct bank quads.
//
// Block: NW x 64 threads. NW = 4: wave w owns rows 32w..32w+31 x all BN
// columns (2 x BN/16 accumulators); NW = 8 (the chained launches of
// csrc/chain_step.hip that share a 512-thread block with the row cells):
// wave w owns rows 32(w%4).. x column half w/4 (2 x BN/32 accumulators).
// MFMA v_mfma_f32_16x16x32_bf16: lane l
// holds A[row l&15][k 8(l>>4) .. +7] and B[k 8(l>>4) .. +7][col l&15];
// C/D: col = l&15, row = 4(l>>4) + i.
//
// (Weight loads use the default cache policy: every weight is re-read each
// time step and stays Infinity-Cache resident; nt loads measured slower,
// 30.3 vs 28.5 ms/step on vae_large, profiles/r2s5/bench_gemm_nt.log.)
#pragma once
#include "common.h"

namespace skr {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;

constexpr int BM = 128, BK = 64;

template <int GPW, int NS>
__device__ __forceinline__ void wait_ahead(int ahead) {
    // tile kt landed (for this wave) once at most `ahead` younger tiles are pending
    if constexpr (NS - 2 >= 4) if (ahead >= 4) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * GPW) : "memory"); return; }
    if constexpr (NS - 2 >= 3) if (ahead == 3) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * GPW) : "memory"); return; }
    if constexpr (NS - 2 >= 2) if (ahead == 2) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GPW) : "memory"); return; }
    if (ahead == 1) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GPW) : "memory"); return; }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// LDS bytes of the ring.
template <int BN, int NS>
constexpr int glds_lds_bytes() { return NS * (BM + BN) * BK * 2; }

// Column tiles (16 wide) of one wave's accumulator.
template <int BN, int NW>
constexpr int glds_nj() { return BN / 16 / (NW / 4); }

template <int BN, int NS, int NW = 4>
__device__ __forceinline__ void glds_mma(const __hip_bfloat16* __restrict__ A, int64_t lda,
                                         const __hip_bfloat16* __restrict__ Bt, int64_t ldb, int M, int n0,
                                         int64_t k0, int kslice, __hip_bfloat16* smem,
                                         f32x4_t (&acc)[2][glds_nj<BN, NW>()]) {
    constexpr int NJ = glds_nj<BN, NW>();
    constexpr int A_CH = BM / 8, B_CH = BN / 8;     // 1-KiB chunks (8 rows) per tile
    static_assert((NW == 4 || NW == 8) && A_CH % NW == 0 && B_CH % NW == 0, "glds_mma: wave layout");
    constexpr int GPW = (A_CH + B_CH) / NW;         // glds per wave per tile
    constexpr int TILE = (BM + BN) * BK;            // bf16 elements per stage
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wr = w % 4, wc = w / 4;               // row quarter, column part (NW = 8)
    const int n = kslice / BK;

    // per-lane source rows / swizzled chunk (fixed across tiles)
    const int r8 = lane >> 3, slot = lane & 7;
    const __hip_bfloat16* asrc[A_CH / NW];
    const __hip_bfloat16* bsrc[B_CH / NW];
#pragma unroll
    for (int i = 0; i < A_CH / NW; ++i) {
        const int row = (w + NW * i) * 8 + r8;
        const int kc = slot ^ ((row >> 1) & 7);
        // rows past M: every lane of the chunk reads the same 16 bytes (one
        // line instead of 1 KiB; the wave's glds count stays uniform)
        asrc[i] = row < M ? A + (int64_t)row * lda + k0 + kc * 8 : A + (int64_t)(M - 1) * lda + k0;
    }
#pragma unroll
    for (int i = 0; i < B_CH / NW; ++i) {
        const int row = (w + NW * i) * 8 + r8;
        const int kc = slot ^ ((row >> 1) & 7);
        bsrc[i] = Bt + (int64_t)(n0 + row) * ldb + k0 + kc * 8;
    }
    auto issue = [&](int kt) {
        __hip_bfloat16* st = smem + (kt % NS) * TILE;
        const int64_t ko = (int64_t)kt * BK;
#pragma unroll
        for (int i = 0; i < A_CH / NW; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + ko),
                                             (__attribute__((address_space(3))) void*)(st + (w + NW * i) * 512), 16, 0, 0);
#pragma unroll
        for (int i = 0; i < B_CH / NW; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + ko),
                                             (__attribute__((address_space(3))) void*)(st + BM * BK + (w + NW * i) * 512),
                                             16, 0, 0);
    };

#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
    for (int p = 0; p < NS - 1; ++p)
        if (p < n) issue(p);
    for (int kt = 0; kt < n; ++kt) {
        wait_ahead<GPW, NS>(min(n - 1 - kt, NS - 2));
        __builtin_amdgcn_s_barrier();  // ... and for every wave; buffer (kt-1) % NS is free
        if (kt + NS - 1 < n) issue(kt + NS - 1);
        const __hip_bfloat16* As = smem + (kt % NS) * TILE;
        const __hip_bfloat16* Bs = As + BM * BK;
#pragma unroll
        for (int ks = 0; ks < BK; ks += 32) {
            const int kc = ks / 8 + fq;
            bf16x8_t af[2], bfr[NJ];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int row = 32 * wr + 16 * i + fr;
                af[i] = *(const bf16x8_t*)(&As[row * BK + ((kc ^ ((row >> 1) & 7)) * 8)]);
            }
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int row = 16 * (wc * NJ + j) + fr;
                bfr[j] = *(const bf16x8_t*)(&Bs[row * BK + ((kc ^ ((row >> 1) & 7)) * 8)]);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
    }
}

// A-in-registers variant (RA): each wave reads ITS OWN rows of A (rows
// 32 (w % 4) .. + 31; no other wave needs them) straight into MFMA fragment
// registers with 16-byte global loads -- A[row][k 8 fq .. +7] is the
// fragment, contiguous in memory -- NS - 1 stages ahead in an NS-deep
// register ring; only B (shared by the waves) goes through the LDS-DMA ring
// (BN x BK per stage: 8 KiB at BN = 64). Same fragments, same k order per
// output element as glds_mma: bit-identical accumulators. Measured SLOWER
// (ops.gemm.SKINNY_RA; profiles/r6/skinny_ra_ab.log: vae_large 25.47 / 25.47
// ms/step at depth 3, 25.59 at 6, against 24.00 / 23.99): the LDS-DMA ring
// is not the bottleneck of these tiles -- it streams 84 GB/s per CU from an
// L2- or Infinity-Cache-resident footprint (scripts/micro/l2_rate.hip,
// profiles/r6/l2_rate.jsonl) -- and the register loads put their latency
// in front of every stage's MFMAs.
template <int BN, int NS, int NW = 4>
__device__ __forceinline__ void ra_mma(const __hip_bfloat16* __restrict__ A, int64_t lda,
                                       const __hip_bfloat16* __restrict__ Bt, int64_t ldb, int M, int n0,
                                       int64_t k0, int kslice, __hip_bfloat16* smem,
                                       f32x4_t (&acc)[2][glds_nj<BN, NW>()]) {
    constexpr int NJ = glds_nj<BN, NW>();
    constexpr int B_CH = BN / 8;                    // 1-KiB chunks (8 rows) of B per stage
    static_assert((NW == 4 || NW == 8) && B_CH % NW == 0, "ra_mma: wave layout");
    constexpr int GPWB = B_CH / NW;
    constexpr int GPW = GPWB + 4;                   // VMEM instructions per wave per stage (4 A fragment loads)
    constexpr int TILE = BN * BK;                   // bf16 elements per LDS stage (B only)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wr = w % 4, wc = w / 4;
    const int n = kslice / BK;
    const int fr = lane & 15, fq = lane >> 4;
    const int r8 = lane >> 3, slot = lane & 7;
    const __hip_bfloat16* bsrc[GPWB];
#pragma unroll
    for (int i = 0; i < GPWB; ++i) {
        const int row = (w + NW * i) * 8 + r8;
        const int kc = slot ^ ((row >> 1) & 7);
        bsrc[i] = Bt + (int64_t)(n0 + row) * ldb + k0 + kc * 8;
    }
    const __hip_bfloat16* arow[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) arow[i] = A + (int64_t)min(32 * wr + 16 * i + fr, M - 1) * lda + k0 + 8 * fq;
    bf16x8_t ar[NS][2][2];                          // [register stage][row tile][k32 half]
    auto issue = [&](int kt, bf16x8_t (&dst)[2][2]) {
        const int64_t ko = (int64_t)kt * BK;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int h = 0; h < 2; ++h) dst[i][h] = *(const bf16x8_t*)(arow[i] + ko + 32 * h);
        __hip_bfloat16* st = smem + (kt % NS) * TILE;
#pragma unroll
        for (int i = 0; i < GPWB; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + ko),
                                             (__attribute__((address_space(3))) void*)(st + (w + NW * i) * 512), 16, 0, 0);
    };
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int p = 0; p < NS - 1; ++p)
        if (p < n) issue(p, ar[p]);
    for (int kb = 0; kb < n; kb += NS) {
#pragma unroll
        for (int u = 0; u < NS; ++u) {              // stage kt = kb + u: register set u, LDS buffer u
            const int kt = kb + u;
            if (kt >= n) break;
            wait_ahead<GPW, NS>(min(n - 1 - kt, NS - 2));
            __builtin_amdgcn_s_barrier();           // B of stage kt landed for every wave; buffer (kt-1) % NS is free
            if (kt + NS - 1 < n) issue(kt + NS - 1, ar[(u + NS - 1) % NS]);
            const __hip_bfloat16* Bs = smem + u * TILE;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int kc = 4 * h + fq;
                bf16x8_t bfr[NJ];
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    const int row = 16 * (wc * NJ + j) + fr;
                    bfr[j] = *(const bf16x8_t*)(&Bs[row * BK + ((kc ^ ((row >> 1) & 7)) * 8)]);
                }
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < NJ; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ar[u][i][h], bfr[j], acc[i][j], 0, 0, 0);
            }
        }
    }
}

}  // namespace skr
