// One [M <= 128, BN] output tile of the skinny split-K GEMM and the grouped
// launch's workgroup -> (problem, row block, split, N tile) map, shared by
// csrc/skinny_gemm.hip (plain and grouped launches) and csrc/chain_step.hip
// (grouped launches whose producer tiles publish to waiting cell rows).
#pragma once
#include "common.h"
#include "glds_mma.h"

// One product of a grouped launch: C_s = A[:, Ks] . Bt[:, Ks]^T, S = splits
// fp32 partial slabs (c_slab apart). Mirrored by sketch_rnn_amd/ops/_hipapi.py.
struct GemmProblem {
    const void* A; int64_t lda;
    const void* Bt; int64_t ldb;
    float* C; int64_t ldc; int64_t c_slab;
    int M, N, K, splits;
};

namespace {

typedef __attribute__((ext_vector_type(4))) float tile_f32x4;

constexpr int kMaxGroup = 4;
struct GemmGroup {
    GemmProblem p[kMaxGroup];
    int start[kMaxGroup + 1];
    int n;
};

// (row block, split, N tile) of workgroup `local` of a problem: row blocks of
// 128 rows outermost, then splits, then N tiles
struct TileIdx { int rb, rows, split, nt; };
__device__ __forceinline__ TileIdx tile_idx(int local, int M, int N, int splits, int bn) {
    const int ntiles = N / bn, per_rb = ntiles * splits;
    TileIdx t;
    t.rb = local / per_rb;
    const int rem = local - t.rb * per_rb;
    t.split = rem / ntiles;
    t.nt = rem - t.split * ntiles;
    t.rows = min(skr::BM, M - t.rb * skr::BM);
    return t;
}

__host__ __device__ constexpr int row_blocks_of(int M) { return M <= skr::BM ? 1 : (M + skr::BM - 1) / skr::BM; }

template <typename P>
__device__ __forceinline__ int64_t split_off(const P& p, const TileIdx& t) {
    return (int64_t)t.split * p.c_slab + (int64_t)t.rb * skr::BM * p.ldc;
}

// The tile: glds_mma's accumulators stored to C (fp32, or bf16 with CBF16).
// SC1: write-through (sc1) fp32 stores, for tiles whose slabs a cell row of
// the same launch reads after the arrival counter (csrc/chain_step.hip;
// CDNA4 guide, hand-off table row 1), as relaxed agent-scope atomic stores
// (global_store_dword ... sc1). The value is copied out of the accumulator
// vector first: __builtin_bit_cast of an ext-vector ELEMENT (acc[i][j][e])
// reads element 0 for every e on ROCm 7.2 (measured: rows 1-3 of every
// 4-row accumulator group held row 0's values).
// RA: A in registers, only B through the LDS ring (skr::ra_mma).
template <int BN, int NS, bool CBF16 = false, int NW = 4, bool SC1 = false, bool RA = false>
__device__ __forceinline__ void glds_tile(const __hip_bfloat16* __restrict__ A, int64_t lda,
                                          const __hip_bfloat16* __restrict__ Bt, int64_t ldb,
                                          void* __restrict__ Cv, int64_t ldc, int M, int n0, int64_t k0, int kslice,
                                          __hip_bfloat16* smem) {
    constexpr int NJ = skr::glds_nj<BN, NW>();
    tile_f32x4 acc[2][NJ];
    if constexpr (RA) skr::ra_mma<BN, NS, NW>(A, lda, Bt, ldb, M, n0, k0, kslice, smem, acc);
    else skr::glds_mma<BN, NS, NW>(A, lda, Bt, ldb, M, n0, k0, kslice, smem, acc);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wr = w % 4, c0 = n0 + (w / 4) * NJ * 16;
    const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = 32 * wr + 16 * i + fq * 4 + e;
                if (row < M) {
                    const int64_t o = row * ldc + c0 + 16 * j + fr;
                    if constexpr (CBF16) ((__hip_bfloat16*)Cv)[o] = skr::to_bf16(acc[i][j][e]);
                    else if constexpr (SC1) {   // relaxed agent-scope store = global_store_dword ... sc1
                        const float v = acc[i][j][e];   // (not bit_cast(acc[i][j][e]): see above)
                        __hip_atomic_store((uint32_t*)Cv + o, __builtin_bit_cast(uint32_t, v), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    }
                    else ((float*)Cv)[o] = acc[i][j][e];
                }
            }
}

// Workgroup `id` of a grouped launch: find its problem through the prefix
// sums `start` and run that tile.
template <int BN, int NS, int NW = 4, bool SC1 = false, bool RA = false>
__device__ __forceinline__ void group_tile(const GemmGroup& g, const int id, __hip_bfloat16* smem) {
    int q = 0;
#pragma unroll
    for (int i = 1; i < kMaxGroup; ++i) q += (i < g.n && id >= g.start[i]) ? 1 : 0;
    const GemmProblem& p = g.p[q];
    const TileIdx t = tile_idx(id - g.start[q], p.M, p.N, p.splits, BN);
    const int kslice = p.K / p.splits;
    glds_tile<BN, NS, false, NW, SC1, RA>((const __hip_bfloat16*)p.A + (int64_t)t.rb * skr::BM * p.lda, p.lda,
                                      (const __hip_bfloat16*)p.Bt, p.ldb, p.C + split_off(p, t), p.ldc, t.rows,
                                      t.nt * BN, (int64_t)t.split * kslice, kslice, smem);
}

// Host-side validation of one problem for 64-wide tiles (0: ok). M > 128:
// ceil(M / 128) row blocks, the last one partial (tile_idx: t.rows).
inline int check_problem64(const GemmProblem& p) {
    if (p.M < 1 || p.M > 8 * skr::BM || p.N % 64 != 0 || p.splits < 1 || p.K % p.splits != 0) return -2;
    if ((p.K / p.splits) % skr::BK != 0 || p.lda % 8 != 0 || p.ldb % 8 != 0) return -3;
    if (((uintptr_t)p.A | (uintptr_t)p.Bt) & 15) return -4;
    return 0;
}

}  // namespace
