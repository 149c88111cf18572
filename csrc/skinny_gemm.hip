// Skinny split-K GEMM for the recurrent steps: C_s = A[:, Ks] . Bt[:, Ks]^T
//
// Every per-time-step product in the RNN is "few rows, long K or wide N":
// M = batch (<= 128), N in {256 .. 24576}, K in {256 .. 24576}. Library
// kernels tile these for square problems and leave most of the 256 CUs idle
// (e.g. [100 x 24576] x [24576 x 256] ran as 28 workgroups). This kernel
// always covers all M rows in one 128-row tile, tiles N by BN (64 or 128)
// and splits K over gridDim.y so that (N/BN) * S ~ 1-2 workgroups per CU.
// Each split writes its own fp32 partial slab; the CONSUMER (the fused cell
// kernels) sums the S slabs while loading -- the reduction costs no extra
// launch and no atomics, and the result is deterministic.
//
// Both operands are K-contiguous ("NT"): A [M, K] row-major, Bt [N, K]
// row-major (weights are kept in bf16 in both orientations), so MFMA
// fragments are 16-byte vector reads. MFMA: v_mfma_f32_16x16x32_bf16; lane l
// holds A[row l&15][k 8(l>>4) .. +7] and B[k 8(l>>4) .. +7][col l&15];
// C/D: col = l&15, row = 4(l>>4) + i.
//
// Block: 256 threads (4 waves); wave w owns rows 32w..32w+31 x all BN cols
// (2 x BN/16 accumulator tiles). K tile 64, staged by an LDS-DMA ring (below).
// gridDim.z batches independent problems (both encoder directions).
#include <cstdlib>

#include "common.h"
#include "cell_bwd_body.h"
#include "skinny_tile.h"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

using skr::BM;
using skr::BK;
using skr::wait_ahead;

template <int BN, int NS, bool CBF16 = false, bool RA = false>
__global__ __launch_bounds__(256) void skinny_gemm_glds_kernel(
    const __hip_bfloat16* __restrict__ A, int64_t lda, int64_t a_batch,
    const __hip_bfloat16* __restrict__ Bt, int64_t ldb, int64_t b_batch,
    void* __restrict__ C, int64_t ldc, int64_t c_slab, int64_t c_batch, int M, int kslice) {
    extern __shared__ __attribute__((aligned(16))) __hip_bfloat16 smem[];
    const int64_t co = blockIdx.z * c_batch + blockIdx.y * c_slab;
    glds_tile<BN, NS, CBF16, 4, false, RA>(A + blockIdx.z * a_batch, lda, Bt + blockIdx.z * b_batch, ldb,
                  CBF16 ? (void*)((__hip_bfloat16*)C + co) : (void*)((float*)C + co), ldc, M, blockIdx.x * BN,
                  (int64_t)blockIdx.y * kslice, kslice, smem);
}

// Grouped launch: up to kMaxGroup independent products (different operands,
// shapes and split factors, same N-tile width) in ONE launch. The per-step
// products of a recurrence that do not depend on each other (HyperLSTM:
// h @ W_h for the main gates and [h | hh] @ W_y for the hyper gates; in the
// backward dR_main @ W_h^T and dvec @ P^T) then share one kernel boundary
// and fill the chip together instead of each leaving most CUs idle.
// Workgroup id -> (problem, row block, split, N tile) through the prefix
// sums `start` (csrc/skinny_tile.h). A problem with M > 128 rows (M % 128 ==
// 0: the wide decode of sample/hyper_step.py) runs as M / 128 row blocks
// sharing B.
template <int BN, int NS, int NW = 4, bool RA = false>
__global__ __launch_bounds__(NW * 64) void skinny_gemm_group_kernel(const GemmGroup g) {
    extern __shared__ __attribute__((aligned(16))) __hip_bfloat16 smem[];
    group_tile<BN, NS, NW, false, RA>(g, blockIdx.x, smem);
}

// Grouped GEMM tiles + the rows of one backward LayerNorm cell step in ONE
// launch: workgroups [0, B) run the cell rows (one workgroup per row, 256
// threads, one unit per thread: H <= 256), the rest the GEMM tiles. The
// HyperLSTM backward runs its hyper cell -- which needs only the dvec P^T
// slabs of this step -- beside dR_main W_h^T, which only the next step's
// main cell reads: the 100-CU cell step hides under the weight stream
// instead of being its own launch on the critical path.
template <int BN, int NS, int DHS>
__global__ __launch_bounds__(256) void skinny_gemm_group_cellbwd_kernel(const GemmGroup g, const skr::BwdArgs cell) {
    extern __shared__ __attribute__((aligned(16))) __hip_bfloat16 smem[];
    if ((int)blockIdx.x < cell.B) {
        cell_bwd_body<256, 1, 1, true, 0, DHS>(cell, 0, blockIdx.x, 1);
        return;
    }
    group_tile<BN, NS>(g, blockIdx.x - cell.B, smem);
}

// fp32 operands (fp32 parity runs): the same LDS-DMA ring with K-tiles of
// 32 floats (128-byte LDS rows, same chunk swizzle), v_mfma_f32_16x16x4_f32.
// An MFMA consumes one k per lane group, so a lane reads a float4 of its row
// (chunk fq or fq + 4 of the tile) and feeds its four elements to four
// MFMAs: MFMA (g, j) covers k = 16g + 4fq + j -- a permutation of the
// tile's 32 k shared by A and B, so every product term is summed once.
constexpr int BKF = 32;

template <int BN, int NS>
__device__ __forceinline__ void glds_tile_f32(const float* __restrict__ A, int64_t lda, const float* __restrict__ Bt,
                                              int64_t ldb, float* __restrict__ C, int64_t ldc, int M, int n0,
                                              int64_t k0, int kslice, float* smem) {
    constexpr int NJ = BN / 16;
    constexpr int A_CH = BM / 8, B_CH = BN / 8;     // 1-KiB chunks (8 rows x 128 B) per tile
    constexpr int GPW = (A_CH + B_CH) / 4;
    constexpr int TILE = (BM + BN) * BKF;           // floats per stage
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int n = kslice / BKF;
    const int r8 = lane >> 3, slot = lane & 7;
    const float* asrc[A_CH / 4];
    const float* bsrc[B_CH / 4];
#pragma unroll
    for (int i = 0; i < A_CH / 4; ++i) {
        const int row = (w + 4 * i) * 8 + r8;
        const int kc = slot ^ ((row >> 1) & 7);
        asrc[i] = row < M ? A + (int64_t)row * lda + k0 + kc * 4 : A + (int64_t)(M - 1) * lda + k0;
    }
#pragma unroll
    for (int i = 0; i < B_CH / 4; ++i) {
        const int row = (w + 4 * i) * 8 + r8;
        const int kc = slot ^ ((row >> 1) & 7);
        bsrc[i] = Bt + (int64_t)(n0 + row) * ldb + k0 + kc * 4;
    }
    auto issue = [&](int kt) {
        float* st = smem + (kt % NS) * TILE;
        const int64_t ko = (int64_t)kt * BKF;
#pragma unroll
        for (int i = 0; i < A_CH / 4; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + ko),
                                             (__attribute__((address_space(3))) void*)(st + (w + 4 * i) * 256), 16, 0, 0);
#pragma unroll
        for (int i = 0; i < B_CH / 4; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + ko),
                                             (__attribute__((address_space(3))) void*)(st + BM * BKF + (w + 4 * i) * 256),
                                             16, 0, 0);
    };
    f32x4 acc[2][NJ];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
    for (int p = 0; p < NS - 1; ++p)
        if (p < n) issue(p);
    for (int kt = 0; kt < n; ++kt) {
        wait_ahead<GPW, NS>(min(n - 1 - kt, NS - 2));
        __builtin_amdgcn_s_barrier();
        if (kt + NS - 1 < n) issue(kt + NS - 1);
        const float* As = smem + (kt % NS) * TILE;
        const float* Bs = As + BM * BKF;
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            const int kc = fq + 4 * g;
            f32x4 af[2], bfr[NJ];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int row = 32 * w + 16 * i + fr;
                af[i] = *(const f32x4*)(&As[row * BKF + ((kc ^ ((row >> 1) & 7)) * 4)]);
            }
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int row = 16 * j + fr;
                bfr[j] = *(const f32x4*)(&Bs[row * BKF + ((kc ^ ((row >> 1) & 7)) * 4)]);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < NJ; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][e], bfr[j][e], acc[i][j], 0, 0, 0);
        }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = 32 * w + 16 * i + fq * 4 + e;
                if (row < M) C[row * ldc + n0 + 16 * j + fr] = acc[i][j][e];
            }
}

template <int BN, int NS>
__global__ __launch_bounds__(256) void skinny_gemm_f32_kernel(const float* __restrict__ A, int64_t lda,
                                                              int64_t a_batch, const float* __restrict__ Bt,
                                                              int64_t ldb, int64_t b_batch, float* __restrict__ C,
                                                              int64_t ldc, int64_t c_slab, int64_t c_batch, int M,
                                                              int kslice) {
    extern __shared__ __attribute__((aligned(16))) float smemf[];
    glds_tile_f32<BN, NS>(A + blockIdx.z * a_batch, lda, Bt + blockIdx.z * b_batch, ldb,
                          C + blockIdx.z * c_batch + blockIdx.y * c_slab, ldc, M, blockIdx.x * BN,
                          (int64_t)blockIdx.y * kslice, kslice, smemf);
}

}  // namespace

// Ring depth of the v2 / grouped kernels (stages of (BM + BN) x 128 B):
// 3, 4 or 6 (6 only with BN = 64: 144 KiB). skr_gemm_set_nstage() tunes it
// (scripts/bench_gemm.py sweeps it).
static int g_nstage = 3;   // measured best: 2 workgroups per CU fit (72 KiB at BN = 64)
// A in registers (skr::ra_mma) for the plain and grouped launches: 0 off, or
// the register / B-ring depth (3, 4 or 6); skr_gemm_set_ra.
static int g_ra = 0;
SKR_API int skr_gemm_set_ra(int ns) {
    const int prev = g_ra;
    if (ns == 0 || ns == 3 || ns == 4 || ns == 6) g_ra = ns;
    return prev;
}
SKR_API int skr_gemm_set_nstage(int ns) {
    if (ns != 3 && ns != 4 && ns != 6) return -2;
    g_nstage = ns;
    return 0;
}

namespace {

template <typename K>
void set_lds_attr(K k, size_t lds) {
    // per instantiation, once (a HIP graph capture must not see the call twice)
    static bool done = false;
    if (!done) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        done = true;
    }
}

template <int BN, int NS, bool CBF16 = false, bool RA = false>
int launch_v2_k(dim3 grid, hipStream_t s, const void* A, int64_t lda, int64_t a_batch, const void* Bt, int64_t ldb,
                int64_t b_batch, void* C, int64_t ldc, int64_t c_slab, int64_t c_batch, int M, int kslice) {
    const size_t lds = (size_t)NS * ((RA ? 0 : BM) + BN) * BK * 2;
    set_lds_attr(skinny_gemm_glds_kernel<BN, NS, CBF16, RA>, lds);
    hipLaunchKernelGGL((skinny_gemm_glds_kernel<BN, NS, CBF16, RA>), grid, dim3(256), lds, s, (const __hip_bfloat16*)A,
                       lda, a_batch, (const __hip_bfloat16*)Bt, ldb, b_batch, C, ldc, c_slab, c_batch, M, kslice);
    return SKR_CHECK_LAUNCH();
}

template <int BN, int NS, bool CBF16 = false>
int launch_v2(dim3 grid, hipStream_t s, const void* A, int64_t lda, int64_t a_batch, const void* Bt, int64_t ldb,
              int64_t b_batch, void* C, int64_t ldc, int64_t c_slab, int64_t c_batch, int M, int kslice) {
    if (BN == 64 && g_ra) {   // A in registers (4-wave 64-wide tiles)
        if (g_ra == 3) return launch_v2_k<64, 3, CBF16, true>(grid, s, A, lda, a_batch, Bt, ldb, b_batch, C, ldc, c_slab, c_batch, M, kslice);
        if (g_ra == 4) return launch_v2_k<64, 4, CBF16, true>(grid, s, A, lda, a_batch, Bt, ldb, b_batch, C, ldc, c_slab, c_batch, M, kslice);
        return launch_v2_k<64, 6, CBF16, true>(grid, s, A, lda, a_batch, Bt, ldb, b_batch, C, ldc, c_slab, c_batch, M, kslice);
    }
    return launch_v2_k<BN, NS, CBF16, false>(grid, s, A, lda, a_batch, Bt, ldb, b_batch, C, ldc, c_slab, c_batch, M, kslice);
}

template <int BN, int NS, int NW = 4, bool RA = false>
int launch_group_k(const GemmGroup& g, hipStream_t s) {
    const size_t lds = (size_t)NS * ((RA ? 0 : BM) + BN) * BK * 2;
    set_lds_attr(skinny_gemm_group_kernel<BN, NS, NW, RA>, lds);
    hipLaunchKernelGGL((skinny_gemm_group_kernel<BN, NS, NW, RA>), dim3(g.start[g.n]), dim3(NW * 64), lds, s, g);
    return SKR_CHECK_LAUNCH();
}

template <int BN, int NS, int NW = 4>
int launch_group(const GemmGroup& g, hipStream_t s) {
    if (BN == 64 && NW == 4 && g_ra) {
        if (g_ra == 3) return launch_group_k<64, 3, 4, true>(g, s);
        if (g_ra == 4) return launch_group_k<64, 4, 4, true>(g, s);
        return launch_group_k<64, 6, 4, true>(g, s);
    }
    return launch_group_k<BN, NS, NW, false>(g, s);
}

}  // namespace

// Same contract as skr_skinny_gemm, LDS-DMA ring kernel (v2).
SKR_API int skr_skinny_gemm_v2(const void* A, int64_t lda, int64_t a_batch, const void* Bt, int64_t ldb,
                               int64_t b_batch, float* C, int64_t ldc, int64_t c_slab, int64_t c_batch, int M, int N,
                               int K, int splits, int batch, int bn, hipStream_t s) {
    // 64-wide N tiles: with the 3-deep ring two workgroups share a CU and
    // 64 beat 128 on every recurrent shape (scripts/bench_gemm.py)
    if (bn == 0) bn = (g_nstage == 3) ? 64 : ((N % 128 == 0 && (N / 128) * splits * batch >= 144) ? 128 : 64);
    if (M < 1 || M > BM || (bn != 64 && bn != 128) || N % bn != 0 || splits < 1 || K % splits != 0)
        return -2;
    const int kslice = K / splits;
    if (kslice % BK != 0 || lda % 8 != 0 || ldb % 8 != 0) return -3;
    if (((uintptr_t)A | (uintptr_t)Bt) & 15) return -4;
    const dim3 grid(N / bn, splits, batch);
#define SKR_V2(BN_, NS_) launch_v2<BN_, NS_>(grid, s, A, lda, a_batch, Bt, ldb, b_batch, C, ldc, c_slab, c_batch, M, kslice)
    if (bn == 128) return g_nstage == 3 ? SKR_V2(128, 3) : SKR_V2(128, 4);
    return g_nstage == 3 ? SKR_V2(64, 3) : g_nstage == 6 ? SKR_V2(64, 6) : SKR_V2(64, 4);
#undef SKR_V2
}

// As skr_skinny_gemm_v2 with a bf16 output (one slab: splits == 1), for
// products consumed only as bf16 (the HyperLSTM modulation vectors).
SKR_API int skr_skinny_gemm_v2_bf16out(const void* A, int64_t lda, int64_t a_batch, const void* Bt, int64_t ldb,
                                       int64_t b_batch, void* C, int64_t ldc, int64_t c_batch, int M, int N, int K,
                                       int batch, hipStream_t s) {
    if (M < 1 || M > BM || N % 64 != 0 || K % BK != 0 || lda % 8 != 0 || ldb % 8 != 0) return -2;
    if (((uintptr_t)A | (uintptr_t)Bt) & 15) return -4;
    const dim3 grid(N / 64, 1, batch);
    return g_nstage == 3 ? launch_v2<64, 3, true>(grid, s, A, lda, a_batch, Bt, ldb, b_batch, C, ldc, 0, c_batch, M, K)
                         : launch_v2<64, 4, true>(grid, s, A, lda, a_batch, Bt, ldb, b_batch, C, ldc, 0, c_batch, M, K);
}

// Grouped bf16 products (see skinny_gemm_group_kernel): each problem as
// skr_skinny_gemm_v2 with batch 1; all use N tiles of `bn` (0: 64).
SKR_API int skr_skinny_gemm_group(const GemmProblem* probs, int n, int bn, hipStream_t s) {
    if (n < 1 || n > kMaxGroup) return -2;
    if (bn == 0) bn = 64;
    if (bn != 64 && bn != 128) return -2;
    GemmGroup g{};
    g.n = n;
    g.start[0] = 0;
    for (int i = 0; i < n; ++i) {
        const GemmProblem& p = probs[i];
        if (p.M < 1 || p.M > 8 * BM || p.N % bn != 0 || p.splits < 1 || p.K % p.splits != 0) return -2;
        if ((p.K / p.splits) % BK != 0 || p.lda % 8 != 0 || p.ldb % 8 != 0) return -3;
        if (((uintptr_t)p.A | (uintptr_t)p.Bt) & 15) return -4;
        g.p[i] = p;
        g.start[i + 1] = g.start[i] + (p.N / bn) * p.splits * row_blocks_of(p.M);
    }
    for (int i = n + 1; i <= kMaxGroup; ++i) g.start[i] = g.start[n];
    // 128-wide tiles run on 8 waves (512 threads: wave w = row quarter w % 4 x
    // column half w / 4): the same per-wave work as two 64-wide 4-wave
    // workgroups, with the activation rows staged once for 128 columns
    if (bn == 128) return g_nstage == 3 ? launch_group<128, 3, 8>(g, s) : launch_group<128, 4, 8>(g, s);
    return g_nstage == 3 ? launch_group<64, 3>(g, s) : g_nstage == 6 ? launch_group<64, 6>(g, s)
                                                                    : launch_group<64, 4>(g, s);
}

// skr_skinny_gemm_group (64-wide tiles, 3-stage ring) plus one backward
// LayerNorm cell step (lstm_cell.hip semantics, mod 0, one workgroup per
// row: H <= 256, no cluster, no resets) in the same launch.
SKR_API int skr_skinny_gemm_group_cellbwd(const GemmProblem* probs, int n, const skr::BwdArgs* cell, hipStream_t s) {
    if (n < 1 || n > kMaxGroup || cell == nullptr) return -2;
    const skr::BwdArgs& a = *cell;
    if (a.H < 1 || a.H > 256 || a.cluster > 1 || a.reset != nullptr || a.B < 1) return -2;
    if ((a.dh_rec && (a.dhr_nslab < 1 || a.dhr_nslab > kRecSlabs)) ||
        (a.dh_rec2 && (a.dhr2_nslab < 1 || a.dhr2_nslab > kRecSlabs)))
        return -3;
    const int no = a.dh_out ? a.dho_nslab : 1;
    const int dhs = no == 1 ? 1 : no <= 8 ? 8 : no <= 32 ? 32 : no <= 64 ? 64 : 0;
    if (dhs == 0) return -3;
    GemmGroup g{};
    g.n = n;
    g.start[0] = 0;
    for (int i = 0; i < n; ++i) {
        const GemmProblem& p = probs[i];
        const int rc = check_problem64(p);
        if (rc) return rc;
        g.p[i] = p;
        g.start[i + 1] = g.start[i] + (p.N / 64) * p.splits * row_blocks_of(p.M);
    }
    for (int i = n + 1; i <= kMaxGroup; ++i) g.start[i] = g.start[n];
    const size_t lds = (size_t)3 * (BM + 64) * BK * 2;
    const dim3 grid(a.B + g.start[n]);
#define SKR_GC(D)                                                                                           \
    do {                                                                                                    \
        set_lds_attr(skinny_gemm_group_cellbwd_kernel<64, 3, D>, lds);                                      \
        hipLaunchKernelGGL((skinny_gemm_group_cellbwd_kernel<64, 3, D>), grid, dim3(256), lds, s, g, a);    \
    } while (0)
    switch (dhs) {
        case 1: SKR_GC(1); break;
        case 8: SKR_GC(8); break;
        case 32: SKR_GC(32); break;
        default: SKR_GC(64); break;
    }
#undef SKR_GC
    return SKR_CHECK_LAUNCH();
}

// fp32 operands: same contract as skr_skinny_gemm_v2 with kslice % 32 == 0
// (64-wide N tiles, 3-deep ring of (128 + 64) x 128 B stages).
SKR_API int skr_skinny_gemm_f32(const void* A, int64_t lda, int64_t a_batch, const void* Bt, int64_t ldb,
                                int64_t b_batch, float* C, int64_t ldc, int64_t c_slab, int64_t c_batch, int M, int N,
                                int K, int splits, int batch, hipStream_t s) {
    if (M < 1 || M > BM || N % 64 != 0 || splits < 1 || K % splits != 0) return -2;
    const int kslice = K / splits;
    if (kslice % BKF != 0 || lda % 4 != 0 || ldb % 4 != 0) return -3;
    if (((uintptr_t)A | (uintptr_t)Bt) & 15) return -4;
    const dim3 grid(N / 64, splits, batch);
    const size_t lds = (size_t)3 * (BM + 64) * BKF * 4;
    set_lds_attr(skinny_gemm_f32_kernel<64, 3>, lds);
    hipLaunchKernelGGL((skinny_gemm_f32_kernel<64, 3>), grid, dim3(256), lds, s, (const float*)A, lda, a_batch,
                       (const float*)Bt, ldb, b_batch, C, ldc, c_slab, c_batch, M, kslice);
    return SKR_CHECK_LAUNCH();
}

SKR_API int skr_gemm_problem_size() { return (int)sizeof(GemmProblem); }
