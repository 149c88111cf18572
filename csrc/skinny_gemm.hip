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
// (2 x BN/16 accumulator tiles). K tile 64. Pipeline depth 3: tile kt in LDS
// (double-buffered), tile kt+1 in staging registers, tile kt+2's global
// loads issued before tile kt's MFMAs -- with so few MFMAs per tile, one
// tile of lookahead cannot cover the L2/MALL latency.
// Rows padded by 16 B in LDS (conflict-free ds_read_b128 fragment reads).
// gridDim.z batches independent problems (both encoder directions).
#include <cstdlib>

#include "common.h"
#include "cell_fwd_body.h"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int BM = 128, BK = 64, PAD = 8, LDK = BK + PAD;  // LDS row = 144 B

template <int BN>
__global__ __launch_bounds__(256) void skinny_gemm_nt_kernel(
    const __hip_bfloat16* __restrict__ A, int64_t lda, int64_t a_batch,
    const __hip_bfloat16* __restrict__ Bt, int64_t ldb, int64_t b_batch,
    float* __restrict__ C, int64_t ldc, int64_t c_slab, int64_t c_batch, int M, int kslice) {
    constexpr int NJ = BN / 16;
    __shared__ __attribute__((aligned(16))) __hip_bfloat16 As[2][BM * LDK];
    __shared__ __attribute__((aligned(16))) __hip_bfloat16 Bs[2][BN * LDK];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int n0 = blockIdx.x * BN;
    const int64_t k0 = (int64_t)blockIdx.y * kslice;
    const int n = kslice / BK;
    A += blockIdx.z * a_batch;
    Bt += blockIdx.z * b_batch;
    C += blockIdx.z * c_batch + blockIdx.y * c_slab;

    // Staging registers are named scalars, not an array: a private array
    // captured by a lambda is promoted to LDS by the AMDGPU backend, which
    // turns every prefetch into load -> wait -> LDS round trip.
    // Thread t stages A rows t/8 + {0, 32, 64, 96} and B rows t/8 + 32j,
    // 16 bytes each at k offset (t % 8) * 8 -- 128 contiguous bytes per row.
    // Rows >= M re-read row M-1 (never stored): an unconditional load keeps
    // hipcc from branching around it and draining vmcnt.
    const int srow = tid >> 3, skc = (tid & 7) * 8;
    const __hip_bfloat16* a0 = A + (int64_t)min(srow, M - 1) * lda + k0 + skc;
    const __hip_bfloat16* a1 = A + (int64_t)min(srow + 32, M - 1) * lda + k0 + skc;
    const __hip_bfloat16* a2 = A + (int64_t)min(srow + 64, M - 1) * lda + k0 + skc;
    const __hip_bfloat16* a3 = A + (int64_t)min(srow + 96, M - 1) * lda + k0 + skc;
    const __hip_bfloat16* b0 = Bt + (int64_t)(n0 + srow) * ldb + k0 + skc;
    const int64_t bstep = 32 * ldb;
    uint4 xa0, xa1, xa2, xa3, xb0, xb1, xb2, xb3;  // register set X
    uint4 ya0, ya1, ya2, ya3, yb0, yb1, yb2, yb3;  // register set Y
#define SKR_LOAD(P, kt)                                           \
    do {                                                          \
        const int64_t ko = (int64_t)min(kt, n - 1) * BK;          \
        P##a0 = *(const uint4*)(a0 + ko);                         \
        P##a1 = *(const uint4*)(a1 + ko);                         \
        P##a2 = *(const uint4*)(a2 + ko);                         \
        P##a3 = *(const uint4*)(a3 + ko);                         \
        P##b0 = *(const uint4*)(b0 + ko);                         \
        P##b1 = *(const uint4*)(b0 + bstep + ko);                 \
        if constexpr (BN == 128) {                                \
            P##b2 = *(const uint4*)(b0 + 2 * bstep + ko);         \
            P##b3 = *(const uint4*)(b0 + 3 * bstep + ko);         \
        }                                                         \
    } while (0)
#define SKR_STORE(P, buf)                                          \
    do {                                                           \
        *(uint4*)(&As[buf][srow * LDK + skc]) = P##a0;             \
        *(uint4*)(&As[buf][(srow + 32) * LDK + skc]) = P##a1;      \
        *(uint4*)(&As[buf][(srow + 64) * LDK + skc]) = P##a2;      \
        *(uint4*)(&As[buf][(srow + 96) * LDK + skc]) = P##a3;      \
        *(uint4*)(&Bs[buf][srow * LDK + skc]) = P##b0;             \
        *(uint4*)(&Bs[buf][(srow + 32) * LDK + skc]) = P##b1;      \
        if constexpr (BN == 128) {                                 \
            *(uint4*)(&Bs[buf][(srow + 64) * LDK + skc]) = P##b2;  \
            *(uint4*)(&Bs[buf][(srow + 96) * LDK + skc]) = P##b3;  \
        }                                                          \
    } while (0)

    f32x4 acc[2][NJ];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int fr = lane & 15, fk = (lane >> 4) * 8;
    auto compute = [&](int buf) {
#pragma unroll
        for (int ks = 0; ks < BK; ks += 32) {
            bf16x8 af[2], bfr[NJ];
#pragma unroll
            for (int i = 0; i < 2; ++i)
                af[i] = *(const bf16x8*)(&As[buf][(32 * w + 16 * i + fr) * LDK + ks + fk]);
#pragma unroll
            for (int j = 0; j < NJ; ++j) bfr[j] = *(const bf16x8*)(&Bs[buf][(16 * j + fr) * LDK + ks + fk]);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
    };

    // prologue: tile 0 -> LDS[0], tile 1 -> Y (in flight)
    SKR_LOAD(x, 0);
    SKR_LOAD(y, 1);
    SKR_STORE(x, 0);
    __syncthreads();
    // Each half-iteration: issue loads two tiles ahead into the free register
    // set, MFMA the LDS tile, then write the one-ahead set into the other LDS
    // buffer (its wait leaves the newest loads in flight), barrier.
    // Loads past the last tile re-read it (min above): branch-free body.
    // The asm clobber + sched_barrier pin the order: hipcc would otherwise
    // hoist the LDS writes (and their vmcnt wait) above the MFMAs.
    int kt = 0;
    for (;;) {
        SKR_LOAD(x, kt + 2);
        __builtin_amdgcn_sched_barrier(0);
        compute(kt & 1);
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        SKR_STORE(y, (kt + 1) & 1);
        skr::lds_barrier();
        if (++kt >= n) break;
        SKR_LOAD(y, kt + 2);
        __builtin_amdgcn_sched_barrier(0);
        compute(kt & 1);
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        SKR_STORE(x, (kt + 1) & 1);
        skr::lds_barrier();
        if (++kt >= n) break;
    }
#undef SKR_LOAD
#undef SKR_STORE
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = 32 * w + 16 * i + (lane >> 4) * 4 + e;
                if (row < M) C[row * ldc + n0 + 16 * j + fr] = acc[i][j][e];
            }
}

// ---------------------------------------------------------------------------
// v2: LDS-DMA ring. Tiles move global -> LDS with global_load_lds_dwordx4
// (no staging registers, no ds_write), NSTAGE buffers deep: NSTAGE-1 K-tiles
// are in flight while one is multiplied. One counted `s_waitcnt vmcnt(N)`
// plus a raw s_barrier per K-tile (a __syncthreads() would drain every
// prefetch, CDNA4 guide "Pipelining across barriers"). LDS rows are 128 B
// (BK = 64 bf16) with the 16-byte chunk index XOR-swizzled by (row >> 1) & 7
// -- applied on the per-lane GLOBAL address, since an LDS-DMA wave writes
// 1 KiB linearly -- so the 16 rows of a ds_read_b128 fragment read hit 16
// distinct bank quads.
constexpr int NSTAGE = 4;

// One [M<=128, BN] output tile over K range [k0, k0 + kslice) of
// C = A . Bt^T (C points at this split's slab). Shared by the single-problem
// and the grouped launch.
template <int GPW, int NS>
__device__ __forceinline__ void wait_ahead(int ahead) {
    // tile kt landed (for this wave) once at most `ahead` younger tiles are pending
    if constexpr (NS - 2 >= 4) if (ahead >= 4) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * GPW) : "memory"); return; }
    if constexpr (NS - 2 >= 3) if (ahead == 3) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * GPW) : "memory"); return; }
    if constexpr (NS - 2 >= 2) if (ahead == 2) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GPW) : "memory"); return; }
    if (ahead == 1) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GPW) : "memory"); return; }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// BPOL: cache-policy bits of the weight (B) stream's LDS-DMA loads (0 =
// default; 2 = nt, SKR_GEMM_NT=1: CDNA4 guide "nt-weights").
template <int BN, int NS, bool CBF16 = false, int BPOL = 0, bool SC1 = false>
__device__ __forceinline__ void glds_tile(const __hip_bfloat16* __restrict__ A, int64_t lda,
                                          const __hip_bfloat16* __restrict__ Bt, int64_t ldb,
                                          void* __restrict__ Cv, int64_t ldc, int M, int n0, int64_t k0, int kslice,
                                          __hip_bfloat16* smem) {
    constexpr int NJ = BN / 16;
    constexpr int A_CH = BM / 8, B_CH = BN / 8;     // 1-KiB chunks (8 rows) per tile
    constexpr int GPW = (A_CH + B_CH) / 4;          // glds per wave per tile
    constexpr int TILE = (BM + BN) * BK;            // bf16 elements per stage
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int n = kslice / BK;

    // per-lane source rows / swizzled chunk (fixed across tiles)
    const int r8 = lane >> 3, slot = lane & 7;
    const __hip_bfloat16* asrc[A_CH / 4];
    const __hip_bfloat16* bsrc[B_CH / 4];
#pragma unroll
    for (int i = 0; i < A_CH / 4; ++i) {
        const int row = (w + 4 * i) * 8 + r8;
        const int kc = slot ^ ((row >> 1) & 7);
        // rows past M: every lane of the chunk reads the same 16 bytes (one
        // line instead of 1 KiB; the wave's glds count stays uniform)
        asrc[i] = row < M ? A + (int64_t)row * lda + k0 + kc * 8 : A + (int64_t)(M - 1) * lda + k0;
    }
#pragma unroll
    for (int i = 0; i < B_CH / 4; ++i) {
        const int row = (w + 4 * i) * 8 + r8;
        const int kc = slot ^ ((row >> 1) & 7);
        bsrc[i] = Bt + (int64_t)(n0 + row) * ldb + k0 + kc * 8;
    }
    auto issue = [&](int kt) {
        __hip_bfloat16* st = smem + (kt % NS) * TILE;
        const int64_t ko = (int64_t)kt * BK;
#pragma unroll
        for (int i = 0; i < A_CH / 4; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + ko),
                                             (__attribute__((address_space(3))) void*)(st + (w + 4 * i) * 512), 16, 0, 0);
#pragma unroll
        for (int i = 0; i < B_CH / 4; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + ko),
                                             (__attribute__((address_space(3))) void*)(st + BM * BK + (w + 4 * i) * 512),
                                             16, 0, BPOL);
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
        __builtin_amdgcn_s_barrier();  // ... and for every wave; buffer (kt-1) % NS is free
        if (kt + NS - 1 < n) issue(kt + NS - 1);
        const __hip_bfloat16* As = smem + (kt % NS) * TILE;
        const __hip_bfloat16* Bs = As + BM * BK;
#pragma unroll
        for (int ks = 0; ks < BK; ks += 32) {
            const int kc = ks / 8 + fq;
            bf16x8 af[2], bfr[NJ];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int row = 32 * w + 16 * i + fr;
                af[i] = *(const bf16x8*)(&As[row * BK + ((kc ^ ((row >> 1) & 7)) * 8)]);
            }
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int row = 16 * j + fr;
                bfr[j] = *(const bf16x8*)(&Bs[row * BK + ((kc ^ ((row >> 1) & 7)) * 8)]);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = 32 * w + 16 * i + fq * 4 + e;
                if (row < M) {
                    if constexpr (CBF16) ((__hip_bfloat16*)Cv)[row * ldc + n0 + 16 * j + fr] = skr::to_bf16(acc[i][j][e]);
                    else if constexpr (SC1)   // write-through: read by other workgroups of this launch
                        __hip_atomic_store((uint32_t*)Cv + row * ldc + n0 + 16 * j + fr,
                                           __float_as_uint(acc[i][j][e]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    else ((float*)Cv)[row * ldc + n0 + 16 * j + fr] = acc[i][j][e];
                }
            }
}

// v3 ("A in registers"): the B (weight) tiles alone go through the LDS-DMA
// ring, NSB stages deep (8 KiB per stage at BN = 64, so 7 tiles of weights
// are in flight per workgroup instead of 2), while each wave loads its own
// 32 rows of the small, L2-resident A operand straight into MFMA fragment
// registers, NSB tiles deep as well (a register ring indexed by the
// unrolled slot). Per tile and lane: 4 A loads + B_CH/4 glds, in that
// order; the counted wait covers both.
template <int LPT, int AHEAD>
__device__ __forceinline__ void wait_tiles_ra(int ahead) {
    if constexpr (AHEAD >= 6) if (ahead >= 6) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 * LPT) : "memory"); return; }
    if constexpr (AHEAD >= 5) if (ahead == 5) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(5 * LPT) : "memory"); return; }
    if constexpr (AHEAD >= 4) if (ahead == 4) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * LPT) : "memory"); return; }
    if constexpr (AHEAD >= 3) if (ahead == 3) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * LPT) : "memory"); return; }
    if constexpr (AHEAD >= 2) if (ahead == 2) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LPT) : "memory"); return; }
    if (ahead == 1) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPT) : "memory"); return; }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int BN, int NSB, bool CBF16 = false>
__device__ __forceinline__ void glds_tile_ra(const __hip_bfloat16* __restrict__ A, int64_t lda,
                                             const __hip_bfloat16* __restrict__ Bt, int64_t ldb,
                                             void* __restrict__ Cv, int64_t ldc, int M, int n0, int64_t k0,
                                             int kslice, __hip_bfloat16* smem) {
    constexpr int NJ = BN / 16;
    constexpr int B_CH = BN / 8;                    // 1-KiB chunks (8 rows) per B tile
    constexpr int GPW = B_CH / 4;                   // glds per wave per tile
    constexpr int LPT = 4 + GPW;                    // vector-memory ops per lane per tile
    constexpr int TILE = BN * BK;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int n = kslice / BK;
    const int fr = lane & 15, fq = lane >> 4;
    const int r8 = lane >> 3, slot8 = lane & 7;
    const __hip_bfloat16* bsrc[GPW];
#pragma unroll
    for (int i = 0; i < GPW; ++i) {
        const int row = (w + 4 * i) * 8 + r8;
        const int kc = slot8 ^ ((row >> 1) & 7);
        bsrc[i] = Bt + (int64_t)(n0 + row) * ldb + k0 + kc * 8;
    }
    // A fragment rows of this wave (rows past M re-read row M-1; never stored)
    const __hip_bfloat16* asrc0 = A + (int64_t)min(32 * w + fr, M - 1) * lda + k0 + fq * 8;
    const __hip_bfloat16* asrc1 = A + (int64_t)min(32 * w + 16 + fr, M - 1) * lda + k0 + fq * 8;
    bf16x8 ar[NSB][2][2];   // [slot][row tile][k step]

#define SKR_RA_ISSUE(KT, SL)                                                                                   \
    do {                                                                                                      \
        const int64_t ko_ = (int64_t)(KT) * BK;                                                               \
        ar[SL][0][0] = *(const bf16x8*)(asrc0 + ko_);                                                         \
        ar[SL][0][1] = *(const bf16x8*)(asrc0 + ko_ + 32);                                                    \
        ar[SL][1][0] = *(const bf16x8*)(asrc1 + ko_);                                                         \
        ar[SL][1][1] = *(const bf16x8*)(asrc1 + ko_ + 32);                                                    \
        __hip_bfloat16* st_ = smem + (SL) * TILE;                                                             \
        _Pragma("unroll") for (int i_ = 0; i_ < GPW; ++i_)                                                    \
            __builtin_amdgcn_global_load_lds((const void*)(bsrc[i_] + ko_),                                   \
                                             (__attribute__((address_space(3))) void*)(st_ + (w + 4 * i_) * 512), \
                                             16, 0, 0);                                                       \
    } while (0)

    f32x4 acc[2][NJ];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int p = 0; p < NSB - 1; ++p)
        if (p < n) SKR_RA_ISSUE(p, p);
    for (int kt0 = 0; kt0 < n; kt0 += NSB) {
#pragma unroll
        for (int j = 0; j < NSB; ++j) {
            const int kt = kt0 + j;
            if (kt < n) {
                wait_tiles_ra<LPT, NSB - 2>(min(n - 1 - kt, NSB - 2));
                __builtin_amdgcn_s_barrier();   // every wave's B chunks of tile kt landed; slot (kt-1) free
                if (kt + NSB - 1 < n) SKR_RA_ISSUE(kt + NSB - 1, (j + NSB - 1) % NSB);
                const __hip_bfloat16* Bs = smem + j * TILE;
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    const int kc = ks * 4 + fq;
                    bf16x8 bfr[NJ];
#pragma unroll
                    for (int jj = 0; jj < NJ; ++jj) {
                        const int row = 16 * jj + fr;
                        bfr[jj] = *(const bf16x8*)(&Bs[row * BK + ((kc ^ ((row >> 1) & 7)) * 8)]);
                    }
#pragma unroll
                    for (int i = 0; i < 2; ++i)
#pragma unroll
                        for (int jj = 0; jj < NJ; ++jj)
                            acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ar[j][i][ks], bfr[jj], acc[i][jj], 0, 0, 0);
                }
            }
        }
    }
#undef SKR_RA_ISSUE
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = 32 * w + 16 * i + fq * 4 + e;
                if (row < M) {
                    if constexpr (CBF16) ((__hip_bfloat16*)Cv)[row * ldc + n0 + 16 * j + fr] = skr::to_bf16(acc[i][j][e]);
                    else ((float*)Cv)[row * ldc + n0 + 16 * j + fr] = acc[i][j][e];
                }
            }
}

template <int BN, int NSB, bool CBF16 = false>
__global__ __launch_bounds__(256) void skinny_gemm_ra_kernel(
    const __hip_bfloat16* __restrict__ A, int64_t lda, int64_t a_batch,
    const __hip_bfloat16* __restrict__ Bt, int64_t ldb, int64_t b_batch,
    void* __restrict__ C, int64_t ldc, int64_t c_slab, int64_t c_batch, int M, int kslice) {
    extern __shared__ __attribute__((aligned(16))) __hip_bfloat16 smem[];
    const int64_t co = blockIdx.z * c_batch + blockIdx.y * c_slab;
    glds_tile_ra<BN, NSB, CBF16>(A + blockIdx.z * a_batch, lda, Bt + blockIdx.z * b_batch, ldb,
                                 CBF16 ? (void*)((__hip_bfloat16*)C + co) : (void*)((float*)C + co), ldc, M,
                                 blockIdx.x * BN, (int64_t)blockIdx.y * kslice, kslice, smem);
}

template <int BN, int NS, bool CBF16 = false, int BPOL = 0>
__global__ __launch_bounds__(256) void skinny_gemm_glds_kernel(
    const __hip_bfloat16* __restrict__ A, int64_t lda, int64_t a_batch,
    const __hip_bfloat16* __restrict__ Bt, int64_t ldb, int64_t b_batch,
    void* __restrict__ C, int64_t ldc, int64_t c_slab, int64_t c_batch, int M, int kslice) {
    extern __shared__ __attribute__((aligned(16))) __hip_bfloat16 smem[];
    const int64_t co = blockIdx.z * c_batch + blockIdx.y * c_slab;
    glds_tile<BN, NS, CBF16, BPOL>(A + blockIdx.z * a_batch, lda, Bt + blockIdx.z * b_batch, ldb,
                  CBF16 ? (void*)((__hip_bfloat16*)C + co) : (void*)((float*)C + co), ldc, M, blockIdx.x * BN,
                  (int64_t)blockIdx.y * kslice, kslice, smem);
}

// Grouped launch: up to kMaxGroup independent products (different operands,
// shapes and split factors, same N-tile width) in ONE launch. The per-step
// products of a recurrence that do not depend on each other (HyperLSTM:
// h @ W_h for the main gates and [h | hh] @ W_y for the hyper gates; in the
// backward dR_main @ W_h^T and dvec @ P^T) then share one kernel boundary
// and fill the chip together instead of each leaving most CUs idle.
// Workgroup id -> (problem, split, N tile) through the prefix sums `start`.
}  // namespace

struct GemmProblem {
    const void* A; int64_t lda;
    const void* Bt; int64_t ldb;
    float* C; int64_t ldc; int64_t c_slab;
    int M, N, K, splits;
};

namespace {

constexpr int kMaxGroup = 4;
struct GemmGroup {
    GemmProblem p[kMaxGroup];
    int start[kMaxGroup + 1];
    int n;
};

template <int BN, int NS, int BPOL = 0>
__global__ __launch_bounds__(256) void skinny_gemm_group_kernel(const GemmGroup g) {
    extern __shared__ __attribute__((aligned(16))) __hip_bfloat16 smem[];
    const int id = blockIdx.x;
    int q = 0;
#pragma unroll
    for (int i = 1; i < kMaxGroup; ++i) q += (i < g.n && id >= g.start[i]) ? 1 : 0;
    const GemmProblem& p = g.p[q];
    const int local = id - g.start[q];
    const int ntiles = p.N / BN;
    const int split = local / ntiles, nt = local - split * ntiles;
    const int kslice = p.K / p.splits;
    glds_tile<BN, NS, false, BPOL>((const __hip_bfloat16*)p.A, p.lda, (const __hip_bfloat16*)p.Bt, p.ldb,
                                   p.C + split * p.c_slab, p.ldc, p.M, nt * BN, (int64_t)split * kslice, kslice, smem);
}

template <int BN, int NSB>
__global__ __launch_bounds__(256) void skinny_gemm_group_ra_kernel(const GemmGroup g) {
    extern __shared__ __attribute__((aligned(16))) __hip_bfloat16 smem[];
    const int id = blockIdx.x;
    int q = 0;
#pragma unroll
    for (int i = 1; i < kMaxGroup; ++i) q += (i < g.n && id >= g.start[i]) ? 1 : 0;
    const GemmProblem& p = g.p[q];
    const int local = id - g.start[q];
    const int ntiles = p.N / BN;
    const int split = local / ntiles, nt = local - split * ntiles;
    const int kslice = p.K / p.splits;
    glds_tile_ra<BN, NSB>((const __hip_bfloat16*)p.A, p.lda, (const __hip_bfloat16*)p.Bt, p.ldb, p.C + split * p.c_slab,
                          p.ldc, p.M, nt * BN, (int64_t)split * kslice, kslice, smem);
}

// Grouped launch with the HyperLSTM's hyper cell in its tail (forward).
// Problem 0 is the hyper gates' product R_hyp = [h | hh] @ W_y (its
// workgroups get the lowest ids, so they are dispatched first and are all
// resident); the other problems (R_main) run as in skinny_gemm_group_kernel.
// A problem-0 workgroup stores its split-K slab write-through (sc1), drains,
// and adds one to the step's arrival counter; once all n0 have arrived
// (bounded relaxed poll by one lane, then ONE agent-scope acquire for the
// workgroup: CDNA4 guide Guideline 16) it runs the hyper cell
// (csrc/cell_fwd_body.h: LayerNorm LSTM, 256 units, 4 slabs, one row per
// workgroup pass) for rows local, local + n0, ... So the cell overlaps the
// R_main weight stream instead of costing its own launch.
constexpr unsigned kFuseSpinLimit = 1u << 22;

template <int BN, int NS, int HNS>
__global__ __launch_bounds__(256) void skinny_gemm_group_hyper_kernel(const GemmGroup g, const FwdArgs hc,
                                                                      int* __restrict__ counter, int* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) __hip_bfloat16 smem[];
    const int id = blockIdx.x;
    int q = 0;
#pragma unroll
    for (int i = 1; i < kMaxGroup; ++i) q += (i < g.n && id >= g.start[i]) ? 1 : 0;
    const GemmProblem& p = g.p[q];
    const int local = id - g.start[q];
    const int ntiles = p.N / BN;
    const int split = local / ntiles, nt = local - split * ntiles;
    const int kslice = p.K / p.splits;
    if (q != 0) {
        glds_tile<BN, NS>((const __hip_bfloat16*)p.A, p.lda, (const __hip_bfloat16*)p.Bt, p.ldb, p.C + split * p.c_slab,
                          p.ldc, p.M, nt * BN, (int64_t)split * kslice, kslice, smem);
        return;
    }
    glds_tile<BN, NS, false, 0, true>((const __hip_bfloat16*)p.A, p.lda, (const __hip_bfloat16*)p.Bt, p.ldb,
                                      p.C + split * p.c_slab, p.ldc, p.M, nt * BN, (int64_t)split * kslice, kslice,
                                      smem);
    const int n0 = g.start[1];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its sc1 slab stores
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned spins = 0;
        while (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < n0) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > kFuseSpinLimit) {
                __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    for (int b = local; b < hc.B; b += n0) {
        cell_fwd_body<256, 1, HNS, true, 0>(hc, 0, b, 1);
        __syncthreads();   // the body's LDS scratch is reused by the next row
    }
}

// ---------------------------------------------------------------------------
// fp8 (OCP e4m3) variant of the v2 ring for inference-time recurrent
// products: operands are bytes, a K-tile is 128 elements (the same 128-byte
// LDS rows and swizzle as the bf16 kernel), v_mfma_f32_16x16x32_fp8_fp8
// (lane l: 8 bytes of row l&15 at k 8(l>>4)). Epilogue applies the per-
// output-column weight scale and the activation scale: C = acc * sa * sb[n].
constexpr int BK8 = 128;

template <int BN>
__global__ __launch_bounds__(256) void skinny_gemm_fp8_kernel(
    const uint8_t* __restrict__ A, int64_t lda, int64_t a_batch,
    const uint8_t* __restrict__ Bt, int64_t ldb, int64_t b_batch, const float* __restrict__ b_scale,
    int64_t bs_batch, float a_scale,
    float* __restrict__ C, int64_t ldc, int64_t c_slab, int64_t c_batch, int M, int kslice) {
    constexpr int NJ = BN / 16;
    constexpr int A_CH = BM / 8, B_CH = BN / 8;      // 1-KiB chunks (8 rows x 128 B) per tile
    constexpr int GPW = (A_CH + B_CH) / 4;
    constexpr int TILE = (BM + BN) * BK8;            // bytes per stage
    extern __shared__ __attribute__((aligned(16))) uint8_t smem8[];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int n0 = blockIdx.x * BN;
    const int64_t k0 = (int64_t)blockIdx.y * kslice;
    const int n = kslice / BK8;
    A += blockIdx.z * a_batch;
    Bt += blockIdx.z * b_batch;
    b_scale += blockIdx.z * bs_batch;
    C += blockIdx.z * c_batch + blockIdx.y * c_slab;

    const int r8 = lane >> 3, slot = lane & 7;
    const uint8_t* asrc[A_CH / 4];
    const uint8_t* bsrc[B_CH / 4];
#pragma unroll
    for (int i = 0; i < A_CH / 4; ++i) {
        const int row = (w + 4 * i) * 8 + r8;
        asrc[i] = A + (int64_t)min(row, M - 1) * lda + k0 + (slot ^ ((row >> 1) & 7)) * 16;
    }
#pragma unroll
    for (int i = 0; i < B_CH / 4; ++i) {
        const int row = (w + 4 * i) * 8 + r8;
        bsrc[i] = Bt + (int64_t)(n0 + row) * ldb + k0 + (slot ^ ((row >> 1) & 7)) * 16;
    }
    auto issue = [&](int kt) {
        uint8_t* st = smem8 + (kt % NSTAGE) * TILE;
        const int64_t ko = (int64_t)kt * BK8;
#pragma unroll
        for (int i = 0; i < A_CH / 4; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + ko),
                                             (__attribute__((address_space(3))) void*)(st + (w + 4 * i) * 1024), 16, 0, 0);
#pragma unroll
        for (int i = 0; i < B_CH / 4; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + ko),
                                             (__attribute__((address_space(3))) void*)(st + BM * BK8 + (w + 4 * i) * 1024),
                                             16, 0, 0);
    };

    f32x4 acc[2][NJ];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
    for (int p = 0; p < NSTAGE - 1; ++p)
        if (p < n) issue(p);
    for (int kt = 0; kt < n; ++kt) {
        const int ahead = min(n - 1 - kt, NSTAGE - 2);
        if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GPW) : "memory");
        else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GPW) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (kt + NSTAGE - 1 < n) issue(kt + NSTAGE - 1);
        const uint8_t* As = smem8 + (kt % NSTAGE) * TILE;
        const uint8_t* Bs = As + BM * BK8;
#pragma unroll
        for (int ks = 0; ks < BK8 / 32; ++ks) {
            const int c16 = ks * 2 + (fq >> 1), half = (fq & 1) * 8;
            long af[2], bfr[NJ];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int row = 32 * w + 16 * i + fr;
                af[i] = *(const long*)(&As[row * BK8 + ((c16 ^ ((row >> 1) & 7)) * 16) + half]);
            }
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int row = 16 * j + fr;
                bfr[j] = *(const long*)(&Bs[row * BK8 + ((c16 ^ ((row >> 1) & 7)) * 16) + half]);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const float sc = a_scale * b_scale[n0 + 16 * j + fr];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = 32 * w + 16 * i + fq * 4 + e;
                if (row < M) C[row * ldc + n0 + 16 * j + fr] = acc[i][j][e] * sc;
            }
    }
}

// fp8 v2: the same tile as glds_tile (ring depth NS, counted waits, grouped
// launch, optional bf16 output) on e4m3 operands: K-tiles of 128 bytes,
// v_mfma_f32_16x16x32_fp8_fp8, epilogue C = acc * a_scale * b_scale[n]. At
// NS = 3 a stage is (128 + 64) x 128 B = 24 KiB: two workgroups per CU, like
// the bf16 ring, while every byte moved carries twice the K extent.
template <int BN, int NS, bool CBF16>
__device__ __forceinline__ void glds_tile_fp8(const uint8_t* __restrict__ A, int64_t lda,
                                              const uint8_t* __restrict__ Bt, int64_t ldb,
                                              const float* __restrict__ b_scale, float a_scale,
                                              void* __restrict__ Cv, int64_t ldc, int M, int n0, int64_t k0,
                                              int kslice, uint8_t* smem8) {
    constexpr int NJ = BN / 16;
    constexpr int A_CH = BM / 8, B_CH = BN / 8;
    constexpr int GPW = (A_CH + B_CH) / 4;
    constexpr int TILE = (BM + BN) * BK8;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int n = kslice / BK8;
    const int r8 = lane >> 3, slot = lane & 7;
    const uint8_t* asrc[A_CH / 4];
    const uint8_t* bsrc[B_CH / 4];
#pragma unroll
    for (int i = 0; i < A_CH / 4; ++i) {
        const int row = (w + 4 * i) * 8 + r8;
        // rows past M: every lane of the chunk reads the same 16 bytes
        asrc[i] = row < M ? A + (int64_t)row * lda + k0 + (slot ^ ((row >> 1) & 7)) * 16
                          : A + (int64_t)(M - 1) * lda + k0;
    }
#pragma unroll
    for (int i = 0; i < B_CH / 4; ++i) {
        const int row = (w + 4 * i) * 8 + r8;
        bsrc[i] = Bt + (int64_t)(n0 + row) * ldb + k0 + (slot ^ ((row >> 1) & 7)) * 16;
    }
    auto issue = [&](int kt) {
        uint8_t* st = smem8 + (kt % NS) * TILE;
        const int64_t ko = (int64_t)kt * BK8;
#pragma unroll
        for (int i = 0; i < A_CH / 4; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + ko),
                                             (__attribute__((address_space(3))) void*)(st + (w + 4 * i) * 1024), 16, 0, 0);
#pragma unroll
        for (int i = 0; i < B_CH / 4; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + ko),
                                             (__attribute__((address_space(3))) void*)(st + BM * BK8 + (w + 4 * i) * 1024),
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
        const uint8_t* As = smem8 + (kt % NS) * TILE;
        const uint8_t* Bs = As + BM * BK8;
#pragma unroll
        for (int ks = 0; ks < BK8 / 32; ++ks) {
            const int c16 = ks * 2 + (fq >> 1), half = (fq & 1) * 8;
            long af[2], bfr[NJ];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int row = 32 * w + 16 * i + fr;
                af[i] = *(const long*)(&As[row * BK8 + ((c16 ^ ((row >> 1) & 7)) * 16) + half]);
            }
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int row = 16 * j + fr;
                bfr[j] = *(const long*)(&Bs[row * BK8 + ((c16 ^ ((row >> 1) & 7)) * 16) + half]);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const float sc = a_scale * b_scale[n0 + 16 * j + fr];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = 32 * w + 16 * i + fq * 4 + e;
                if (row < M) {
                    const float v = acc[i][j][e] * sc;
                    if constexpr (CBF16) ((__hip_bfloat16*)Cv)[row * ldc + n0 + 16 * j + fr] = skr::to_bf16(v);
                    else ((float*)Cv)[row * ldc + n0 + 16 * j + fr] = v;
                }
            }
    }
}

template <int BN, int NS, bool CBF16>
__global__ __launch_bounds__(256) void skinny_gemm_fp8v2_kernel(const uint8_t* __restrict__ A, int64_t lda,
                                                                const uint8_t* __restrict__ Bt, int64_t ldb,
                                                                const float* __restrict__ b_scale, float a_scale,
                                                                void* __restrict__ C, int64_t ldc, int64_t c_slab,
                                                                int M, int kslice) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem8[];
    const int64_t co = blockIdx.y * c_slab;
    glds_tile_fp8<BN, NS, CBF16>(A, lda, Bt, ldb, b_scale, a_scale,
                                 CBF16 ? (void*)((__hip_bfloat16*)C + co) : (void*)((float*)C + co), ldc, M,
                                 blockIdx.x * BN, (int64_t)blockIdx.y * kslice, kslice, smem8);
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

// C[z][s] (slab s of batch z) = A[z][:, s*kslice:(s+1)*kslice] . Bt[z][:, same]^T
// bn: N tile (64 or 128; 0 = choose). Requirements: M <= 128, N % bn == 0,
// kslice % 64 == 0, splits * kslice == K, 16-byte aligned rows.
SKR_API int skr_skinny_gemm(const void* A, int64_t lda, int64_t a_batch, const void* Bt, int64_t ldb,
                            int64_t b_batch, float* C, int64_t ldc, int64_t c_slab, int64_t c_batch, int M, int N,
                            int K, int splits, int batch, int bn, hipStream_t s) {
    if (bn == 0) bn = (N % 128 == 0 && (N / 128) * splits * batch >= 192) ? 128 : 64;
    if (M < 1 || M > BM || (bn != 64 && bn != 128) || N % bn != 0 || splits < 1 || K % splits != 0) return -2;
    const int kslice = K / splits;
    if (kslice % BK != 0 || lda % 8 != 0 || ldb % 8 != 0) return -3;
    if (((uintptr_t)A | (uintptr_t)Bt) & 15) return -4;
    const dim3 grid(N / bn, splits, batch);
    if (bn == 128)
        hipLaunchKernelGGL(skinny_gemm_nt_kernel<128>, grid, dim3(256), 0, s, (const __hip_bfloat16*)A, lda, a_batch,
                           (const __hip_bfloat16*)Bt, ldb, b_batch, C, ldc, c_slab, c_batch, M, kslice);
    else
        hipLaunchKernelGGL(skinny_gemm_nt_kernel<64>, grid, dim3(256), 0, s, (const __hip_bfloat16*)A, lda, a_batch,
                           (const __hip_bfloat16*)Bt, ldb, b_batch, C, ldc, c_slab, c_batch, M, kslice);
    return SKR_CHECK_LAUNCH();
}

// Ring depth of the v2 / grouped kernels (stages of (BM + BN) x 128 B):
// 3, 4 or 6 (6 only with BN = 64: 144 KiB). skr_gemm_set_nstage() tunes it
// (scripts/bench_gemm.py sweeps it).
static int g_nstage = 3;   // measured best: 2 workgroups per CU fit (72 KiB at BN = 64)
// v3 (A operand in registers, B-only LDS ring of kRaStages): SKR_GEMM_AREG=1.
// Off by default -- measured on MI355X: vae_large 32.5 ms/step against
// 29.6 with the v2 ring (numerics identical to the tolerance of the tests).
static const int kRaStages = 8;
static int g_areg = -1;
static bool areg_on() {
    if (g_areg < 0) {
        const char* e = getenv("SKR_GEMM_AREG");
        g_areg = (e != nullptr && atoi(e) == 1) ? 1 : 0;
    }
    return g_areg == 1;
}

// Weight-stream cache policy of the v2 / grouped kernels: SKR_GEMM_NT=1
// loads the B operand non-temporally (nt); default policy otherwise.
// OFF by default -- measured on MI355X: vae_large 30.3 vs 28.5 ms/step, the
// grouped forward GEMM 14.0 vs 12.8 us (profiles/r2s5/bench_gemm_nt.log):
// each weight is re-read every time step and the default policy keeps it
// cache-resident between steps.
static int g_bnt = -1;
static bool bnt_on() {
    if (g_bnt < 0) {
        const char* e = getenv("SKR_GEMM_NT");
        g_bnt = (e != nullptr && atoi(e) == 1) ? 1 : 0;
    }
    return g_bnt == 1;
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

template <int BN, int NS, bool CBF16 = false>
int launch_v2(dim3 grid, hipStream_t s, const void* A, int64_t lda, int64_t a_batch, const void* Bt, int64_t ldb,
              int64_t b_batch, void* C, int64_t ldc, int64_t c_slab, int64_t c_batch, int M, int kslice) {
    if (BN == 64 && areg_on()) {   // (v3 is instantiated for 64-wide tiles only)
        const size_t lds_ra = (size_t)kRaStages * BN * BK * 2;
        set_lds_attr(skinny_gemm_ra_kernel<BN, kRaStages, CBF16>, lds_ra);
        hipLaunchKernelGGL((skinny_gemm_ra_kernel<BN, kRaStages, CBF16>), grid, dim3(256), lds_ra, s,
                           (const __hip_bfloat16*)A, lda, a_batch, (const __hip_bfloat16*)Bt, ldb, b_batch, C, ldc,
                           c_slab, c_batch, M, kslice);
        return SKR_CHECK_LAUNCH();
    }
    const size_t lds = (size_t)NS * (BM + BN) * BK * 2;
    if (bnt_on()) {
        set_lds_attr(skinny_gemm_glds_kernel<BN, NS, CBF16, 2>, lds);
        hipLaunchKernelGGL((skinny_gemm_glds_kernel<BN, NS, CBF16, 2>), grid, dim3(256), lds, s,
                           (const __hip_bfloat16*)A, lda, a_batch, (const __hip_bfloat16*)Bt, ldb, b_batch, C, ldc,
                           c_slab, c_batch, M, kslice);
        return SKR_CHECK_LAUNCH();
    }
    set_lds_attr(skinny_gemm_glds_kernel<BN, NS, CBF16>, lds);
    hipLaunchKernelGGL((skinny_gemm_glds_kernel<BN, NS, CBF16>), grid, dim3(256), lds, s, (const __hip_bfloat16*)A,
                       lda, a_batch, (const __hip_bfloat16*)Bt, ldb, b_batch, C, ldc, c_slab, c_batch, M, kslice);
    return SKR_CHECK_LAUNCH();
}

template <int BN, int NS>
int launch_group(const GemmGroup& g, hipStream_t s) {
    if (BN == 64 && areg_on()) {   // (v3 is instantiated for 64-wide tiles only)
        const size_t lds_ra = (size_t)kRaStages * BN * BK * 2;
        set_lds_attr(skinny_gemm_group_ra_kernel<BN, kRaStages>, lds_ra);
        hipLaunchKernelGGL((skinny_gemm_group_ra_kernel<BN, kRaStages>), dim3(g.start[g.n]), dim3(256), lds_ra, s, g);
        return SKR_CHECK_LAUNCH();
    }
    const size_t lds = (size_t)NS * (BM + BN) * BK * 2;
    if (bnt_on()) {
        set_lds_attr(skinny_gemm_group_kernel<BN, NS, 2>, lds);
        hipLaunchKernelGGL((skinny_gemm_group_kernel<BN, NS, 2>), dim3(g.start[g.n]), dim3(256), lds, s, g);
        return SKR_CHECK_LAUNCH();
    }
    set_lds_attr(skinny_gemm_group_kernel<BN, NS>, lds);
    hipLaunchKernelGGL((skinny_gemm_group_kernel<BN, NS>), dim3(g.start[g.n]), dim3(256), lds, s, g);
    return SKR_CHECK_LAUNCH();
}

}  // namespace

// Same contract as skr_skinny_gemm, LDS-DMA ring kernel (v2).
SKR_API int skr_skinny_gemm_v2(const void* A, int64_t lda, int64_t a_batch, const void* Bt, int64_t ldb,
                               int64_t b_batch, float* C, int64_t ldc, int64_t c_slab, int64_t c_batch, int M, int N,
                               int K, int splits, int batch, int bn, hipStream_t s) {
    // 64-wide N tiles: with the 3-deep ring two workgroups share a CU and
    // 64 beat 128 on every recurrent shape (scripts/bench_gemm.py)
    if (bn == 0) bn = (g_nstage == 3) ? 64 : ((N % 128 == 0 && (N / 128) * splits * batch >= 144) ? 128 : 64);
    if (M < 1 || M > BM || (bn != 64 && bn != 128) || N % bn != 0 || splits < 1 || K % splits != 0) return -2;
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
        if (p.M < 1 || p.M > BM || p.N % bn != 0 || p.splits < 1 || p.K % p.splits != 0) return -2;
        if ((p.K / p.splits) % BK != 0 || p.lda % 8 != 0 || p.ldb % 8 != 0) return -3;
        if (((uintptr_t)p.A | (uintptr_t)p.Bt) & 15) return -4;
        g.p[i] = p;
        g.start[i + 1] = g.start[i] + (p.N / bn) * p.splits;
    }
    for (int i = n + 1; i <= kMaxGroup; ++i) g.start[i] = g.start[n];
    if (bn == 128) return g_nstage == 3 ? launch_group<128, 3>(g, s) : launch_group<128, 4>(g, s);
    return g_nstage == 3 ? launch_group<64, 3>(g, s) : g_nstage == 6 ? launch_group<64, 6>(g, s)
                                                                    : launch_group<64, 4>(g, s);
}

// Grouped bf16 products with the hyper cell fused into the tail (see
// skinny_gemm_group_hyper_kernel). probs[0] = R_hyp ([B, 4*256] over 4
// splits: the slabs hc->R points at), probs[1..] = other independent
// products; hc = the hyper cell's forward arguments (training-mode LayerNorm
// cell, H = 256, one workgroup per row); counter = an int zeroed before the
// sequence (one per step); err = timeout flag (the trainers raise on it).
SKR_API int skr_skinny_gemm_group_hyper(const GemmProblem* probs, int n, const FwdArgs* hc, int* counter, int* err,
                                        hipStream_t s) {
    if (n < 1 || n > kMaxGroup || hc == nullptr || counter == nullptr || err == nullptr) return -2;
    const GemmProblem& h = probs[0];
    if (hc->H != 256 || (hc->R_nslab != 4 && hc->R_nslab != 9) || h.splits != hc->R_nslab || h.N != 4 * hc->H ||
        h.M != hc->B || hc->cluster > 1 ||
        (const void*)hc->R != (const void*)h.C || h.c_slab != hc->R_slab || h.ldc != hc->ld_R)
        return -3;
    if (hc->ln_g == nullptr) return -3;   // LayerNorm cell only
    if (g_nstage != 3 || areg_on()) return -5;
    GemmGroup g{};
    g.n = n;
    g.start[0] = 0;
    for (int i = 0; i < n; ++i) {
        const GemmProblem& p = probs[i];
        if (p.M < 1 || p.M > BM || p.N % 64 != 0 || p.splits < 1 || p.K % p.splits != 0) return -2;
        if ((p.K / p.splits) % BK != 0 || p.lda % 8 != 0 || p.ldb % 8 != 0) return -3;
        if (((uintptr_t)p.A | (uintptr_t)p.Bt) & 15) return -4;
        g.p[i] = p;
        g.start[i + 1] = g.start[i] + (p.N / 64) * p.splits;
    }
    for (int i = n + 1; i <= kMaxGroup; ++i) g.start[i] = g.start[n];
    // the problem-0 workgroups wait for each other: they are dispatched first
    // and must all fit on the chip at once (one per CU is always possible)
    static int cus = 0;   // queried on the first (eager) call, before any graph capture
    if (cus == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return -8;
    }
    if (g.start[1] > cus) return -8;
    const size_t lds = (size_t)3 * (BM + 64) * BK * 2;
    if (hc->R_nslab == 9) {
        set_lds_attr(skinny_gemm_group_hyper_kernel<64, 3, 9>, lds);
        hipLaunchKernelGGL((skinny_gemm_group_hyper_kernel<64, 3, 9>), dim3(g.start[g.n]), dim3(256), lds, s, g, *hc,
                           counter, err);
    } else {
        set_lds_attr(skinny_gemm_group_hyper_kernel<64, 3, 4>, lds);
        hipLaunchKernelGGL((skinny_gemm_group_hyper_kernel<64, 3, 4>), dim3(g.start[g.n]), dim3(256), lds, s, g, *hc,
                           counter, err);
    }
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

// ---- fp8 v2 (inference): single product (optionally bf16 output) and grouped launch
struct GemmProblem8 {
    const void* A; int64_t lda;
    const void* Bt; int64_t ldb;
    const float* b_scale; float a_scale;
    float* C; int64_t ldc; int64_t c_slab;
    int M, N, K, splits;
};

namespace {
struct GemmGroup8 {
    GemmProblem8 p[kMaxGroup];
    int start[kMaxGroup + 1];
    int n;
};

template <int BN, int NS>
__global__ __launch_bounds__(256) void skinny_gemm_group_fp8_kernel(const GemmGroup8 g) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem8[];
    const int id = blockIdx.x;
    int q = 0;
#pragma unroll
    for (int i = 1; i < kMaxGroup; ++i) q += (i < g.n && id >= g.start[i]) ? 1 : 0;
    const GemmProblem8& p = g.p[q];
    const int local = id - g.start[q];
    const int ntiles = p.N / BN;
    const int split = local / ntiles, nt = local - split * ntiles;
    const int kslice = p.K / p.splits;
    glds_tile_fp8<BN, NS, false>((const uint8_t*)p.A, p.lda, (const uint8_t*)p.Bt, p.ldb, p.b_scale, p.a_scale,
                                 p.C + split * p.c_slab, p.ldc, p.M, nt * BN, (int64_t)split * kslice, kslice, smem8);
}

constexpr int kNs8 = 3;

template <typename K>
void lds_attr_once(K kern, size_t lds) {
    static bool done = false;
    if (!done) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        done = true;
    }
}

int check8(const GemmProblem8& p) {
    if (p.M < 1 || p.M > BM || p.N % 64 != 0 || p.splits < 1 || p.K % p.splits != 0) return -2;
    if ((p.K / p.splits) % BK8 != 0 || p.lda % 16 != 0 || p.ldb % 16 != 0) return -3;
    if (((uintptr_t)p.A | (uintptr_t)p.Bt) & 15) return -4;
    return 0;
}
}  // namespace

// C[s] = a_scale * b_scale[n] * A8[:, ks] . Bt8[:, ks]^T (fp32 slabs), or with
// cbf16 one bf16 output (splits must be 1). 64-wide N tiles, 3-deep ring.
SKR_API int skr_skinny_gemm_fp8_v2(const GemmProblem8* p, int cbf16, hipStream_t s) {
    int rc = check8(*p);
    if (rc) return rc;
    if (cbf16 && p->splits != 1) return -2;
    const dim3 grid(p->N / 64, p->splits);
    const size_t lds = (size_t)kNs8 * (BM + 64) * BK8;
    const int kslice = p->K / p->splits;
    if (cbf16) {
        auto k = skinny_gemm_fp8v2_kernel<64, kNs8, true>;
        lds_attr_once(k, lds);
        hipLaunchKernelGGL(k, grid, dim3(256), lds, s, (const uint8_t*)p->A, p->lda, (const uint8_t*)p->Bt, p->ldb,
                           p->b_scale, p->a_scale, (void*)p->C, p->ldc, p->c_slab, p->M, kslice);
    } else {
        auto k = skinny_gemm_fp8v2_kernel<64, kNs8, false>;
        lds_attr_once(k, lds);
        hipLaunchKernelGGL(k, grid, dim3(256), lds, s, (const uint8_t*)p->A, p->lda, (const uint8_t*)p->Bt, p->ldb,
                           p->b_scale, p->a_scale, (void*)p->C, p->ldc, p->c_slab, p->M, kslice);
    }
    return SKR_CHECK_LAUNCH();
}

SKR_API int skr_skinny_gemm_group_fp8(const GemmProblem8* probs, int n, hipStream_t s) {
    if (n < 1 || n > kMaxGroup) return -2;
    GemmGroup8 g{};
    g.n = n;
    g.start[0] = 0;
    for (int i = 0; i < n; ++i) {
        const int rc = check8(probs[i]);
        if (rc) return rc;
        g.p[i] = probs[i];
        g.start[i + 1] = g.start[i] + (probs[i].N / 64) * probs[i].splits;
    }
    for (int i = n + 1; i <= kMaxGroup; ++i) g.start[i] = g.start[n];
    const size_t lds = (size_t)kNs8 * (BM + 64) * BK8;
    auto k = skinny_gemm_group_fp8_kernel<64, kNs8>;
    lds_attr_once(k, lds);
    hipLaunchKernelGGL(k, dim3(g.start[n]), dim3(256), lds, s, g);
    return SKR_CHECK_LAUNCH();
}

SKR_API int skr_gemm_problem8_size() { return (int)sizeof(GemmProblem8); }

// fp8 e4m3 operands (bytes): C[z][s] = a_scale * b_scale[n] * A8[z][:, ks] . Bt8[z][:, ks]^T.
// Requirements as skr_skinny_gemm_v2 with kslice % 128 == 0 and 16-byte aligned rows.
SKR_API int skr_skinny_gemm_fp8(const void* A, int64_t lda, int64_t a_batch, const void* Bt, int64_t ldb,
                                int64_t b_batch, const float* b_scale, int64_t bs_batch, float a_scale, float* C,
                                int64_t ldc, int64_t c_slab, int64_t c_batch, int M, int N, int K, int splits,
                                int batch, int bn, hipStream_t s) {
    if (bn == 0) bn = (N % 128 == 0 && (N / 128) * splits * batch >= 144) ? 128 : 64;
    if (M < 1 || M > BM || (bn != 64 && bn != 128) || N % bn != 0 || splits < 1 || K % splits != 0) return -2;
    const int kslice = K / splits;
    if (kslice % BK8 != 0 || lda % 16 != 0 || ldb % 16 != 0) return -3;
    if (((uintptr_t)A | (uintptr_t)Bt) & 15) return -4;
    const dim3 grid(N / bn, splits, batch);
    const size_t lds = (size_t)NSTAGE * (BM + bn) * BK8;
    if (bn == 128) {
        static bool attr = false;
        if (!attr) {
            (void)hipFuncSetAttribute((const void*)skinny_gemm_fp8_kernel<128>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            attr = true;
        }
        hipLaunchKernelGGL(skinny_gemm_fp8_kernel<128>, grid, dim3(256), lds, s, (const uint8_t*)A, lda, a_batch,
                           (const uint8_t*)Bt, ldb, b_batch, b_scale, bs_batch, a_scale, C, ldc, c_slab, c_batch,
                           M, kslice);
    } else {
        static bool attr = false;
        if (!attr) {
            (void)hipFuncSetAttribute((const void*)skinny_gemm_fp8_kernel<64>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            attr = true;
        }
        hipLaunchKernelGGL(skinny_gemm_fp8_kernel<64>, grid, dim3(256), lds, s, (const uint8_t*)A, lda, a_batch,
                           (const uint8_t*)Bt, ldb, b_batch, b_scale, bs_batch, a_scale, C, ldc, c_slab, c_batch,
                           M, kslice);
    }
    return SKR_CHECK_LAUNCH();
}
