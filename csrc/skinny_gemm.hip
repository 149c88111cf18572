// Skinny split-K GEMM for the recurrent steps: C_s = A[:, Ks] . Bt[:, Ks]^T
//
// Every per-time-step product in the RNN is "few rows, long K or wide N":
// M = batch (<= 128), N in {256 .. 24576}, K in {256 .. 24576}. Library
// kernels tile these for square problems and leave most of the 256 CUs idle
// (e.g. [100 x 24576] x [24576 x 256] ran as 28 workgroups). This kernel
// always covers all M rows in one 128-row tile, tiles N by 64 and splits K
// over gridDim.y so that (N/64) * S ~ 1-2 workgroups per CU. Each split
// writes its own fp32 partial slab; the CONSUMER (the fused cell kernel of
// csrc/lstm_cell.hip) sums the S slabs while loading -- the reduction costs
// no extra launch and no atomics, and the result is deterministic.
//
// Both operands are K-contiguous ("NT"): A [M, K] row-major, Bt [N, K]
// row-major (weights are kept in bf16 in both orientations), so MFMA
// fragments are 16-byte vector reads. MFMA: v_mfma_f32_16x16x32_bf16; lane l
// holds A[row l&15][k 8(l>>4) .. +7] and B[k 8(l>>4) .. +7][col l&15];
// C/D: col = l&15, row = 4(l>>4) + i.
//
// Block: 256 threads (4 waves); wave w owns rows 32w..32w+31 x all 64 cols
// (2 x 4 accumulator tiles). K tile 64, double-buffered LDS with register
// prefetch of the next tile; rows padded by 16 B against bank conflicts.
// gridDim.z batches independent problems (both encoder directions).
#include "common.h"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int BM = 128, BN = 64, BK = 64, PAD = 8, LDK = BK + PAD;  // LDS row = 144 B

__global__ __launch_bounds__(256) void skinny_gemm_nt_kernel(
    const __hip_bfloat16* __restrict__ A, int64_t lda, int64_t a_batch,
    const __hip_bfloat16* __restrict__ Bt, int64_t ldb, int64_t b_batch,
    float* __restrict__ C, int64_t ldc, int64_t c_slab, int64_t c_batch, int M, int kslice) {
    __shared__ __attribute__((aligned(16))) __hip_bfloat16 As[2][BM * LDK];
    __shared__ __attribute__((aligned(16))) __hip_bfloat16 Bs[2][BN * LDK];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int n0 = blockIdx.x * BN;
    const int64_t k0 = (int64_t)blockIdx.y * kslice;
    const int ntiles = kslice / BK;
    A += blockIdx.z * a_batch;
    Bt += blockIdx.z * b_batch;
    C += blockIdx.z * c_batch + blockIdx.y * c_slab;

    uint4 ra[4], rb[2];
    auto load = [&](int kt) {
        const int64_t kb = k0 + (int64_t)kt * BK;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int c = tid + i * 256, row = c >> 3, kc = (c & 7) * 8;
            ra[i] = row < M ? *(const uint4*)(A + row * lda + kb + kc) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int c = tid + i * 256, col = c >> 3, kc = (c & 7) * 8;
            rb[i] = *(const uint4*)(Bt + (int64_t)(n0 + col) * ldb + kb + kc);
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int c = tid + i * 256, row = c >> 3, kc = (c & 7) * 8;
            *(uint4*)(&As[buf][row * LDK + kc]) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int c = tid + i * 256, col = c >> 3, kc = (c & 7) * 8;
            *(uint4*)(&Bs[buf][col * LDK + kc]) = rb[i];
        }
    };

    f32x4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    load(0);
    store(0);
    __syncthreads();
    const int fr = lane & 15, fk = (lane >> 4) * 8;
    for (int kt = 0; kt < ntiles; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < ntiles) load(kt + 1);
#pragma unroll
        for (int ks = 0; ks < BK; ks += 32) {
            bf16x8 af[2], bfr[4];
#pragma unroll
            for (int i = 0; i < 2; ++i)
                af[i] = *(const bf16x8*)(&As[buf][(32 * w + 16 * i + fr) * LDK + ks + fk]);
#pragma unroll
            for (int j = 0; j < 4; ++j) bfr[j] = *(const bf16x8*)(&Bs[buf][(16 * j + fr) * LDK + ks + fk]);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
        if (kt + 1 < ntiles) store(buf ^ 1);
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = 32 * w + 16 * i + (lane >> 4) * 4 + e;
                if (row < M) C[row * ldc + n0 + 16 * j + fr] = acc[i][j][e];
            }
}

}  // namespace

// C[z][s] (slab s of batch z) = A[z][:, s*kslice:(s+1)*kslice] . Bt[z][:, same]^T
// Requirements: M <= 128, N % 64 == 0, kslice % 64 == 0, splits * kslice == K,
// 16-byte aligned rows (lda, ldb multiples of 8 elements).
SKR_API int skr_skinny_gemm(const void* A, int64_t lda, int64_t a_batch, const void* Bt, int64_t ldb,
                            int64_t b_batch, float* C, int64_t ldc, int64_t c_slab, int64_t c_batch, int M, int N,
                            int K, int splits, int batch, hipStream_t s) {
    if (M < 1 || M > BM || N % BN != 0 || splits < 1 || K % splits != 0) return -2;
    const int kslice = K / splits;
    if (kslice % BK != 0 || lda % 8 != 0 || ldb % 8 != 0) return -3;
    if (((uintptr_t)A | (uintptr_t)Bt) & 15) return -4;
    hipLaunchKernelGGL(skinny_gemm_nt_kernel, dim3(N / BN, splits, batch), dim3(256), 0, s,
                       (const __hip_bfloat16*)A, lda, a_batch, (const __hip_bfloat16*)Bt, ldb, b_batch, C, ldc,
                       c_slab, c_batch, M, kslice);
    return SKR_CHECK_LAUNCH();
}
