// Small fp32 GEMMs of the VAE's per-sequence layers: the latent heads
// (mu / presig = h W + b), the decoder's initial state (z W_init + b), the
// z part of the decoder input projections (z W_x[z rows]) and their
// gradients. Every one has a batch-sized dimension (B = 100) and another of
// at most a few thousand: 0.1-100 MFLOP each, too small for MFMA tiling to
// matter and too odd-shaped (K = 100 contractions, transposed operands) for
// the skinny / wgrad kernels. One generic kernel with arbitrary operand
// strides (so transposes are views, never copies) and a deterministic
// split-K (fixed-order two-pass sum) replaces the ~15 library GEMM calls
// per vae_large training step.
//
//   C[m, n] = (acc ? C[m, n] : 0) + bias[n] + sum_k A[m*sam + k*sak] * B[k*sbk + n*sbn]
//
// Tile: 64 x 64 outputs per workgroup (256 threads, a 4 x 4 block each:
// rows 4 ty .., columns 4 tx .., one 16-byte LDS read per operand per k), K
// staged through LDS 32 at a time with the next chunk's global loads in
// flight (registers) during the current chunk's math.
// Split-K: S > 1 slices write fp32 partials to work[S][M][N]; a second
// launch sums them in slice order (+ bias, + C if acc).
#include "common.h"

namespace {

constexpr int TM = 64, TN = 64, TK = 32, NT = 256;

// One 64 x 64 output tile (bx, by) of split / batch bz (= bt * S + s).
__device__ __forceinline__ void small_gemm_tile(const float* __restrict__ A, int64_t sam, int64_t sak,
                                                const float* __restrict__ B, int64_t sbk, int64_t sbn,
                                                float* __restrict__ C, int64_t ldc, const float* __restrict__ bias,
                                                int M, int N, int K, int kslice, int acc, float* __restrict__ work,
                                                int S, int64_t a_batch, int64_t b_batch, int64_t c_batch, int bx, int by,
                                                int bz) {
    // LDS rows padded to 68 floats: 16-byte aligned, so a thread's 4 rows /
    // 4 columns are one ds_read_b128 each
    __shared__ __attribute__((aligned(16))) float As[TK][TM + 4];
    __shared__ __attribute__((aligned(16))) float Bs[TK][TN + 4];
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    const int m0 = by * TM, n0 = bx * TN, s = bz % S, bt = bz / S;
    A += bt * a_batch;
    B += bt * b_batch;
    C += bt * c_batch;
    if (work != nullptr) work += (int64_t)bt * S * M * N;
    const int k0 = s * kslice, k1 = min(K, k0 + kslice);
    float c[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) c[i][j] = 0.f;
    // loader mapping: 256 threads x 8 elements per operand tile; the fastest
    // thread index runs along the operand's unit-stride axis when it has one
    const bool a_krow = sak == 1;   // A rows are K-contiguous
    const bool b_ncol = sbn == 1;   // B rows are N-contiguous
    float ra[8], rb[8];
    auto load = [&](int kb) {   // next K chunk into registers (in flight during the current chunk's math)
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const int e = tid + r * NT;   // 0 .. 2047
            const int mm = a_krow ? e / TK : e % TM, kk = a_krow ? e % TK : e / TM;
            const int gm = m0 + mm, gk = kb + kk;
            ra[r] = (gm < M && gk < k1) ? A[gm * sam + gk * sak] : 0.f;
            const int nn = b_ncol ? e % TN : e / TK, kq = b_ncol ? e / TN : e % TK;
            const int gn = n0 + nn, gq = kb + kq;
            rb[r] = (gn < N && gq < k1) ? B[gq * sbk + gn * sbn] : 0.f;
        }
    };
    auto stash = [&]() {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const int e = tid + r * NT;
            const int mm = a_krow ? e / TK : e % TM, kk = a_krow ? e % TK : e / TM;
            As[kk][mm] = ra[r];
            const int nn = b_ncol ? e % TN : e / TK, kq = b_ncol ? e / TN : e % TK;
            Bs[kq][nn] = rb[r];
        }
    };
    if (k0 < k1) load(k0);
    for (int kb = k0; kb < k1; kb += TK) {
        stash();
        __syncthreads();
        if (kb + TK < k1) load(kb + TK);
#pragma unroll 8
        for (int kk = 0; kk < TK; ++kk) {
            const float4 a4 = *(const float4*)&As[kk][4 * ty];
            const float4 b4 = *(const float4*)&Bs[kk][4 * tx];
            const float a[4] = {a4.x, a4.y, a4.z, a4.w}, b[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) c[i][j] += a[i] * b[j];
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + 4 * ty + i;
        if (m >= M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + 4 * tx + j;
            if (n >= N) continue;
            if (work != nullptr) {
                work[((int64_t)s * M + m) * N + n] = c[i][j];
            } else {
                float v = c[i][j] + (bias ? bias[n] : 0.f);
                if (acc) v += C[m * ldc + n];
                C[m * ldc + n] = v;
            }
        }
    }
}

__global__ __launch_bounds__(NT) void small_gemm_kernel(const float* __restrict__ A, int64_t sam, int64_t sak,
                                                        const float* __restrict__ B, int64_t sbk, int64_t sbn,
                                                        float* __restrict__ C, int64_t ldc, const float* __restrict__ bias,
                                                        int M, int N, int K, int kslice, int acc,
                                                        float* __restrict__ work, int S, int64_t a_batch,
                                                        int64_t b_batch, int64_t c_batch) {
    small_gemm_tile(A, sam, sak, B, sbk, sbn, C, ldc, bias, M, N, K, kslice, acc, work, S, a_batch, b_batch, c_batch,
                    blockIdx.x, blockIdx.y, blockIdx.z);
}

__device__ __forceinline__ void small_gemm_sum(const float* __restrict__ work, int S, int M, int N,
                                               float* __restrict__ C, int64_t ldc, const float* __restrict__ bias,
                                               int acc, int64_t c_batch, int64_t i, int bt) {
    if (i >= (int64_t)M * N) return;
    work += (int64_t)bt * S * M * N;
    C += bt * c_batch;
    const int m = (int)(i / N), n = (int)(i - (int64_t)m * N);
    float v = 0.f;
    for (int s = 0; s < S; ++s) v += work[(int64_t)s * M * N + i];
    v += bias ? bias[n] : 0.f;
    if (acc) v += C[m * ldc + n];
    C[m * ldc + n] = v;
}

__global__ void small_gemm_reduce(const float* __restrict__ work, int S, int M, int N, float* __restrict__ C,
                                  int64_t ldc, const float* __restrict__ bias, int acc, int64_t c_batch) {
    small_gemm_sum(work, S, M, N, C, ldc, bias, acc, c_batch, (int64_t)blockIdx.x * blockDim.x + threadIdx.x,
                   blockIdx.y);
}

}  // namespace

// Split-K factor the launcher uses for an (M, N, K) problem (the Python side
// sizes the workspace with it): ~256 workgroups, K slices of >= 64.
SKR_API int skr_small_gemm_splits(int M, int N, int K) {
    if (M <= 0 || N <= 0 || K <= 0) return 1;
    const int tiles = ((M + TM - 1) / TM) * ((N + TN - 1) / TN);
    int S = 256 / tiles;
    S = S < 1 ? 1 : S;
    const int maxS = (K + 63) / 64;
    return S < maxS ? S : maxS;
}

// nbatch independent problems of the same shape: operand / output bases
// advance by a_batch / b_batch / c_batch elements (a shared bias); workspace
// nbatch * S * M * N floats when S > 1.
SKR_API int skr_small_gemm_batched(const float* A, int64_t a_batch, int64_t sam, int64_t sak, const float* B,
                                   int64_t b_batch, int64_t sbk, int64_t sbn, float* C, int64_t c_batch, int64_t ldc,
                                   const float* bias, int M, int N, int K, int acc, int nbatch, float* work,
                                   int64_t work_elems, hipStream_t s) {
    if (M <= 0 || N <= 0 || nbatch <= 0) return 0;
    if (K <= 0) return -2;
    int S = skr_small_gemm_splits(M, N, K);
    int kslice = (K + S - 1) / S;
    kslice = (kslice + TK - 1) / TK * TK;
    S = (K + kslice - 1) / kslice;
    if (S > 1 && (work == nullptr || work_elems < (int64_t)nbatch * S * M * N)) return -3;
    const dim3 grid((N + TN - 1) / TN, (M + TM - 1) / TM, S * nbatch);
    hipLaunchKernelGGL(small_gemm_kernel, grid, dim3(NT), 0, s, A, sam, sak, B, sbk, sbn, C, ldc, bias, M, N, K,
                       kslice, acc, S > 1 ? work : nullptr, S, a_batch, b_batch, c_batch);
    if (S > 1) {
        const int64_t n = (int64_t)M * N;
        hipLaunchKernelGGL(small_gemm_reduce, dim3((unsigned)((n + 255) / 256), nbatch), dim3(256), 0, s, work, S,
                           M, N, C, ldc, bias, acc, c_batch);
    }
    return SKR_CHECK_LAUNCH();
}

SKR_API int skr_small_gemm(const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk, int64_t sbn,
                           float* C, int64_t ldc, const float* bias, int M, int N, int K, int acc, float* work,
                           int64_t work_elems, hipStream_t s) {
    return skr_small_gemm_batched(A, 0, sam, sak, B, 0, sbk, sbn, C, 0, ldc, bias, M, N, K, acc, 1, work, work_elems,
                                  s);
}

// ---- grouped launch -----------------------------------------------------------------
// Up to kSgMax independent small products (each with its own shape, strides,
// batch count and split factor -- the same tiles and the same split-K
// summation order as skr_small_gemm_batched, so the results are identical)
// in ONE launch, plus one launch summing the split-K partials of those that
// split: the latent-node and hyper-projection gradients are groups of 2-4
// such products per phase, each otherwise a launch (+ a reduce launch) of
// its own.
struct SgProb {
    const float* A; int64_t sam, sak, a_batch;
    const float* B; int64_t sbk, sbn, b_batch;
    float* C; int64_t ldc, c_batch;
    const float* bias;
    int M, N, K, acc, nbatch;
    float* work; int64_t work_elems;
};
constexpr int kSgMax = 6;

namespace {
struct SgPlan {
    SgProb p[kSgMax];
    int S[kSgMax], kslice[kSgMax];
    int n;
    int start[kSgMax + 1];     // tile workgroups: prefix of ntn * ntm * S * nbatch
    int rstart[kSgMax + 1];    // reduce workgroups: prefix of ceil(M N / 256) * nbatch (S > 1 only)
};

__global__ __launch_bounds__(NT) void small_gemm_group_kernel(const SgPlan g) {
    int q = 0;
    while (q + 1 < g.n && (int)blockIdx.x >= g.start[q + 1]) ++q;
    const SgProb& P = g.p[q];
    const int ntn = (P.N + TN - 1) / TN, ntm = (P.M + TM - 1) / TM;
    const int local = blockIdx.x - g.start[q];
    const int bz = local / (ntn * ntm), rem = local - bz * ntn * ntm;
    small_gemm_tile(P.A, P.sam, P.sak, P.B, P.sbk, P.sbn, P.C, P.ldc, P.bias, P.M, P.N, P.K, g.kslice[q], P.acc,
                    g.S[q] > 1 ? P.work : nullptr, g.S[q], P.a_batch, P.b_batch, P.c_batch, rem % ntn, rem / ntn, bz);
}

__global__ __launch_bounds__(256) void small_gemm_group_reduce(const SgPlan g) {
    int q = 0;
    while (q + 1 < g.n && (int)blockIdx.x >= g.rstart[q + 1]) ++q;
    const SgProb& P = g.p[q];
    const int per = (int)(((int64_t)P.M * P.N + 255) / 256);
    const int local = blockIdx.x - g.rstart[q];
    const int bt = local / per;
    small_gemm_sum(P.work, g.S[q], P.M, P.N, P.C, P.ldc, P.bias, P.acc, P.c_batch,
                   (int64_t)(local - bt * per) * 256 + threadIdx.x, bt);
}
}  // namespace

SKR_API int skr_small_gemm_group(const SgProb* probs, int n, hipStream_t s) {
    if (n < 1 || n > kSgMax) return -2;
    SgPlan g{};
    g.n = n;
    for (int q = 0; q < n; ++q) {
        const SgProb& P = probs[q];
        if (P.M <= 0 || P.N <= 0 || P.nbatch <= 0 || P.K <= 0) return -2;
        int S = skr_small_gemm_splits(P.M, P.N, P.K);
        int kslice = (P.K + S - 1) / S;
        kslice = (kslice + TK - 1) / TK * TK;
        S = (P.K + kslice - 1) / kslice;
        if (S > 1 && (P.work == nullptr || P.work_elems < (int64_t)P.nbatch * S * P.M * P.N)) return -3;
        g.p[q] = P;
        g.S[q] = S;
        g.kslice[q] = kslice;
        g.start[q + 1] = g.start[q] + ((P.N + TN - 1) / TN) * ((P.M + TM - 1) / TM) * S * P.nbatch;
        g.rstart[q + 1] = g.rstart[q] + (S > 1 ? (int)(((int64_t)P.M * P.N + 255) / 256) * P.nbatch : 0);
    }
    for (int q = n + 1; q <= kSgMax; ++q) g.start[q] = g.start[n], g.rstart[q] = g.rstart[n];
    hipLaunchKernelGGL(small_gemm_group_kernel, dim3(g.start[n]), dim3(NT), 0, s, g);
    if (g.rstart[n] > 0) hipLaunchKernelGGL(small_gemm_group_reduce, dim3(g.rstart[n]), dim3(256), 0, s, g);
    return SKR_CHECK_LAUNCH();
}

SKR_API int skr_small_gemm_prob_size() { return (int)sizeof(SgProb); }
