// MX-fp8 GEMM for the decode step's h W_h product (BASELINE config 5: fp8
// gate GEMM, dec = 2048, sampling under a HIP graph; reference per-stroke
// step /root/reference/model.py:213-249).
//
//   C[M, N] (fp32) = (A8 (.) SA)[M, K] . ((W8 (.) SW)[N, K])^T
//
// Both operands are OCP e4m3 with one E8M0 scale per 32 consecutive k of a
// row (the OCP MX block): W8 / SW are quantized once per weight version
// (skr_mx8_quant_t, from the fp32 [K, N] weight), A8 / SA by the PRODUCER --
// the decode main cell writes h in this form beside its bf16 copy
// (csrc/cell_fwd_body.h, FwdArgs::h_q8), so the GEMM itself does no
// conversion work. gfx950's block-scaled v_mfma_scale_f32_16x16x128_f8f6f4
// applies both scales in hardware at twice the bf16 MFMA rate.
//
// Scale layout [rows][4][K/128] ("j-major"): block b = k / 32 of row r sits
// at r * K/32 + (b % 4) * K/128 + b / 4, so MFMA lane (r, j = lane >> 4) finds
// the scales of ALL its K-steps in K/128 consecutive bytes -- one 16-byte
// load per fragment for K <= 2048.
//
// Tile 256 x 128 x K, 512 threads (8 waves, 4 x 2, each 64 x 64 = 4 x 4 MFMA
// tiles), K-steps of 128 through a 3-stage LDS-DMA ring, two K-steps in
// flight behind counted vmcnt waits (global_load_lds
// 16 B per lane, 128-byte LDS rows with the 16-byte chunk index XOR
// (row >> 1) & 7 applied on the global address, like csrc/glds_mma.h):
// 144 KB of LDS, one 8-wave workgroup per CU. MFMA operands (measured,
// scripts/micro/mx8_diag.py): lane l holds row / column l & 15, bytes 0-15 =
// k [16 g, +16) and bytes 16-31 = k [64 + 16 g, +16) of the K-step, g = l >> 4,
// and its scale operand applies to k [32 g, +32) -- so 32-k block g of a
// row is scaled by lane group g's byte (a contiguous 32-byte fragment is
// exact with unit scales but scales the wrong k: profiles/r6/mx8_diag.jsonl).
// C/D: col = l & 15, rows 4 (l >> 4) + i. Tile order is XCD-aware: the 8 row
// blocks that read one W column band share an XCD's L2.
#include "common.h"


namespace {

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int TM = 256, TN = 128, TK = 128, NT = 512, NSTG = 3;
constexpr int STG = (TM + TN) * TK;          // bytes per stage
constexpr int GPW = (TM + TN) / 8 / 8;       // 1-KiB DMA pieces per wave per stage (6)

__device__ __forceinline__ int scale_off(int r, int b, int K) { return r * (K / 32) + (b & 3) * (K / 128) + (b >> 2); }

// E8M0 exponent X of a block with absolute maximum amax: amax / 2^(X - 127)
// lands in [128, 256), inside e4m3's 448 range (X clamped to [0, 254]).
__device__ __forceinline__ int e8m0_of(float amax) {
    const int e = (int)((__float_as_uint(amax) >> 23) & 0xff);
    return min(max(e - 7, 0), 254);
}
__device__ __forceinline__ float inv_scale(int X) { return __uint_as_float((uint32_t)(254 - X) << 23); }   // 2^(127 - X)

__device__ __forceinline__ uint32_t pack4_fp8(float a, float b, float c, float d) {
    int v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
    return (uint32_t)v;
}

// W [K, N] fp32 (row stride ldw) -> Q [N, K] e4m3 + S [N][4][K/128]: one
// thread per (n, 32-k block); adjacent threads read adjacent n (coalesced).
__global__ __launch_bounds__(256) void mx8_quant_t_kernel(const float* __restrict__ W, int64_t ldw, int K, int N,
                                                          uint8_t* __restrict__ Q, uint8_t* __restrict__ S) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)N * (K / 32)) return;
    const int n = (int)(i % N), b = (int)(i / N);
    float v[32], amax = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        v[k] = W[(int64_t)(32 * b + k) * ldw + n];
        amax = fmaxf(amax, fabsf(v[k]));
    }
    const int X = e8m0_of(amax);
    const float s = inv_scale(X);
    u32x4 o[2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const int k = 16 * h + 4 * w;
            o[h][w] = pack4_fp8(v[k] * s, v[k + 1] * s, v[k + 2] * s, v[k + 3] * s);
        }
    u32x4* q = (u32x4*)(Q + (int64_t)n * K + 32 * b);
    q[0] = o[0];
    q[1] = o[1];
    S[scale_off(n, b, K)] = (uint8_t)X;
}

// rows of A [M, K] (bf16 or fp32, row stride lda) -> Q [M, K] + S [M][4][K/128]
__global__ __launch_bounds__(256) void mx8_quant_rows_kernel(const void* __restrict__ A, int64_t lda, int bf16, int M,
                                                             int K, uint8_t* __restrict__ Q, int64_t ldq,
                                                             uint8_t* __restrict__ S) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)M * (K / 32)) return;
    const int b = (int)(i % (K / 32)), r = (int)(i / (K / 32));
    float v[32], amax = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        const int64_t o = (int64_t)r * lda + 32 * b + k;
        v[k] = bf16 ? __bfloat162float(((const __hip_bfloat16*)A)[o]) : ((const float*)A)[o];
        amax = fmaxf(amax, fabsf(v[k]));
    }
    const int X = e8m0_of(amax);
    const float s = inv_scale(X);
    u32x4* q = (u32x4*)(Q + (int64_t)r * ldq + 32 * b);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        u32x4 o;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const int k = 16 * h + 4 * w;
            o[w] = pack4_fp8(v[k] * s, v[k + 1] * s, v[k + 2] * s, v[k + 3] * s);
        }
        q[h] = o;
    }
    S[scale_off(r, b, K)] = (uint8_t)X;
}

// MFMA operand of one row (A) / column (W) for lane group fq = lane >> 4.
// LAYOUT 1: the 32 bytes are k [16 fq, +16) and [64 + 16 fq, +16) of the
// K-step (16-byte chunks fq and 4 + fq); LAYOUT 0: k [32 fq, +32).
template <int LAYOUT>
__device__ __forceinline__ i32x8 frag(const uint8_t* S, int row) {
    const int fq = (threadIdx.x & 63) >> 4, sw = (row >> 1) & 7;
    const int c0 = LAYOUT ? fq : 2 * fq, c1 = LAYOUT ? 4 + fq : 2 * fq + 1;
    const int4 lo = *(const int4*)(&S[row * TK + ((c0 ^ sw) * 16)]);
    const int4 hi = *(const int4*)(&S[row * TK + ((c1 ^ sw) * 16)]);
    return i32x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
}

__device__ __forceinline__ f32x4 mma(i32x8 a, i32x8 b, f32x4 c, int sa, int sb) {
    // formats 0 / 0: e4m3 x e4m3; byte 0 of each scale operand is this lane's block scale
    return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa, 0, sb);
}

// byte kt of a lane's 16 scale bytes (one per K-step), as the low byte
__device__ __forceinline__ int scale_byte(const u32x4& v, int kt) {
    const int q = kt >> 2;
    const uint32_t w = q == 0 ? v[0] : q == 1 ? v[1] : q == 2 ? v[2] : v[3];
    return (int)(w >> (8 * (kt & 3)));
}

template <int LAYOUT>
__global__ __launch_bounds__(NT) void mx8_gemm_kernel(const uint8_t* __restrict__ A8, int64_t lda,
                                                         const uint8_t* __restrict__ SA,
                                                         const uint8_t* __restrict__ W8, int64_t ldw,
                                                         const uint8_t* __restrict__ SW, float* __restrict__ C,
                                                         int64_t ldc, int M, int N, int K, int per_xcd) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int mb = (M + TM - 1) / TM;
    const int lin = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
    if (lin >= mb * (N / TN)) return;
    const int m0 = (lin % mb) * TM, n0 = (lin / mb) * TN;     // the row blocks of one column band: consecutive
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w >> 1, wn = w & 1, fr = lane & 15, fq = lane >> 4;   // wave: rows 64 wm.., columns 64 wn..
    const int nk = K / TK;

    // ---- DMA sources: wave w moves 1-KiB pieces w, w + 8, ... (8 rows x 128 B each): A rows, then W rows
    constexpr int APC = TM / 8;                                // A pieces per stage
    const int r8 = lane >> 3, slot = lane & 7;
    const uint8_t* src[GPW];
#pragma unroll
    for (int i = 0; i < GPW; ++i) {
        const int piece = w + 8 * i;
        const int row = (piece < APC ? piece : piece - APC) * 8 + r8;
        const int c = slot ^ ((row >> 1) & 7);
        src[i] = piece < APC ? A8 + (int64_t)min(m0 + row, M - 1) * lda + 16 * c
                             : W8 + (int64_t)(n0 + row) * ldw + 16 * c;
    }
    auto issue = [&](int kt) {
        uint8_t* st = smem + (kt % NSTG) * STG;
#pragma unroll
        for (int i = 0; i < GPW; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(src[i] + (int64_t)kt * TK),
                                             (__attribute__((address_space(3))) void*)(st + (w + 8 * i) * 1024), 16, 0, 0);
    };
    // ---- this lane's block scales for every K-step: K / 128 bytes per fragment (K <= 2048)
    u32x4 sa[4], sb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = min(m0 + 64 * wm + 16 * i + fr, M - 1);
        const uint32_t* pa = (const uint32_t*)(SA + (int64_t)r * (K / 32) + fq * (K / 128));
        const int c = n0 + 64 * wn + 16 * i + fr;
        const uint32_t* pb = (const uint32_t*)(SW + (int64_t)c * (K / 32) + fq * (K / 128));
#pragma unroll
        for (int q = 0; q < 4; ++q) {                          // K / 512 words: one per 4 K-steps
            sa[i][q] = q < K / 512 ? pa[q] : 0u;
            sb[i][q] = q < K / 512 ? pb[q] : 0u;
        }
    }
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int p = 0; p < NSTG - 1; ++p)
        if (p < nk) issue(p);
    for (int kt = 0; kt < nk; ++kt) {
        // stage kt landed for this wave: all but the (up to) NSTG - 2 younger
        // stages' DMAs are done (the scale loads above are older still)
        if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GPW) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();                       // ... for every wave; stage kt - 1 is free
        if (kt + NSTG - 1 < nk) issue(kt + NSTG - 1);
        const uint8_t* As = smem + (kt % NSTG) * STG;
        const uint8_t* Ws = As + TM * TK;
        i32x8 af[4];
        int a_s[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            af[i] = frag<LAYOUT>(As, 64 * wm + 16 * i + fr);
            a_s[i] = scale_byte(sa[i], kt);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {          // one W fragment live at a time
            const i32x8 bf = frag<LAYOUT>(Ws, 64 * wn + 16 * j + fr);
            const int b_s = scale_byte(sb[j], kt);
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[i][j] = mma(af[i], bf, acc[i][j], a_s[i], b_s);
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = m0 + 64 * wm + 16 * i + 4 * fq + e;
                if (row < M) C[(int64_t)row * ldc + n0 + 64 * wn + 16 * j + fr] = acc[i][j][e];
            }
}

}  // namespace

static int g_mx8_layout = 1;

// W [K, N] fp32 -> Q [N, K] e4m3 + S [N][4][K/128] (K % 128 == 0)
SKR_API int skr_mx8_quant_t(const float* W, int64_t ldw, int K, int N, void* Q, void* S, hipStream_t s) {
    if (K <= 0 || N <= 0 || K % 128 || ((uintptr_t)Q & 15)) return -2;
    const int64_t n = (int64_t)N * (K / 32);
    hipLaunchKernelGGL(mx8_quant_t_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, W, ldw, K, N,
                       (uint8_t*)Q, (uint8_t*)S);
    return SKR_CHECK_LAUNCH();
}

// rows of A [M, K] (bf16 if bf16 != 0, else fp32; row stride lda elements) ->
// Q [M, K] (row stride ldq bytes) + S [M][4][K/128]
SKR_API int skr_mx8_quant_rows(const void* A, int64_t lda, int bf16, int M, int K, void* Q, int64_t ldq, void* S,
                               hipStream_t s) {
    if (M <= 0 || K <= 0 || K % 128 || ldq % 16 || ((uintptr_t)Q & 15)) return -2;
    const int64_t n = (int64_t)M * (K / 32);
    hipLaunchKernelGGL(mx8_quant_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, A, lda, bf16, M, K,
                       (uint8_t*)Q, ldq, (uint8_t*)S);
    return SKR_CHECK_LAUNCH();
}

// C [M, N] fp32 (row stride ldc) = A8 [M, K] (lda bytes) x W8 [N, K]^T (ldw
// bytes) with MX scales SA [M][4][K/128], SW [N][4][K/128].
// N % 128 == 0, K % 512 == 0, K <= 2048, 16-byte aligned rows.
SKR_API int skr_mx8_gemm(const void* A8, int64_t lda, const void* SA, const void* W8, int64_t ldw, const void* SW,
                         float* C, int64_t ldc, int M, int N, int K, hipStream_t s) {
    if (M <= 0 || N % TN || K % 512 || K > 2048 || lda % 16 || ldw % 16) return -2;
    if (((uintptr_t)A8 | (uintptr_t)W8 | (uintptr_t)SA | (uintptr_t)SW) & 15) return -4;
    const int tiles = ((M + TM - 1) / TM) * (N / TN);
    const int per_xcd = (tiles + 7) / 8;
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute((const void*)mx8_gemm_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                NSTG * STG) != hipSuccess ||
            hipFuncSetAttribute((const void*)mx8_gemm_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                NSTG * STG) != hipSuccess)
            return -6;
        attr = true;
    }
    if (g_mx8_layout)
        hipLaunchKernelGGL(mx8_gemm_kernel<1>, dim3(8 * per_xcd), dim3(NT), NSTG * STG, s, (const uint8_t*)A8, lda,
                           (const uint8_t*)SA, (const uint8_t*)W8, ldw, (const uint8_t*)SW, C, ldc, M, N, K, per_xcd);
    else
        hipLaunchKernelGGL(mx8_gemm_kernel<0>, dim3(8 * per_xcd), dim3(NT), NSTG * STG, s, (const uint8_t*)A8, lda,
                           (const uint8_t*)SA, (const uint8_t*)W8, ldw, (const uint8_t*)SW, C, ldc, M, N, K, per_xcd);
    return SKR_CHECK_LAUNCH();
}

// Diagnostic hook: the operand byte layout of the MFMA fragments (see frag);
// returns the previous one.
SKR_API int skr_mx8_set_layout(int l) {
    const int prev = g_mx8_layout;
    if (l >= 0) g_mx8_layout = l;
    return prev;
}
