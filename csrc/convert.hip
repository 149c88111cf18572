// Per-step weight preparation: fp32 master weights -> the bf16 GEMM operands
// the recurrent kernels read, in BOTH layouts (W for the backward products
// dG @ W^T, W^T for the forward products h @ W: every skinny GEMM wants its
// B operand K-contiguous) in ONE pass over the fp32 tensor.
//
// The framework's first version did this with torch ops (cast, then
// .t().contiguous() of the bf16 copy): on MI355X the transposing copy of
// the 2048 x 8192 HyperLSTM W_h alone took ~48 us per step (strided reads),
// the cast another ~20. Here a 64 x 64 tile is read once with float4 loads
// (coalesced), written straight back as bf16 (8 bytes per thread), and
// transposed through LDS (65-float padded rows: conflict-free column reads)
// for a second set of coalesced 8-byte stores.
#include "common.h"

namespace {

constexpr int TS = 64;

__global__ __launch_bounds__(256) void cast_transpose_kernel(const float* __restrict__ src, int64_t ld_src,
                                                             int64_t sb_src, int R, int C,
                                                             __hip_bfloat16* __restrict__ dst, int64_t ld_dst,
                                                             int64_t sb_dst, __hip_bfloat16* __restrict__ dstT,
                                                             int64_t ld_dstT, int64_t sb_dstT) {
    __shared__ float tile[TS][TS + 1];
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    const int c0 = blockIdx.x * TS, r0 = blockIdx.y * TS, z = blockIdx.z;
    src += z * sb_src;
    // ---- read (and write the same-layout bf16 copy)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int rl = ty + 16 * i, r = r0 + rl, c = c0 + tx * 4;
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        if (r < R) {
            if (c + 3 < C) {
                const float4 q = *(const float4*)(src + (int64_t)r * ld_src + c);
                v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (c + j < C) v[j] = src[(int64_t)r * ld_src + c + j];
            }
            if (dst != nullptr) {
                __hip_bfloat16* d = dst + z * sb_dst + (int64_t)r * ld_dst + c;
                if (c + 3 < C) {
                    __hip_bfloat16 b[4] = {skr::to_bf16(v[0]), skr::to_bf16(v[1]), skr::to_bf16(v[2]),
                                           skr::to_bf16(v[3])};
                    *(uint2*)d = *(const uint2*)b;
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (c + j < C) d[j] = skr::to_bf16(v[j]);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) tile[rl][tx * 4 + j] = v[j];
    }
    if (dstT == nullptr) return;
    __syncthreads();
    // ---- transposed write: dstT[c][r], 4 consecutive r per thread
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int cl = ty + 16 * i, c = c0 + cl, r = r0 + tx * 4;
        if (c >= C) continue;
        __hip_bfloat16* d = dstT + z * sb_dstT + (int64_t)c * ld_dstT + r;
        if (r + 3 < R) {
            __hip_bfloat16 b[4] = {skr::to_bf16(tile[tx * 4 + 0][cl]), skr::to_bf16(tile[tx * 4 + 1][cl]),
                                   skr::to_bf16(tile[tx * 4 + 2][cl]), skr::to_bf16(tile[tx * 4 + 3][cl])};
            *(uint2*)d = *(const uint2*)b;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (r + j < R) d[j] = skr::to_bf16(tile[tx * 4 + j][cl]);
        }
    }
}

}  // namespace

// src fp32 [nb][R][C] (row stride ld_src, batch stride sb_src) -> dst bf16
// [nb][R][C] and/or dstT bf16 [nb][C][R] (either may be null). 8-byte stores
// need ld_dst, ld_dstT, sb_* and the base pointers 8-byte aligned in elements
// of 4 (checked); float4 loads need ld_src % 4 == 0 and a 16-byte aligned src.
SKR_API int skr_cast_transpose_bf16(const float* src, int64_t ld_src, int64_t sb_src, int R, int C, int nb,
                                    void* dst, int64_t ld_dst, int64_t sb_dst, void* dstT, int64_t ld_dstT,
                                    int64_t sb_dstT, hipStream_t s) {
    if (R <= 0 || C <= 0 || nb <= 0) return 0;
    if (ld_src % 4 || sb_src % 4 || ((uintptr_t)src & 15)) return -3;
    if (dst && (ld_dst % 4 || sb_dst % 4 || ((uintptr_t)dst & 7))) return -3;
    if (dstT && (ld_dstT % 4 || sb_dstT % 4 || ((uintptr_t)dstT & 7))) return -3;
    const dim3 grid((C + TS - 1) / TS, (R + TS - 1) / TS, nb);
    hipLaunchKernelGGL(cast_transpose_kernel, grid, dim3(256), 0, s, src, ld_src, sb_src, R, C,
                       (__hip_bfloat16*)dst, ld_dst, sb_dst, (__hip_bfloat16*)dstT, ld_dstT, sb_dstT);
    return SKR_CHECK_LAUNCH();
}
