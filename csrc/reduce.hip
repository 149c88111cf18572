// Column reductions over the [T*B, C] per-step saves, for the parameter
// gradients that are sums over every (time, row) position: LayerNorm gamma /
// beta (sum dy*xhat, sum dy), biases (sum dg). One pass reads X (and Y) once
// -- instead of an elementwise product materialised at full size and a
// second reduction kernel -- and handles a two-level row index (i < R1 with
// stride s1, j < R2 with stride s2) so per-direction groups of the
// bidirectional encoder ([T, nd, B, C] views) reduce without a copy.
//
// Grid (ceil(C/256), RS): thread = one column, block row RS_idx owns a slice
// of the R1*R2 rows; per-slice partial sums go to part[RS][C] (fp32),
// summed by a deterministic second pass. RS is chosen by the caller
// (ops/reduce.py): about 1024 / ceil(C/256) slices, capped at R/16 rows per
// slice -- e.g. the [30000, 123] MDN-head bias gradient runs RS = 1024
// slices of ~30 rows.
#include "common.h"

namespace {

template <bool XBF16>
__device__ __forceinline__ float ldx(const void* x, int64_t i) {
    if constexpr (XBF16) return __bfloat162float(((const __hip_bfloat16*)x)[i]);
    else return ((const float*)x)[i];
}

template <bool XBF16>
__global__ __launch_bounds__(256) void colsum_kernel(const void* __restrict__ X, const float* __restrict__ Y,
                                                     int64_t R1, int64_t s1, int64_t R2, int64_t s2, int C,
                                                     float* __restrict__ part_xy, float* __restrict__ part_x) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= C) return;
    const int64_t R = R1 * R2;
    const int64_t per = (R + gridDim.y - 1) / gridDim.y;
    const int64_t r0 = blockIdx.y * per, r1 = min(R, r0 + per);
    float sxy = 0.f, sx = 0.f;
    // walk (i, j) incrementally: no 64-bit division per element
    int64_t i = r0 / R2, j = r0 % R2;
    int64_t r = r0;
    for (; r + 4 <= r1; r += 4) {
        float xv[4], yv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t off = i * s1 + j * s2 + c;
            xv[k] = ldx<XBF16>(X, off);
            yv[k] = Y ? Y[off] : 0.f;
            if (++j == R2) {
                j = 0;
                ++i;
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            sx += xv[k];
            sxy += xv[k] * yv[k];
        }
    }
    for (; r < r1; ++r) {
        const int64_t off = i * s1 + j * s2 + c;
        const float xv = ldx<XBF16>(X, off);
        sx += xv;
        if (Y) sxy += xv * Y[off];
        if (++j == R2) {
            j = 0;
            ++i;
        }
    }
    part_x[(int64_t)blockIdx.y * C + c] = sx;
    if (Y) part_xy[(int64_t)blockIdx.y * C + c] = sxy;
}

}  // namespace

// x_kind: 1 bf16, 2 fp32. Y (fp32, same strides) may be null (then part_xy unused).
SKR_API int skr_colsum(const void* X, int x_kind, const float* Y, int64_t R1, int64_t s1, int64_t R2, int64_t s2,
                       int C, int RS, float* part_xy, float* part_x, hipStream_t s) {
    if (C <= 0 || RS <= 0 || R1 * R2 <= 0) return -2;
    const dim3 grid((C + 255) / 256, RS);
    if (x_kind == 1)
        hipLaunchKernelGGL(colsum_kernel<true>, grid, dim3(256), 0, s, X, Y, R1, s1, R2, s2, C, part_xy, part_x);
    else
        hipLaunchKernelGGL(colsum_kernel<false>, grid, dim3(256), 0, s, X, Y, R1, s1, R2, s2, C, part_xy, part_x);
    return SKR_CHECK_LAUNCH();
}
