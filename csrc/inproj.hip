// Input projection of the bidirectional encoder for narrow inputs (stroke-5:
// IN = 5), both directions in one pass, written straight into the [T, 2B, G]
// layout the recurrence reads (direction d owns rows d*B .. d*B+B-1 of every
// step):
//
//   xp[t, d*B + b, g] = bias_d[g] + sum_i x_d[t, b, i] * W_d[i, g]
//   x_0 = x,   x_1[t, b] = x[len_b - 1 - t, b] for t < len_b, else x[t, b]
//
// (the backward direction reads each sketch reversed within its length --
// the reference reverse_padded -- without materialising the reversed copy).
// A K = 5 product is pure output bandwidth: a library GEMM, a separate bias
// add and a concatenation each re-stream the [T, 2B, G] fp32 tensor.
//
// Backward: dW_d[i, g] = sum_{t,b} x_d[t,b,i] dxp[t, dB+b, g] and
// dbias_d[g] = sum_{t,b} dxp[t, dB+b, g] in one read of dxp; per-slice
// partials [RS, 2, IN+1, G] are summed by the caller.
#include "common.h"

namespace {

__device__ __forceinline__ int src_row(int t, int d, const int64_t* len, int b) {
    if (d == 0) return t;
    const int L = (int)len[b];
    return t < L ? L - 1 - t : t;
}

template <int IN>
__global__ __launch_bounds__(256) void inproj_fwd(const float* __restrict__ x, const int64_t* __restrict__ len,
                                                  const float* __restrict__ W, const float* __restrict__ bias,
                                                  float* __restrict__ xp, int T, int B, int G) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    const int t = blockIdx.y, d = blockIdx.z;
    if (g >= G) return;
    float w[IN];
#pragma unroll
    for (int i = 0; i < IN; ++i) w[i] = W[((int64_t)d * IN + i) * G + g];
    const float b0 = bias ? bias[(int64_t)d * G + g] : 0.f;
    float* out = xp + ((int64_t)t * 2 * B + (int64_t)d * B) * G + g;
#pragma unroll 4
    for (int b = 0; b < B; ++b) {
        const float* xr = x + ((int64_t)src_row(t, d, len, b) * B + b) * IN;
        float acc = b0;
#pragma unroll
        for (int i = 0; i < IN; ++i) acc += xr[i] * w[i];
        __builtin_nontemporal_store(acc, out + (int64_t)b * G);
    }
}

template <int IN>
__global__ __launch_bounds__(256) void inproj_bwd(const float* __restrict__ x, const int64_t* __restrict__ len,
                                                  const float* __restrict__ dxp, float* __restrict__ part,
                                                  int T, int B, int G) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    const int rs = blockIdx.y, RS = gridDim.y, d = blockIdx.z;
    if (g >= G) return;
    const int per = (T + RS - 1) / RS;
    const int t0 = rs * per, t1 = min(T, t0 + per);
    float acc[IN + 1];
#pragma unroll
    for (int i = 0; i <= IN; ++i) acc[i] = 0.f;
    for (int t = t0; t < t1; ++t) {
        const float* drow = dxp + ((int64_t)t * 2 * B + (int64_t)d * B) * G + g;
#pragma unroll 4
        for (int b = 0; b < B; ++b) {
            const float dv = drow[(int64_t)b * G];
            const float* xr = x + ((int64_t)src_row(t, d, len, b) * B + b) * IN;
#pragma unroll
            for (int i = 0; i < IN; ++i) acc[i] += xr[i] * dv;
            acc[IN] += dv;
        }
    }
    float* o = part + (((int64_t)rs * 2 + d) * (IN + 1)) * G + g;
#pragma unroll
    for (int i = 0; i <= IN; ++i) o[(int64_t)i * G] = acc[i];
}

template <int IN>
int launch_fwd(const float* x, const int64_t* len, const float* W, const float* bias, float* xp, int T, int B, int G,
               hipStream_t s) {
    hipLaunchKernelGGL(inproj_fwd<IN>, dim3((G + 255) / 256, T, 2), dim3(256), 0, s, x, len, W, bias, xp, T, B, G);
    return SKR_CHECK_LAUNCH();
}

template <int IN>
int launch_bwd(const float* x, const int64_t* len, const float* dxp, float* part, int T, int B, int G, int RS,
               hipStream_t s) {
    hipLaunchKernelGGL(inproj_bwd<IN>, dim3((G + 255) / 256, RS, 2), dim3(256), 0, s, x, len, dxp, part, T, B, G);
    return SKR_CHECK_LAUNCH();
}

}  // namespace

// x [T, B, IN] fp32, len [B] int64 (1 <= len <= T), W [2, IN, G], bias [2, G] or null -> xp [T, 2B, G].
SKR_API int skr_inproj_fwd(const float* x, const int64_t* len, const float* W, const float* bias, float* xp, int T,
                           int B, int IN, int G, hipStream_t s) {
    if (T <= 0 || B <= 0 || G <= 0) return 0;
    switch (IN) {
        case 3: return launch_fwd<3>(x, len, W, bias, xp, T, B, G, s);
        case 5: return launch_fwd<5>(x, len, W, bias, xp, T, B, G, s);
        default: return -2;
    }
}

// dxp [T, 2B, G] -> part [RS, 2, IN + 1, G]: rows i < IN are dW_d[i], row IN is dbias_d.
SKR_API int skr_inproj_bwd(const float* x, const int64_t* len, const float* dxp, float* part, int T, int B, int IN,
                           int G, int RS, hipStream_t s) {
    if (T <= 0 || B <= 0 || G <= 0 || RS <= 0) return -2;
    switch (IN) {
        case 3: return launch_bwd<3>(x, len, dxp, part, T, B, G, RS, s);
        case 5: return launch_bwd<5>(x, len, dxp, part, T, B, G, RS, s);
        default: return -2;
    }
}
