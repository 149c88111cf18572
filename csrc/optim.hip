// Flat-arena optimizer kernels: global gradient norm + fused clip/Adam.
//
// The whole model's parameters, gradients and Adam moments are single
// contiguous fp32 buffers (sketch_rnn_amd/train/optim.py), padded to a
// multiple of 64 elements, so one float4-vectorised launch updates every
// tensor. Scalars live on the device so the step is graph-capturable:
//   scal[0] = lr, scal[1] = t (incremented on device), scal[2] = |g|, scal[3] = clip scale,
//   scal[4] = 1 if this step was skipped, scal[5] = number of skipped steps,
//   scal[6] = gradient scale (data parallel: 1/world folded in here instead of
//   a separate pass over the summed arena; <= 0 reads as 1)
// Failure detection: the global gradient norm is computed every step (all
// clip modes); with nonfinite_policy = 1 a step whose norm is NaN/Inf is
// skipped on the device (no update, t not advanced) and counted, so a
// diverging batch never needs a host sync to be caught.
// Adam is TF's (model.py:183): eps added to sqrt(v), bias corrections folded
// into lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t).
#include "common.h"

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ float grad_scale(const float* scal) {
    const float s = scal ? scal[6] : 1.f;
    return s > 0.f ? s : 1.f;
}

// The norm is taken over the SCALED elements (g * gs rounded to fp32 first),
// so a folded 1/world gives bit for bit the norm of a pre-scaled arena.
__global__ __launch_bounds__(kBlock) void sumsq_partial_kernel(const float4* __restrict__ g, int64_t n4,
                                                               double* __restrict__ partial,
                                                               const float* __restrict__ scal) {
    __shared__ float lds[kBlock / 64];
    const float gs = grad_scale(scal);
    float acc = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kBlock) {
        float4 v = g[i];
        if (gs != 1.f) {
            v.x *= gs;
            v.y *= gs;
            v.z *= gs;
            v.w *= gs;
        }
        acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    float a1[1] = {acc};
    skr::block_sum<1, kBlock / 64>(a1, lds);
    if (threadIdx.x == 0) partial[blockIdx.x] = (double)a1[0];
}

__global__ void finalize_kernel(const double* __restrict__ partial, int nparts, float* __restrict__ scal,
                                int clip_mode, float clip, int nonfinite_policy) {
    // single wave: deterministic order
    double s = 0.0;
    for (int i = threadIdx.x; i < nparts; i += 64) s += partial[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (threadIdx.x == 0) {
        const float norm = (float)sqrt(s);
        scal[2] = norm;
        const bool skip = nonfinite_policy == 1 && !isfinite(norm);
        scal[4] = skip ? 1.0f : 0.0f;
        if (skip) {
            scal[5] += 1.0f;
        } else {
            scal[1] += 1.0f;
        }
        scal[3] = clip_mode == 1 ? clip / fmaxf(norm, clip) : 1.0f;
    }
}

__global__ __launch_bounds__(kBlock) void adam_kernel(float4* __restrict__ p, const float4* __restrict__ g,
                                                      float4* __restrict__ m, float4* __restrict__ v,
                                                      const float* __restrict__ scal, int64_t n4, float b1,
                                                      float b2, float eps, int clip_mode, float clip) {
    if (scal[4] != 0.f) return;  // skipped (non-finite gradient)
    const float t = scal[1];
    const float lr_t = scal[0] * sqrtf(1.f - powf(b2, t)) / (1.f - powf(b1, t));
    const float sc = scal[3];
    const float gs = grad_scale(scal);
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kBlock) {
        float4 gg = g[i], mm = m[i], vv = v[i], pp = p[i];
        float* gv = &gg.x;
        float* mv = &mm.x;
        float* vvv = &vv.x;
        float* pv = &pp.x;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float x = gv[k];
            if (gs != 1.f) x *= gs;
            if (clip_mode == 1) x *= sc;
            else if (clip_mode == 2) x = fminf(fmaxf(x, -clip), clip);
            mv[k] = b1 * mv[k] + (1.f - b1) * x;
            vvv[k] = b2 * vvv[k] + (1.f - b2) * x * x;
            pv[k] -= lr_t * mv[k] / (sqrtf(vvv[k]) + eps);
        }
        m[i] = mm;
        v[i] = vv;
        p[i] = pp;
    }
}

int grid_for(int64_t n4) {
    int64_t g = (n4 + kBlock - 1) / kBlock;
    if (g > 2048) g = 2048;  // grid-stride beyond 8 blocks per CU
    if (g < 1) g = 1;
    return (int)g;
}

}  // namespace

// clip_mode: 0 none, 1 global norm, 2 per-element value. nonfinite_policy: 0 apply (TF semantics),
// 1 skip the step on a non-finite gradient norm. `partial` must hold 2048 doubles; scal 8 floats.
SKR_API int skr_adam_step(float* p, const float* g, float* m, float* v, float* scal, double* partial, int64_t n,
                          float b1, float b2, float eps, int clip_mode, float clip, int nonfinite_policy,
                          hipStream_t s) {
    if (n % 4 != 0) return -2;
    const int64_t n4 = n / 4;
    const int grid = grid_for(n4);
    hipLaunchKernelGGL(sumsq_partial_kernel, dim3(grid), dim3(kBlock), 0, s, (const float4*)g, n4, partial,
                       (const float*)scal);
    hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(64), 0, s, partial, grid, scal, clip_mode, clip,
                       nonfinite_policy);
    hipLaunchKernelGGL(adam_kernel, dim3(grid), dim3(kBlock), 0, s, (float4*)p, (const float4*)g, (float4*)m,
                       (float4*)v, (const float*)scal, n4, b1, b2, eps, clip_mode, clip);
    return SKR_CHECK_LAUNCH();
}

// standalone global norm (diagnostics): writes sqrt(sum g^2) to scal_tmp[2] (scal_tmp: 8 floats)
SKR_API int skr_global_norm(const float* g, int64_t n, double* partial, float* scal_tmp, hipStream_t s) {
    if (n % 4 != 0) return -2;
    const int64_t n4 = n / 4;
    const int grid = grid_for(n4);
    hipLaunchKernelGGL(sumsq_partial_kernel, dim3(grid), dim3(kBlock), 0, s, (const float4*)g, n4, partial,
                       (const float*)nullptr);
    hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(64), 0, s, partial, grid, scal_tmp, 1, 1.0f, 0);
    return SKR_CHECK_LAUNCH();
}
