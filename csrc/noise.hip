// Stateless Gaussian noise for the VAE reparameterisation (z = mu + sigma *
// eps): eps = sqrt(-2 log(1 - u1)) * cos(2 pi u2) with u1, u2 from the hash
// of common.h keyed by (seed, stream, step) and (seed, stream + 0x3C6EF372,
// step) -- the same streams as sketch_rnn_amd/models/cells.py hash_normal,
// whose int64 torch emulation of the 32-bit hash is ~40 tiny kernels per
// call inside the training step. The seed is read from device memory, so a
// captured HIP graph draws fresh noise on every replay.
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void hash_normal_kernel(const int64_t* __restrict__ seed, uint32_t stream,
                                                          uint32_t step, float* __restrict__ out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int64_t s = *seed;
    const float u1 = 1.0f - skr::hash_uniform(skr::hash_key(s, stream, step), (uint32_t)i);
    const float u2 = skr::hash_uniform(skr::hash_key(s, stream + 0x3C6EF372u, step), (uint32_t)i);
    out[i] = sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
}

}  // namespace

SKR_API int skr_hash_normal(const int64_t* seed, uint32_t stream, uint32_t step, float* out, int64_t n,
                            hipStream_t s) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(hash_normal_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, seed, stream, step, out,
                       n);
    return SKR_CHECK_LAUNCH();
}
