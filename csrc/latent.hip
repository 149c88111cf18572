// VAE latent layer glue, fused (reference: magenta sketch_rnn model.py's
// reparameterisation and KL; ours: sketch_rnn_amd/models/vae.py
// SketchVAE.loss, ops/latent.py):
//
//   z  = mu + exp(presig / 2) * eps          eps: stateless hash normal (csrc/noise.hip)
//   kl = max(-0.5 mean(1 + presig - mu^2 - exp(presig)), kl_tolerance)
//   s  = tanh(pre), pre = z @ W_init + b_init, written as the decoder's
//        separate state tensors
//
// The three small GEMMs around it stay library GEMMs (ops/latent.py); as
// torch elementwise ops the rest was ~15 launches forward and ~20 backward
// of a few microseconds each inside the captured step. Here: latent_mid
// (one workgroup: z, eps, the KL mean and clamp), tanh_split, and their
// backward counterparts.
#include "common.h"

namespace {

using namespace skr;

constexpr int NTH = 1024;
constexpr int MAXSEG = 4;

__device__ __forceinline__ float block_sum1(float v, float* lds) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) lds[w] = v;
    __syncthreads();
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NTH / 64; ++k) s += lds[k];
    __syncthreads();
    return s;
}

// one workgroup: n = B*Z elements
__global__ __launch_bounds__(NTH) void latent_mid(const float* __restrict__ mu, const float* __restrict__ ps,
                                                  const float* __restrict__ eps_in, const int64_t* __restrict__ seed,
                                                  uint32_t stream, int n, float kl_tol, float* __restrict__ z,
                                                  float* __restrict__ eps, float* __restrict__ kl_raw,
                                                  float* __restrict__ kl) {
    __shared__ float red[NTH / 64];
    const int64_t s0 = eps_in ? 0 : *seed;
    float term = 0.f;
    for (int i = threadIdx.x; i < n; i += NTH) {
        const float m = mu[i], p = ps[i];
        float e;
        if (eps_in) {
            e = eps_in[i];
        } else {   // as csrc/noise.hip hash_normal_kernel (step 0)
            const float u1 = 1.0f - hash_uniform(hash_key(s0, stream, 0u), (uint32_t)i);
            const float u2 = hash_uniform(hash_key(s0, stream + 0x3C6EF372u, 0u), (uint32_t)i);
            e = sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
        }
        eps[i] = e;
        z[i] = m + expf(p / 2.0f) * e;
        term += ((1.0f + p) - m * m) - expf(p);
    }
    term = block_sum1(term, red);
    if (threadIdx.x == 0) {
        const float raw = -0.5f * (term / (float)n);
        *kl_raw = raw;
        *kl = fmaxf(raw, kl_tol);
    }
}

// dmu = dz + gk mu / n, dps = dz eps exp(ps / 2) / 2 - gk (1 - exp(ps)) / (2n);
// gk = dkl where the clamp passed (raw >= tol)
__global__ __launch_bounds__(256) void latent_mid_bwd(const float* __restrict__ mu, const float* __restrict__ ps,
                                                      const float* __restrict__ eps, const float* __restrict__ kl_raw,
                                                      float kl_tol, const float* __restrict__ dkl,
                                                      const float* __restrict__ dz, const float* __restrict__ dz2,
                                                      const float* __restrict__ dmu_ext,
                                                      const float* __restrict__ dps_ext, int n,
                                                      float* __restrict__ dmu, float* __restrict__ dps) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float gk = (dkl && kl_raw[0] >= kl_tol) ? dkl[0] : 0.f;
    const float m = mu[i], p = ps[i];
    const float g = (dz ? dz[i] : 0.f) + (dz2 ? dz2[i] : 0.f);
    dmu[i] = g + (dmu_ext ? dmu_ext[i] : 0.f) + gk * (m / (float)n);
    dps[i] = g * eps[i] * expf(p / 2.0f) * 0.5f + (dps_ext ? dps_ext[i] : 0.f) +
             gk * (-0.5f * (1.0f - expf(p)) / (float)n);
}

struct Segs {
    int nseg; int seg0[MAXSEG + 1];
    float* p[MAXSEG];
};

__device__ __forceinline__ int seg_of(const Segs& s, int c) {
    int k = 0;
    while (k + 1 < s.nseg && c >= s.seg0[k + 1]) ++k;
    return k;
}

// pre [B, S] -> tanh into the segments (seg k: columns [seg0[k], seg0[k+1]) as [B, width])
__global__ __launch_bounds__(256) void tanh_split(const float* __restrict__ pre, int B, int S, Segs s) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)B * S) return;
    const int b = (int)(i / S), c = (int)(i - (int64_t)b * S);
    const int k = seg_of(s, c);
    const int w0 = s.seg0[k], wd = s.seg0[k + 1] - w0;
    s.p[k][(int64_t)b * wd + (c - w0)] = tanhf(pre[i]);
}

// dpre [B, S] = dseg * (1 - seg^2) (a null segment grad is zero)
__global__ __launch_bounds__(256) void tanh_split_bwd(Segs out, Segs grad, int B, int S, float* __restrict__ dpre) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)B * S) return;
    const int b = (int)(i / S), c = (int)(i - (int64_t)b * S);
    const int k = seg_of(out, c);
    const int w0 = out.seg0[k], wd = out.seg0[k + 1] - w0;
    const int64_t o = (int64_t)b * wd + (c - w0);
    const float y = out.p[k][o];
    dpre[i] = grad.p[k] ? grad.p[k][o] * (1.0f - y * y) : 0.f;
}

}  // namespace

SKR_API int skr_latent_mid(const float* mu, const float* ps, const float* eps_in, const int64_t* seed, uint32_t stream,
                           int n, float kl_tol, float* z, float* eps, float* kl_raw, float* kl, hipStream_t s) {
    if (n <= 0) return -2;
    hipLaunchKernelGGL(latent_mid, dim3(1), dim3(NTH), 0, s, mu, ps, eps_in, seed, stream, n, kl_tol, z, eps, kl_raw,
                       kl);
    return SKR_CHECK_LAUNCH();
}

SKR_API int skr_latent_mid_bwd(const float* mu, const float* ps, const float* eps, const float* kl_raw, float kl_tol,
                               const float* dkl, const float* dz, const float* dz2, const float* dmu_ext,
                               const float* dps_ext, int n, float* dmu, float* dps, hipStream_t s) {
    if (n <= 0) return -2;
    hipLaunchKernelGGL(latent_mid_bwd, dim3((n + 255) / 256), dim3(256), 0, s, mu, ps, eps, kl_raw, kl_tol, dkl, dz, dz2,
                       dmu_ext, dps_ext, n, dmu, dps);
    return SKR_CHECK_LAUNCH();
}

// widths[k] (k < nseg <= 4) partition S; segs / grads: the per-segment tensors
SKR_API int skr_tanh_split(const float* pre, int B, int S, int nseg, const int* widths, float** segs, hipStream_t s) {
    if (B <= 0 || nseg < 1 || nseg > MAXSEG) return -2;
    Segs sg{};
    sg.nseg = nseg;
    for (int k = 0; k < nseg; ++k) {
        sg.seg0[k + 1] = sg.seg0[k] + widths[k];
        sg.p[k] = segs[k];
    }
    if (sg.seg0[nseg] != S) return -2;
    const int64_t n = (int64_t)B * S;
    hipLaunchKernelGGL(tanh_split, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, pre, B, S, sg);
    return SKR_CHECK_LAUNCH();
}

SKR_API int skr_tanh_split_bwd(int B, int S, int nseg, const int* widths, float** segs, float** grads, float* dpre,
                               hipStream_t s) {
    if (B <= 0 || nseg < 1 || nseg > MAXSEG) return -2;
    Segs so{}, sg{};
    so.nseg = sg.nseg = nseg;
    for (int k = 0; k < nseg; ++k) {
        so.seg0[k + 1] = sg.seg0[k + 1] = so.seg0[k] + widths[k];
        so.p[k] = segs[k];
        sg.p[k] = grads[k];
    }
    if (so.seg0[nseg] != S) return -2;
    const int64_t n = (int64_t)B * S;
    hipLaunchKernelGGL(tanh_split_bwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, so, sg, B, S, dpre);
    return SKR_CHECK_LAUNCH();
}
