// On-device MDN sampler (reference capability R14, model.py:187-264).
//
// One wave per batch row. From the head output z [B, 3 + 6M] it draws the
// mixture component (temperature-scaled softmax + inverse CDF with the
// reference's "-1 -> last component" rule), the pen state, and the 2-D
// Gaussian offset (Cholesky of the 2x2 covariance, Box-Muller normals), then
// writes (a) the sampled stroke row into the output sequence and (b) the
// next decoder input -- so an N-step decode loop never returns to the host
// and can be captured whole in one HIP graph. Random numbers come from the
// same stateless hash as the dropout masks (seed read from device memory).
//
// mode 0 = reference: layout [dx, dy, eos, eoc, cont]; pi temperature only
//          from step 2 on; pen temperature ignored unless fix_pen; sigma not
//          scaled; a row stops after emitting eoc (done flag).
// mode 1 = sketch-rnn VAE: layout [dx, dy, p1, p2, p3]; temperature on pi and
//          pen from step 0; sigma scaled by the temperature; a row stops after
//          emitting p3.
// greedy: argmax component / pen, offset = mean.
#include "common.h"

namespace {

__global__ __launch_bounds__(64) void mdn_sample_kernel(const float* __restrict__ z, int64_t ldz, int M, int mode,
                                                        float temp, int greedy, int fix_pen, const int64_t* seed,
                                                        uint32_t step, float* __restrict__ out_row, int64_t ld_out,
                                                        float* __restrict__ next_x, int64_t ld_next,
                                                        int* __restrict__ done, float* __restrict__ params) {
    __shared__ float pi_s[32];
    const int b = blockIdx.x, lane = threadIdx.x;
    const float* zr = z + b * ldz;
    const uint32_t key = skr::hash_key(*seed, 0x5A3Du, step);
    // temperature on pi: reference applies it from step 2 on only
    const bool use_t = mode == 1 || step > 1;
    const float inv_t = use_t ? 1.f / temp : 1.f;
    const bool on = lane < M;
    const float l = on ? zr[3 + lane] * inv_t : -INFINITY;
    float m = l;
    for (int o = 16; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 32));
    const float e = on ? expf(l - m) : 0.f;
    float s = e;
    for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o, 32);
    if (lane < 32) pi_s[lane] = e / s;
    __syncthreads();
    if (lane != 0) return;
    const int rb = (int)b;
    const float u0 = skr::hash_uniform(key, 4u * rb + 0u);
    const float u1 = skr::hash_uniform(key, 4u * rb + 1u);
    const float u2 = skr::hash_uniform(key, 4u * rb + 2u);
    const float u3 = skr::hash_uniform(key, 4u * rb + 3u);
    // component
    int idx = M - 1;
    if (greedy) {
        float best = -1.f;
        for (int k = 0; k < M; ++k)
            if (pi_s[k] > best) { best = pi_s[k]; idx = k; }
    } else {
        float acc = 0.f;
        for (int k = 0; k < M; ++k) {
            acc += pi_s[k];
            if (acc >= u0) { idx = k; break; }
        }
    }
    // pen
    const float pt = (mode == 1 || (fix_pen && step > 1)) ? 1.f / temp : 1.f;
    float pl[3] = {zr[0] * pt, zr[1] * pt, zr[2] * pt};
    const float pm = fmaxf(pl[0], fmaxf(pl[1], pl[2]));
    float pp[3], ps = 0.f;
    for (int k = 0; k < 3; ++k) {
        pp[k] = expf(pl[k] - pm);
        ps += pp[k];
    }
    int pidx = 2;
    if (greedy) {
        pidx = pp[0] >= pp[1] ? (pp[0] >= pp[2] ? 0 : 2) : (pp[1] >= pp[2] ? 1 : 2);
    } else {
        float acc = 0.f;
        for (int k = 0; k < 3; ++k) {
            acc += pp[k] / ps;
            if (acc >= u1) { pidx = k; break; }
        }
    }
    // gaussian
    const float mu1 = zr[3 + M + idx], mu2 = zr[3 + 2 * M + idx];
    float s1 = expf(zr[3 + 3 * M + idx]), s2 = expf(zr[3 + 4 * M + idx]);
    const float rho = tanhf(zr[3 + 5 * M + idx]);
    if (mode == 1) {
        s1 *= temp;
        s2 *= temp;
    }
    float x1 = mu1, x2 = mu2;
    if (!greedy) {
        const float r = sqrtf(-2.f * logf(fmaxf(u2, 1e-12f)));
        const float n1 = r * cosf(6.283185307179586f * u3), n2 = r * sinf(6.283185307179586f * u3);
        x1 = mu1 + s1 * n1;
        x2 = mu2 + s2 * (rho * n1 + sqrtf(fmaxf(1.f - rho * rho, 0.f)) * n2);
    }
    float row[5] = {x1, x2, 0.f, 0.f, 0.f};
    row[2 + pidx] = 1.f;
    const bool was_done = done[b] != 0;
    float* o = out_row + b * ld_out;
    if (was_done) {
        // finished rows emit end-of-sketch padding
        for (int k = 0; k < 5; ++k) o[k] = 0.f;
        o[mode == 1 ? 4 : 3] = 1.f;
    } else {
        for (int k = 0; k < 5; ++k) o[k] = row[k];
    }
    float* nx = next_x + b * ld_next;
    for (int k = 0; k < 5; ++k) nx[k] = row[k];
    const int stop_col = mode == 1 ? 4 : 3;  // p3 | eoc
    if (pidx + 2 == stop_col) done[b] = 1;
    if (params) {
        float* p = params + b * 4;
        p[0] = (float)idx;
        p[1] = (float)pidx;
        p[2] = s1;
        p[3] = s2;
    }
}

}  // namespace

SKR_API int skr_mdn_sample(const float* z, int64_t ldz, int B, int M, int mode, float temp, int greedy, int fix_pen,
                           const int64_t* seed, uint32_t step, float* out_row, int64_t ld_out, float* next_x,
                           int64_t ld_next, int* done, float* params, hipStream_t s) {
    if (M < 1 || M > 32) return -2;
    if (B <= 0) return 0;
    hipLaunchKernelGGL(mdn_sample_kernel, dim3(B), dim3(64), 0, s, z, ldz, M, mode, temp, greedy, fix_pen, seed, step,
                       out_row, ld_out, next_x, ld_next, done, params);
    return SKR_CHECK_LAUNCH();
}
