// MDN sampling of one row by one wave (reference capability R14,
// model.py:187-264), shared by the stand-alone sampler kernel
// (csrc/sampler.hip) and the fused whole-sketch decoder (csrc/decode_ref.hip)
// so both draw bit-identical strokes from the same head output.
//
// From z = [pen logits (3) | pi logits (M) | mu1 | mu2 | log s1 | log s2 |
// atanh rho (M each)] it draws the mixture component (temperature-scaled
// softmax + inverse CDF with the reference's "-1 -> last component" rule),
// the pen state and the 2-D Gaussian offset (Cholesky of the 2x2 covariance,
// Box-Muller normals). Random numbers: the stateless hash of common.h keyed
// by (seed, 0x5A3D, step), element 4*row + k.
//
// mode 0 = reference: pi temperature only from step 2 on; pen temperature
//          ignored unless fix_pen (the reference's pen-temperature bug); sigma
//          not scaled.
// mode 1 = sketch-rnn VAE: temperature on pi and pen from step 0; sigma scaled.
// greedy: argmax component / pen, offset = mean.
#pragma once
#include "common.h"

namespace skr {

struct MdnDraw {
    float row[5];     // [dx, dy, one-hot pen (3)]
    int idx, pidx;    // mixture component, pen state
    float s1, s2;     // (temperature-scaled) sigmas of the component
};

// Every lane of the wave must be active; the result is wave-uniform. The pi
// softmax runs across lanes (lane k holds component k); the inverse CDF then
// sums the M probabilities in component order with scalar adds (readlane),
// the same fp32 order as a sequential loop.
__device__ inline MdnDraw mdn_sample_wave(const float* zr, int M, int mode, float temp, int greedy, int fix_pen,
                                          uint32_t key, uint32_t b, uint32_t step) {
    const int lane = threadIdx.x & 63;
    const bool use_t = mode == 1 || step > 1;
    const float inv_t = use_t ? 1.f / temp : 1.f;
    const bool on = lane < M;
    const float l = on ? zr[3 + lane] * inv_t : -INFINITY;
    float m = l;
    for (int o = 16; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 32));
    const float e = on ? expf(l - m) : 0.f;
    float s = e;
    for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o, 32);
    const float p = e / s;   // lanes < 32: pi of component `lane`
    const float u0 = hash_uniform(key, 4u * b + 0u);
    const float u1 = hash_uniform(key, 4u * b + 1u);
    const float u2 = hash_uniform(key, 4u * b + 2u);
    const float u3 = hash_uniform(key, 4u * b + 3u);
    MdnDraw d;
    // component
    int idx = M - 1;
    if (greedy) {
        float best = -1.f;
        for (int k = 0; k < M; ++k) {
            const float pk = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), k));
            if (pk > best) { best = pk; idx = k; }
        }
    } else {
        float acc = 0.f;
        for (int k = 0; k < M; ++k) {
            acc += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), k));
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
    d.row[0] = x1;
    d.row[1] = x2;
    d.row[2] = pidx == 0 ? 1.f : 0.f;
    d.row[3] = pidx == 1 ? 1.f : 0.f;
    d.row[4] = pidx == 2 ? 1.f : 0.f;
    d.idx = idx;
    d.pidx = pidx;
    d.s1 = s1;
    d.s2 = s2;
    return d;
}

// Head output row b as the sum of `nslab` split-K partial slabs of the head
// GEMM (csrc/skinny_gemm.hip, z = h @ W_out, no bias) plus the bias, by a
// 256-thread workgroup: wave w folds the slabs s = w mod 4 of every column
// with independent (unrolled, clamped) loads, the four partial rows meet in
// LDS (`part` [4][256]), and zrow [nout] is ready after the call (every thread
// passed its barrier). LDS-only barriers: global loads the caller issued
// before the call stay in flight.
__device__ inline void fold_head_slabs(const float* __restrict__ zs, int64_t ldz, int nslab, int64_t slab,
                                       const float* __restrict__ bias, int nout, int b, float (*part)[256],
                                       float* zrow) {
    constexpr int kU = 8;                  // slabs per unrolled batch (per wave)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const float* zb = zs + (int64_t)b * ldz;
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) {
        const int c = lane + 64 * cc;
        if (c >= nout) break;
        float v = 0.f;
        for (int s0 = w; s0 < nslab; s0 += 4 * kU) {
            float t[kU];
#pragma unroll
            for (int k = 0; k < kU; ++k) t[k] = zb[(int64_t)min(s0 + 4 * k, nslab - 1) * slab + c];
#pragma unroll
            for (int k = 0; k < kU; ++k) v += (s0 + 4 * k < nslab) ? t[k] : 0.f;
        }
        part[w][c] = v;
    }
    lds_barrier();
    if (tid < nout) zrow[tid] = bias[tid] + ((part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid]));
    lds_barrier();
}

}  // namespace skr
