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

// LP: dxp is the persistent encoder's bf16 gate gradient, direction-major
// [2][T][B][G] (no fp32 copy of it is ever written); else fp32 [T][2B][G].
template <int IN, bool LP>
__global__ __launch_bounds__(256) void inproj_bwd(const float* __restrict__ x, const int64_t* __restrict__ len,
                                                  const void* __restrict__ dxp, float* __restrict__ part,
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
        const int64_t r0 = LP ? ((int64_t)d * T + t) * B : (int64_t)t * 2 * B + (int64_t)d * B;
#pragma unroll 4
        for (int b = 0; b < B; ++b) {
            const int64_t o = (r0 + b) * G + g;
            const float dv = LP ? __bfloat162float(((const __hip_bfloat16*)dxp)[o]) : ((const float*)dxp)[o];
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
int launch_bwd(const float* x, const int64_t* len, const void* dxp, int lp, float* part, int T, int B, int G, int RS,
               hipStream_t s) {
    if (lp)
        hipLaunchKernelGGL((inproj_bwd<IN, true>), dim3((G + 255) / 256, RS, 2), dim3(256), 0, s, x, len, dxp, part, T, B, G);
    else
        hipLaunchKernelGGL((inproj_bwd<IN, false>), dim3((G + 255) / 256, RS, 2), dim3(256), 0, s, x, len, dxp, part, T, B, G);
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

// dxp [T, 2B, G] fp32 (lp = 0) or [2, T, B, G] bf16 (lp = 1) -> part [RS, 2, IN + 1, G]:
// rows i < IN are dW_d[i], row IN is dbias_d.
SKR_API int skr_inproj_bwd(const float* x, const int64_t* len, const void* dxp, int lp, float* part, int T, int B,
                           int IN, int G, int RS, hipStream_t s) {
    if (T <= 0 || B <= 0 || G <= 0 || RS <= 0) return -2;
    switch (IN) {
        case 3: return launch_bwd<3>(x, len, dxp, lp, part, T, B, G, RS, s);
        case 5: return launch_bwd<5>(x, len, dxp, lp, part, T, B, G, RS, s);
        default: return -2;
    }
}

// ---------------------------------------------------------------------------
// Decoder input projection with a per-sequence broadcast part: the decoder
// input is [stroke-5 | z] with z constant over time, so
//
//   xp[t, b, g] = zw[b, g] + sum_{i<IN} x[t, b, i] * W[i, g]
//
// with zw = z @ W_z (+ bias) computed once per sequence ([B, G], a tiny
// GEMM) instead of a K = 5 + |z| product over all T*B rows. Backward, one
// read of dxp (fp32 or bf16):
//   S[b, g] = sum_t dxp[t, b, g]                    (-> dz, dW_z, dbias)
//   P[b, i, g] = sum_t x[t, b, i] dxp[t, b, g]     (-> dW[:IN] = sum_b P)
namespace {

// OBF: xp written as bf16 (the HyperLSTM fused-modulation path reads xh as
// bf16: half the bytes of the largest tensor the decoder forward writes)
template <int IN, bool OBF>
__global__ __launch_bounds__(256) void bproj_fwd(const float* __restrict__ x, const float* __restrict__ W,
                                                 const float* __restrict__ zw, void* __restrict__ xp, int T, int B,
                                                 int G, int tpb) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    const int b = blockIdx.y;
    if (g >= G) return;
    float w[IN];
#pragma unroll
    for (int i = 0; i < IN; ++i) w[i] = W[(int64_t)i * G + g];
    const float z0 = zw ? zw[(int64_t)b * G + g] : 0.f;
    const int t0 = blockIdx.z * tpb, t1 = min(T, t0 + tpb);
#pragma unroll 4
    for (int t = t0; t < t1; ++t) {
        const float* xr = x + ((int64_t)t * B + b) * IN;
        float acc = z0;
#pragma unroll
        for (int i = 0; i < IN; ++i) acc += xr[i] * w[i];
        if constexpr (OBF)
            __builtin_nontemporal_store(__bfloat16_as_ushort(skr::to_bf16(acc)),
                                        (unsigned short*)xp + ((int64_t)t * B + b) * G + g);
        else
            __builtin_nontemporal_store(acc, (float*)xp + ((int64_t)t * B + b) * G + g);
    }
}

template <int IN, bool BF16>
__global__ __launch_bounds__(256) void bproj_bwd(const float* __restrict__ x, const void* __restrict__ dxp,
                                                 int64_t ld, float* __restrict__ S, float* __restrict__ P, int T,
                                                 int B, int G) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    const int b = blockIdx.y;
    if (g >= G) return;
    float acc[IN + 1];
#pragma unroll
    for (int i = 0; i <= IN; ++i) acc[i] = 0.f;
#pragma unroll 4
    for (int t = 0; t < T; ++t) {
        const int64_t o = ((int64_t)t * B + b) * ld + g;
        const float dv = BF16 ? __bfloat162float(((const __hip_bfloat16*)dxp)[o]) : ((const float*)dxp)[o];
        const float* xr = x + ((int64_t)t * B + b) * IN;
#pragma unroll
        for (int i = 0; i < IN; ++i) acc[i] += xr[i] * dv;
        acc[IN] += dv;
    }
    S[(int64_t)b * G + g] = acc[IN];
#pragma unroll
    for (int i = 0; i < IN; ++i) P[((int64_t)b * IN + i) * G + g] = acc[i];
}

// Wide form of bproj_bwd: NC consecutive columns per lane (one 16-byte load
// per row: 8 bf16 or 4 fp32), the T steps of a row split over the 4 waves
// of the workgroup (wave w: steps [w Tq, (w + 1) Tq)) and the 4 partial sums
// added through LDS in wave order -- 4 independent load chains per column
// and 16-byte loads instead of one 2-byte load per lane per step (the
// narrow kernel's dxp read is latency-bound: 410 MB in 103 us on the
// vae_large dXH). Deterministic; the summation order differs from the
// narrow kernel's (sequential in t).
constexpr int kBpU = 8;   // steps in flight per wave

template <int IN, bool BF16>
__global__ __launch_bounds__(256) void bproj_bwd_wide(const float* __restrict__ x, const void* __restrict__ dxp,
                                                      int64_t ld, float* __restrict__ S, float* __restrict__ P, int T,
                                                      int B, int G) {
    constexpr int NC = BF16 ? 8 : 4;
    __shared__ float red[3][IN + 1][64 * NC];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int b = blockIdx.y;
    const int g = (blockIdx.x * 64 + lane) * NC;
    const bool on = g < G;
    const int gg = on ? g : 0;
    const int Tq = (T + 3) / 4, t0 = w * Tq, t1 = min(T, t0 + Tq);
    float acc[IN + 1][NC];
#pragma unroll
    for (int i = 0; i <= IN; ++i)
#pragma unroll
        for (int e = 0; e < NC; ++e) acc[i][e] = 0.f;
    auto load = [&](int t, float (&v)[NC]) {
        const int64_t o = ((int64_t)t * B + b) * ld + gg;
        if constexpr (BF16) {
            const uint4 u = *(const uint4*)((const __hip_bfloat16*)dxp + o);
            const uint32_t q[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                v[2 * k] = __uint_as_float(q[k] << 16);
                v[2 * k + 1] = __uint_as_float(q[k] & 0xffff0000u);
            }
        } else {
            const float4 f = *(const float4*)((const float*)dxp + o);
            v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
        }
    };
    auto add = [&](int t, const float (&v)[NC]) {
        const float* xr = x + ((int64_t)t * B + b) * IN;   // (wave-uniform: scalar loads)
#pragma unroll
        for (int i = 0; i < IN; ++i) {
            const float xi = xr[i];
#pragma unroll
            for (int e = 0; e < NC; ++e) acc[i][e] += xi * v[e];
        }
#pragma unroll
        for (int e = 0; e < NC; ++e) acc[IN][e] += v[e];
    };
    int t = t0;
    for (; t + kBpU <= t1; t += kBpU) {
        float v[kBpU][NC];
#pragma unroll
        for (int k = 0; k < kBpU; ++k) load(t + k, v[k]);
#pragma unroll
        for (int k = 0; k < kBpU; ++k) add(t + k, v[k]);
    }
    for (; t < t1; ++t) {
        float v[NC];
        load(t, v);
        add(t, v);
    }
    if (w > 0) {
#pragma unroll
        for (int i = 0; i <= IN; ++i)
#pragma unroll
            for (int e = 0; e < NC; ++e) red[w - 1][i][lane * NC + e] = acc[i][e];
    }
    __syncthreads();
    if (w != 0 || !on) return;
#pragma unroll
    for (int ww = 0; ww < 3; ++ww)   // wave order: fixed
#pragma unroll
        for (int i = 0; i <= IN; ++i)
#pragma unroll
            for (int e = 0; e < NC; ++e) acc[i][e] += red[ww][i][lane * NC + e];
#pragma unroll
    for (int e = 0; e < NC; e += 4) {
        *(float4*)(S + (int64_t)b * G + g + e) = float4{acc[IN][e], acc[IN][e + 1], acc[IN][e + 2], acc[IN][e + 3]};
#pragma unroll
        for (int i = 0; i < IN; ++i)
            *(float4*)(P + ((int64_t)b * IN + i) * G + g + e) =
                float4{acc[i][e], acc[i][e + 1], acc[i][e + 2], acc[i][e + 3]};
    }
}

template <int IN>
int bproj_launch_fwd(const float* x, const float* W, const float* zw, void* xp, int T, int B, int G, int obf,
                     hipStream_t s) {
    const int tz = (T + 31) / 32;   // time slices: >= 256 workgroups at B ~ 100
    if (obf)
        hipLaunchKernelGGL((bproj_fwd<IN, true>), dim3((G + 255) / 256, B, tz), dim3(256), 0, s, x, W, zw, xp, T, B, G,
                           (T + tz - 1) / tz);
    else
        hipLaunchKernelGGL((bproj_fwd<IN, false>), dim3((G + 255) / 256, B, tz), dim3(256), 0, s, x, W, zw, xp, T, B,
                           G, (T + tz - 1) / tz);
    return SKR_CHECK_LAUNCH();
}

static int g_bproj_wide = 1;

template <int IN>
int bproj_launch_bwd(const float* x, const void* dxp, int kind, int64_t ld, float* S, float* P, int T, int B, int G,
                     hipStream_t s) {
    const int nc = kind == 1 ? 8 : 4;
    if (g_bproj_wide && G % nc == 0 && ld % nc == 0 && ((uintptr_t)dxp & 15) == 0 && ((uintptr_t)S & 15) == 0 &&
        ((uintptr_t)P & 15) == 0) {
        const dim3 gw((G + 64 * nc - 1) / (64 * nc), B);
        if (kind == 1)
            hipLaunchKernelGGL((bproj_bwd_wide<IN, true>), gw, dim3(256), 0, s, x, dxp, ld, S, P, T, B, G);
        else
            hipLaunchKernelGGL((bproj_bwd_wide<IN, false>), gw, dim3(256), 0, s, x, dxp, ld, S, P, T, B, G);
        return SKR_CHECK_LAUNCH();
    }
    const dim3 grid((G + 255) / 256, B);
    if (kind == 1)
        hipLaunchKernelGGL((bproj_bwd<IN, true>), grid, dim3(256), 0, s, x, dxp, ld, S, P, T, B, G);
    else
        hipLaunchKernelGGL((bproj_bwd<IN, false>), grid, dim3(256), 0, s, x, dxp, ld, S, P, T, B, G);
    return SKR_CHECK_LAUNCH();
}

}  // namespace

// x [T, B, IN] fp32, W [IN, G] fp32 (the stroke rows), zw [B, G] fp32 or null -> xp [T, B, G] fp32 (obf: bf16).
SKR_API int skr_bproj_fwd(const float* x, const float* W, const float* zw, void* xp, int T, int B, int IN, int G,
                          int obf, hipStream_t s) {
    if (T <= 0 || B <= 0 || G <= 0) return 0;
    switch (IN) {
        case 3: return bproj_launch_fwd<3>(x, W, zw, xp, T, B, G, obf, s);
        case 5: return bproj_launch_fwd<5>(x, W, zw, xp, T, B, G, obf, s);
        default: return -2;
    }
}

// A/B hook: 1 the wide backward reduction (bproj_bwd_wide) where its
// alignment holds, 0 the narrow one; returns the previous setting.
SKR_API int skr_bproj_set_wide(int w) {
    const int prev = g_bproj_wide;
    if (w >= 0) g_bproj_wide = w;
    return prev;
}

// dxp [T, B, *] (row stride ld; kind 1 bf16, 2 fp32) -> S [B, G], P [B, IN, G].
SKR_API int skr_bproj_bwd(const float* x, const void* dxp, int kind, int64_t ld, float* S, float* P, int T, int B,
                          int IN, int G, hipStream_t s) {
    if (T <= 0 || B <= 0 || G <= 0) return -2;
    switch (IN) {
        case 3: return bproj_launch_bwd<3>(x, dxp, kind, ld, S, P, T, B, G, s);
        case 5: return bproj_launch_bwd<5>(x, dxp, kind, ld, S, P, T, B, G, s);
        default: return -2;
    }
}
