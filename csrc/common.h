// Shared device helpers for the gfx950 (CDNA4, wave64) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define SKR_API extern "C" __attribute__((visibility("default")))

namespace skr {

constexpr int kWave = 64;  // CDNA wavefront width: never 32

// ---------------------------------------------------------------------------
// stateless dropout hash; bit-identical to sketch_rnn_amd/models/cells.py
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
__device__ __forceinline__ uint32_t hash_key(int64_t seed, uint32_t stream, uint32_t step) {
    uint32_t s = (uint32_t)(seed & 0xffffffffll);
    return mix32(s * 0x9E3779B1u + stream * 0x85EBCA77u + step * 0xC2B2AE3Du);
}
__device__ __forceinline__ float hash_uniform(uint32_t key, uint32_t idx) {
    uint32_t h = mix32(idx ^ key);
    h = mix32(h + key);
    return (float)(h >> 8) * (1.0f / 16777216.0f);
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// Hardware-instruction activations: v_exp_f32 (exp2) + v_rcp_f32, ~1 ulp each
// (absolute error ~1e-7 on sigma, ~2e-7 on tanh), against ~25-45 VALU ops
// per call for the IEEE-exact expf / division / tanhf. Saturate correctly:
// exp2 overflows to +inf -> rcp 0, underflows to 0 -> rcp 1.
__device__ __forceinline__ float sigmoid_fast(float x) {
    return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
}
__device__ __forceinline__ float tanh_fast(float x) {
    return 2.0f * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-2.8853900817779268f * x)) - 1.0f;
}

// ---------------------------------------------------------------------------
// reductions (wave64 shuffles, then LDS across the block's waves)
// ---------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float lane_f32(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
// Sum over the 64 lanes, returned to every lane (wave-uniform). Every lane
// must be active. Four DPP adds build each 16-lane row's sum in VALU
// registers (quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror,
// row_mirror), then the four row sums are read as scalars: no LDS-routed
// ds_bpermute chain (a __shfl_xor butterfly is six dependent LDS round trips).
__device__ __forceinline__ float wave_sum(float v) {
    v += dpp_f32<0xB1>(v);
    v += dpp_f32<0x4E>(v);
    v += dpp_f32<0x141>(v);
    v += dpp_f32<0x140>(v);
    return (lane_f32(v, 0) + lane_f32(v, 16)) + (lane_f32(v, 32) + lane_f32(v, 48));
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops
// (lgkmcnt) but, unlike __syncthreads(), not for its outstanding global loads
// and stores (vmcnt) -- a __syncthreads() after a burst of global stores
// stalls every wave until those stores retire.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Sums N values across a block of NW waves. `lds` must hold NW*N floats.
template <int N, int NW>
__device__ __forceinline__ void block_sum(float (&v)[N], float* lds) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = wave_sum(v[i]);
    if constexpr (NW == 1) {   // one wave: no LDS round trip and no barrier (the same 0 + v as below)
#pragma unroll
        for (int i = 0; i < N; ++i) v[i] = 0.f + v[i];
        (void)lane;
        (void)lds;
        return;
    }
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < N; ++i) lds[w * N + i] = v[i];
    }
    lds_barrier();
#pragma unroll
    for (int i = 0; i < N; ++i) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < NW; ++k) s += lds[k * N + i];
        v[i] = s;
    }
    lds_barrier();
}

__device__ __forceinline__ __hip_bfloat16 to_bf16(float x) { return __float2bfloat16(x); }

// Sum of the NS split-K partial slabs at idx (NS > 0: compile-time count,
// all loads independent); NS == 0: runtime count n, batches of 8 clamped loads.
template <int NS>
__device__ __forceinline__ float slab_sum(const float* p, int64_t idx, int n, int64_t slab) {
    if constexpr (NS > 0) {
        float v[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) v[s] = p[s * slab + idx];
#pragma unroll
        for (int w = 1; w < NS; w *= 2)
#pragma unroll
            for (int s = 0; s + w < NS; s += 2 * w) v[s] += v[s + w];
        return v[0];
    } else {
        float v = 0.f;
        for (int s0 = 0; s0 < n; s0 += 8) {
            float t[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) t[k] = p[(int64_t)min(s0 + k, n - 1) * slab + idx];
#pragma unroll
            for (int k = 0; k < 8; ++k) v += (s0 + k < n) ? t[k] : 0.f;
        }
        return v;
    }
}


// Split-K slab loads with a compile-time ceiling D on the runtime count n
// (1 <= n <= D): all D loads are issued back to back from clamped addresses
// (slabs past n re-read slab n-1: same line, no extra memory traffic), so a
// kernel can start several such sums before its first wait; slab_fold sums
// the first n. A null source contributes zeros without any load.
template <int D>
__device__ __forceinline__ void slab_load(const float* p, int64_t idx, int n, int64_t slab, float (&t)[D]) {
    if (p == nullptr) {
#pragma unroll
        for (int s = 0; s < D; ++s) t[s] = 0.f;
        return;
    }
#pragma unroll
    for (int s = 0; s < D; ++s) t[s] = p[(int64_t)min(s, n - 1) * slab + idx];
}

template <int D>
__device__ __forceinline__ float slab_fold(float (&t)[D], int n) {
#pragma unroll
    for (int s = 1; s < D; ++s) t[s] = s < n ? t[s] : 0.f;
#pragma unroll
    for (int w = 1; w < D; w *= 2)
#pragma unroll
        for (int s = 0; s + w < D; s += 2 * w) t[s] += t[s + w];
    return t[0];
}

}  // namespace skr

#define SKR_CHECK_LAUNCH() (int)hipGetLastError()
