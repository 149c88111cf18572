// Per-CU streaming rate probe (one workgroup per CU, 256 CUs): each
// workgroup streams `per_wg` bytes of a weight-like buffer either
//  (a) into VGPRs with global_load_dwordx4 (D 16-byte loads in flight per lane), or
//  (b) into an LDS ring with global_load_lds_dwordx4 (NS stages of 24 KB, counted
//      vmcnt waits + barrier, the skinny GEMM's pattern),
// and reports GB/s per workgroup from the kernel time. Build: hipcc -O3 --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float f4 __attribute__((ext_vector_type(4)));

template <int D>
__global__ __launch_bounds__(256) void reg_stream(const f4* __restrict__ src, int64_t per_wg_vec, float* out) {
    const f4* p = src + blockIdx.x * per_wg_vec;
    f4 acc = {0, 0, 0, 0};
    const int tid = threadIdx.x;
    for (int64_t i = 0; i < per_wg_vec; i += 256 * D) {
        f4 v[D];
#pragma unroll
        for (int d = 0; d < D; ++d) v[d] = p[i + d * 256 + tid];
#pragma unroll
        for (int d = 0; d < D; ++d) acc += v[d];
    }
    if (acc.x == 1234.5f) out[0] = acc.y;
}

template <int NS>
__global__ __launch_bounds__(256) void lds_stream(const char* __restrict__ src, int64_t per_wg, float* out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const char* p = src + blockIdx.x * per_wg;
    constexpr int TILE = 24 * 1024;                 // 24 KB per stage = 24 x 1 KB wave chunks
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n = (int)(per_wg / TILE);
    auto issue = [&](int kt) {
        char* st = smem + (kt % NS) * TILE;
#pragma unroll
        for (int i = 0; i < 6; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(p + (int64_t)kt * TILE + (w + 4 * i) * 1024 + lane * 16),
                                             (__attribute__((address_space(3))) void*)(st + (w + 4 * i) * 1024), 16, 0, 0);
    };
    for (int s = 0; s < NS - 1; ++s) if (s < n) issue(s);
    float acc = 0.f;
    for (int kt = 0; kt < n; ++kt) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // conservative: wait for everything
        __builtin_amdgcn_s_barrier();
        if (kt + NS - 1 < n) issue(kt + NS - 1);
        acc += ((const float*)(smem + (kt % NS) * TILE))[threadIdx.x];
    }
    if (acc == 1234.5f) out[0] = acc;
}

int main() {
    const int wgs = 256;
    const int64_t per_wg = 384 * 1024;             // the R_main tile's bytes
    char* buf;
    float* out;
    hipMalloc(&buf, per_wg * wgs);
    hipMalloc(&out, 4);
    hipMemset(buf, 0, per_wg * wgs);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto timeit = [&](auto launch, const char* name) {
        for (int i = 0; i < 3; ++i) launch();
        hipDeviceSynchronize();
        hipEventRecord(a);
        const int reps = 50;
        for (int i = 0; i < reps; ++i) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double us = ms * 1e3 / reps;
        printf("{\"probe\": \"%s\", \"us\": %.2f, \"GBps_per_wg\": %.1f, \"TBps_chip\": %.2f}\n", name, us,
               per_wg / us / 1e3, per_wg * wgs / us / 1e6);
    };
    timeit([&] { hipLaunchKernelGGL(reg_stream<4>, dim3(wgs), dim3(256), 0, 0, (const f4*)buf, per_wg / 16, out); }, "reg D4");
    timeit([&] { hipLaunchKernelGGL(reg_stream<8>, dim3(wgs), dim3(256), 0, 0, (const f4*)buf, per_wg / 16, out); }, "reg D8");
    timeit([&] { hipLaunchKernelGGL(reg_stream<16>, dim3(wgs), dim3(256), 0, 0, (const f4*)buf, per_wg / 16, out); }, "reg D16");
    hipFuncSetAttribute((const void*)lds_stream<3>, hipFuncAttributeMaxDynamicSharedMemorySize, 3 * 24576);
    hipFuncSetAttribute((const void*)lds_stream<6>, hipFuncAttributeMaxDynamicSharedMemorySize, 6 * 24576);
    timeit([&] { hipLaunchKernelGGL(lds_stream<3>, dim3(wgs), dim3(256), 3 * 24576, 0, buf, per_wg, out); }, "lds NS3 (vmcnt0)");
    timeit([&] { hipLaunchKernelGGL(lds_stream<6>, dim3(wgs), dim3(256), 6 * 24576, 0, buf, per_wg, out); }, "lds NS6 (vmcnt0)");
    // two workgroups per CU
    timeit([&] { hipLaunchKernelGGL(reg_stream<8>, dim3(2 * wgs), dim3(256), 0, 0, (const f4*)buf, per_wg / 32, out); }, "reg D8 x2/CU half each");
    return 0;
}
