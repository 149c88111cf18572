// PMC calibration: kernels that move a KNOWN number of bytes, so the
// FETCH_SIZE / WRITE_SIZE a rocprofv3 --pmc pass reports for them can be
// divided by the true count (scripts/pmc_calib.py). Every buffer is 1 GiB,
// four times the 256 MiB Infinity Cache, and each launch touches it once:
// no re-read can be served on-die.
//
// Access forms = the ones the framework's kernels use:
//   rd16   global_load_dwordx4, 16 B per lane (skinny / cell / reduce kernels)
//   rd8    global_load_dwordx2,  8 B per lane (bf16 x 4 row-cell loads)
//   lds16  global_load_lds_dwordx4, 16 B per lane (the GEMM rings)
//   wr16   global_store_dwordx4 (cell outputs, wgrad epilogue rows)
//   wr8    global_store_dwordx2 (bf16 x 4 row-cell stores)
// Build: hipcc -O3 --offload-arch=gfx950 -o pmc_calib pmc_calib.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int64_t kBytes = 1ll << 30;
constexpr int kGrid = 2048, kThreads = 256;

__global__ __launch_bounds__(kThreads) void rd16(const f4* __restrict__ p, int64_t n, float* out) {
    f4 acc = {0, 0, 0, 0};
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)kGrid * kThreads) acc += p[i];
    if (acc.x == 1234.5f) out[0] = acc.y;   // never true on the zero-filled buffer: keeps the loads
}

__global__ __launch_bounds__(kThreads) void rd8(const f2* __restrict__ p, int64_t n, float* out) {
    f2 acc = {0, 0};
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)kGrid * kThreads) acc += p[i];
    if (acc.x == 1234.5f) out[0] = acc.y;
}

// each wave moves 1 KiB per instruction into its own LDS slot (4 slots per wave, ring)
__global__ __launch_bounds__(kThreads) void lds16(const char* __restrict__ p, int64_t nchunks, float* out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float acc = 0.f;
    int slot = 0;
    for (int64_t c = (int64_t)blockIdx.x * 4 + w; c < nchunks; c += (int64_t)kGrid * 4) {
        __builtin_amdgcn_global_load_lds((const void*)(p + c * 1024 + lane * 16),
                                         (__attribute__((address_space(3))) void*)(smem + (w * 4 + slot) * 1024), 16, 0,
                                         0);
        slot = (slot + 1) & 3;
        if (slot == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            acc += ((const float*)(smem + w * 4096))[lane];
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (acc == 1234.5f) out[0] = acc;
}

__global__ __launch_bounds__(kThreads) void wr16(f4* __restrict__ p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)kGrid * kThreads)
        p[i] = f4{1.f, 2.f, 3.f, 4.f};
}

__global__ __launch_bounds__(kThreads) void wr8(f2* __restrict__ p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)kGrid * kThreads)
        p[i] = f2{1.f, 2.f};
}

int main() {
    char* buf;
    float* out;
    if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    hipMemset(buf, 0, kBytes);
    hipFuncSetAttribute((const void*)lds16, hipFuncAttributeMaxDynamicSharedMemorySize, 16 * 1024);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto timeit = [&](auto launch, const char* name) {
        launch();
        hipDeviceSynchronize();
        const int reps = 3;
        hipEventRecord(a);
        for (int i = 0; i < reps; ++i) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        printf("{\"kernel\": \"%s\", \"bytes\": %lld, \"launches\": %d, \"us\": %.1f, \"TBps\": %.2f}\n", name,
               (long long)kBytes, reps + 1, ms * 1e3 / reps, kBytes / (ms * 1e-3 / reps) / 1e12);
    };
    timeit([&] { hipLaunchKernelGGL(rd16, dim3(kGrid), dim3(kThreads), 0, 0, (const f4*)buf, kBytes / 16, out); }, "rd16");
    timeit([&] { hipLaunchKernelGGL(rd8, dim3(kGrid), dim3(kThreads), 0, 0, (const f2*)buf, kBytes / 8, out); }, "rd8");
    timeit([&] { hipLaunchKernelGGL(lds16, dim3(kGrid), dim3(kThreads), 16 * 1024, 0, buf, kBytes / 1024, out); },
           "lds16");
    timeit([&] { hipLaunchKernelGGL(wr16, dim3(kGrid), dim3(kThreads), 0, 0, (f4*)buf, kBytes / 16); }, "wr16");
    timeit([&] { hipLaunchKernelGGL(wr8, dim3(kGrid), dim3(kThreads), 0, 0, (f2*)buf, kBytes / 8); }, "wr8");
    return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
