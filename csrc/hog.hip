// Occupancy hog for concurrency tests (tests/test_dp_concurrency_gpu.py):
// a bounded kernel that holds `grid` workgroups of `threads` threads and
// `lds` bytes of LDS each for `us` microseconds of wall time -- the CU
// footprint of an RCCL collective kernel running on a communication stream
// beside the compute stream under data parallelism. Every wave exits after
// the deadline (wall_clock64, the device's constant-rate clock), so the grid always drains.
#include "common.h"

namespace {

__global__ void hog_kernel(int64_t ticks, int nlds, float* sink) {
    extern __shared__ float sm[];
    const int64_t t0 = wall_clock64();
    float v = (float)threadIdx.x;
    int i = 0;
    while (wall_clock64() - t0 < ticks) {
        v = v * 0.999f + 1.0f;
        if (nlds > 0) sm[(threadIdx.x + i) % nlds] = v;
        ++i;
        __builtin_amdgcn_s_sleep(8);
    }
    if (v == -1.0f) sink[0] = v;   // keeps the loop live; never true
}

}  // namespace

SKR_API int skr_occupancy_hog(int grid, int threads, int lds_bytes, int us, float* sink, hipStream_t s) {
    if (grid <= 0 || threads <= 0 || threads > 1024 || lds_bytes < 0 || lds_bytes > 160 * 1024 || us <= 0 || us > 2000000)
        return -2;
    if (lds_bytes > 64 * 1024 &&
        hipFuncSetAttribute((const void*)hog_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes) != hipSuccess)
        return -6;
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
        khz <= 0)
        khz = 100000;                             // 100 MHz
    const int64_t ticks = (int64_t)us * khz / 1000;
    hipLaunchKernelGGL(hog_kernel, dim3(grid), dim3(threads), lds_bytes, s, ticks, lds_bytes / 4, sink);
    return SKR_CHECK_LAUNCH();
}

// A stream on its own hardware queue restricted to the first `ncu` CUs of
// the CU mask (a CU-masked queue): the failure-path test runs the persistent
// encoder backward on it, so that only part of a row block can be resident
// -- the state a co-running kernel holding the rest of the chip creates.
// Tests only.
SKR_API int skr_stream_create_cu_limited(int ncu, hipStream_t* out) {
    if (ncu < 1 || ncu > 1024) return -2;
    uint32_t mask[32] = {};
    for (int i = 0; i < ncu; ++i) mask[i / 32] |= 1u << (i % 32);
    return hipExtStreamCreateWithCUMask(out, (uint32_t)((ncu + 31) / 32), mask) == hipSuccess ? 0 : -3;
}

SKR_API int skr_stream_destroy(hipStream_t s) { return hipStreamDestroy(s) == hipSuccess ? 0 : -1; }
