// Per-CU read rate by footprint: one 256-thread workgroup per CU (256 CUs),
// every workgroup streams the SAME `fp` bytes (offset by a per-workgroup
// rotation so the CUs do not march in lock step) `reps` times into VGPRs
// with global_load_dwordx4 (D loads in flight per lane). Footprints: 2 MB
// (fits one XCD's 4 MB L2), 64 MB (fits the 256 MB Infinity Cache, not L2),
// 1 GB (HBM). Reports GB/s per workgroup and TB/s over the chip.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/micro/l2_rate.hip -o scripts/micro/l2_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));

template <int D>
__global__ __launch_bounds__(256) void shared_stream(const f4* __restrict__ src, int64_t fp_vec, int64_t per_wg_vec,
                                                     float* out) {
    f4 acc = {0, 0, 0, 0};
    const int tid = threadIdx.x;
    const int64_t rot = ((int64_t)blockIdx.x * 4099 * 256) & (fp_vec - 1);
    for (int64_t i = 0; i < per_wg_vec; i += 256 * D) {
        f4 v[D];
#pragma unroll
        for (int d = 0; d < D; ++d) v[d] = src[(rot + i + d * 256 + tid) & (fp_vec - 1)];   // (power-of-two footprints)
#pragma unroll
        for (int d = 0; d < D; ++d) acc += v[d];
    }
    if (acc.x == 1234.5f) out[0] = acc.y;
}

// the same footprints through LDS-DMA (global_load_lds_dwordx4 into an NS-deep
// ring of 24 KB stages, counted vmcnt + barrier: the skinny GEMM's pattern)
template <int NS>
__global__ __launch_bounds__(256) void shared_stream_lds(const char* __restrict__ src, int64_t fp, int64_t per_wg,
                                                         float* out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int TILE = 24 * 1024;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n = (int)(per_wg / TILE);
    const int64_t rot = ((int64_t)blockIdx.x * 4099 * 4096) & (fp - 1);
    auto issue = [&](int kt) {
        char* st = smem + (kt % NS) * TILE;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const int64_t off = (rot + (int64_t)kt * TILE + (w + 4 * i) * 1024 + lane * 16) & (fp - 1);
            __builtin_amdgcn_global_load_lds((const void*)(src + off),
                                             (__attribute__((address_space(3))) void*)(st + (w + 4 * i) * 1024), 16, 0, 0);
        }
    };
    float acc = 0.f;
    for (int p = 0; p < NS - 1; ++p) issue(p);
    for (int kt = 0; kt < n; ++kt) {
        if (kt + NS - 1 < n) {
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 * (NS - 2)) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        if (kt + NS - 1 < n) issue(kt + NS - 1);
        acc += *(const float*)(smem + (kt % NS) * TILE + threadIdx.x * 16);
    }
    if (acc == 1234.5f) out[0] = acc;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int64_t big = (int64_t)1 << 30;
    f4* buf;
    float* out;
    if (hipMalloc(&buf, big) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    hipMemset(buf, 0, big);
    const int64_t per_wg = (int64_t)16 << 20;            // 16 MB read by every workgroup
    const int64_t fps[3] = {(int64_t)2 << 20, (int64_t)64 << 20, big};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int f = 0; f < 3; ++f) {
        const int64_t fp = fps[f];
        // HBM case: every workgroup reads its own 16 MB slice (unique data), no re-reads
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(e0);
            shared_stream<8><<<cus, 256>>>(buf, fp / 16, per_wg / 16, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep == 2)
                printf("{\"mode\": \"reg D8\", \"footprint_MB\": %lld, \"per_wg_MB\": %lld, \"us\": %.1f, \"GBps_per_wg\": %.1f, \"TBps_chip\": %.2f}\n",
                       (long long)(fp >> 20), (long long)(per_wg >> 20), ms * 1e3, per_wg / (ms * 1e-3) / 1e9,
                       per_wg * (double)cus / (ms * 1e-3) / 1e12);
        }
    }
    // LDS-DMA: 3- and 6-deep rings (72 / 144 KB)
    (void)hipFuncSetAttribute((const void*)shared_stream_lds<3>, hipFuncAttributeMaxDynamicSharedMemorySize, 3 * 24 * 1024);
    (void)hipFuncSetAttribute((const void*)shared_stream_lds<6>, hipFuncAttributeMaxDynamicSharedMemorySize, 6 * 24 * 1024);
    for (int f = 0; f < 3; ++f) {
        const int64_t fp = fps[f];
        for (int ns = 3; ns <= 6; ns += 3) {
            for (int rep = 0; rep < 3; ++rep) {
                hipEventRecord(e0);
                if (ns == 3) shared_stream_lds<3><<<cus, 256, 3 * 24 * 1024>>>((const char*)buf, fp, per_wg, out);
                else shared_stream_lds<6><<<cus, 256, 6 * 24 * 1024>>>((const char*)buf, fp, per_wg, out);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                if (rep == 2)
                    printf("{\"mode\": \"lds_dma NS%d\", \"footprint_MB\": %lld, \"us\": %.1f, \"GBps_per_wg\": %.1f, \"TBps_chip\": %.2f}\n",
                           ns, (long long)(fp >> 20), ms * 1e3, per_wg / (ms * 1e-3) / 1e9,
                           per_wg * (double)cus / (ms * 1e-3) / 1e12);
            }
        }
    }
    return 0;
}
