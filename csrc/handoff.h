// In-launch hand-off primitives shared by the persistent kernels
// (csrc/lstm_persist.hip, csrc/decode_ref.hip).
//
// Protocol (CDNA4 guide, Guideline 16, first row of the measured hand-offs
// table): the producer stores its payload write-through (buffer_store ...
// sc1), every storing wave drains (s_waitcnt vmcnt(0)), a workgroup barrier,
// then ONE lane stores the workgroup's epoch into its flag word with an sc1
// store. A consumer wave polls the flag words it depends on with sc1 loads
// (one lane per flag, bounded spin with s_sleep) and then reads the payload
// with sc1 buffer loads only. A timed-out wait sets *err (the host raises)
// and poisons the launch so every other wait returns at once: the grid
// always drains.
#pragma once
#include "common.h"

// Per-launch state of a chained launch (csrc/chain_step.hip, csrc/hyper_mod.hip;
// mirrored by sketch_rnn_amd/ops/_hipapi.py ChainSync).
struct ChainSync {
    uint32_t* counters;   // [n] rotating arrival counters of this launch kind (zeroed once)
    int n, k;             // this launch uses counters[k] and zeroes counters[(k + 1) % n]
    int* err;             // set to 3 by a timed-out wait
};

namespace skr {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kSc1 = 16;                  // buffer cache-policy bits: sc1 (device scope, write-through)
constexpr unsigned kHandoffSpinLimit = 1u << 22;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)(bytes > 0x7fffffff ? 0x7fffffff : bytes),
                                             0x00020000);
}
__device__ __forceinline__ bf16x8 ld_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kSc1));
}
__device__ __forceinline__ float ld_sc1_f32(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, kSc1));
}
__device__ __forceinline__ void st_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kSc1);
}
__device__ __forceinline__ void st_sc1_f32(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off, 0, kSc1);
}

// One wave waits until every flag of `flags[0..n)` (n <= 64) is >= epoch
// (lane i polls flag i with sc1 loads). Bounded by `limit` polls; on a
// timeout (or when another wait of this launch already timed out)
// sets/observes *err and returns false.
__device__ inline bool wait_flags(const uint32_t* flags, int n, uint32_t epoch, int* err,
                                  unsigned limit = kHandoffSpinLimit) {
    const int lane = threadIdx.x & 63;
    const uint32_t* f = flags + (lane < n ? lane : 0);
    for (unsigned spins = 0;; ++spins) {
        const uint32_t v = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__all(lane >= n || v >= epoch)) break;
        if ((spins & 255) == 255) {
            const int e = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (e != 0) return false;
            if (spins > limit) {
                if (lane == 0) __hip_atomic_store(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return false;
            }
        }
        __builtin_amdgcn_s_sleep(1);
    }
    // compiler barrier: the payload loads may not move above the poll
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return true;
}

// Publish: every storing wave already issued its sc1 payload stores.
__device__ __forceinline__ void publish(uint32_t* flag, uint32_t epoch) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ f32x4 ld_sc1_f32x4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kSc1));
}

// ---- chained launches (csrc/chain_step.hip) ---------------------------------------------
// A grouped GEMM launch whose leading "producer" tiles feed cell rows of the
// SAME launch. Producer workgroups store their slabs write-through (sc1),
// drain, join a workgroup barrier and add 1 to the launch's arrival counter
// (agent scope) from one lane; a cell row polls that counter with sc1 loads
// from one lane, joins a barrier and then reads the slabs with sc1 loads
// only (CDNA4 guide, hand-off table row 1). Workgroups are dispatched in id
// order and the producers have the lowest ids and never wait, so every
// producer is resident or done by the time a waiting row is dispatched: the
// waits cannot deadlock on residency. Bounded like wait_flags.
__device__ __forceinline__ void chain_arrive(uint32_t* counter) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// SLEEP: s_sleep units (64 clocks each) between polls -- a longer period
// puts fewer poll requests beside the streams of the workgroups that are
// still producing (128 tiles polling one word every 64 clocks measurably
// slowed a chained launch's rows: scripts/micro/chain3_probe.py).
template <int SLEEP = 1>
__device__ inline void chain_wait(const uint32_t* counter, uint32_t target, int* err) {
    if (threadIdx.x == 0) {
        for (unsigned spins = 0;; spins += SLEEP) {
            if (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
            if ((spins & 255) == 255) {
                if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) break;
                if (spins > kHandoffSpinLimit) {
                    __hip_atomic_store(err, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
            __builtin_amdgcn_s_sleep(SLEEP);
        }
    }
    // compiler barrier + workgroup barrier: no wave's slab loads move above the poll
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __syncthreads();
}
// Rotating counters: launch k of a sequence uses counters[k] and zeroes
// counters[(k + 1) % n] (last used one call earlier, finished: launches on one
// stream are ordered), so every counter starts at zero when its launch runs
// and no reset launch is needed per call (n >= 2; zero-initialised once).
__device__ __forceinline__ void chain_rotate(uint32_t* counters, int n, int k) {
    if (threadIdx.x == 0) __hip_atomic_store(counters + (k + 1) % n, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Flag words are zeroed by a kernel, not hipMemsetAsync: on MI355X with
// torch's HIP 7.0 runtime a memset node captured into a HIP graph is not
// ordered before the next kernel node on replay (see csrc/lstm_persist.hip).
namespace {
__global__ void zero_flags(uint32_t* f, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) f[i] = 0u;
}
}  // namespace

// All workgroups of a persistent launch must be co-resident (they wait on
// each other): check the grid against the occupancy API.
inline bool grid_fits(const void* k, int threads, size_t lds, int grid, int max_per_cu = 2) {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, threads, lds) != hipSuccess)
        return false;
    return per >= 1 && grid <= cus * (per < max_per_cu ? per : max_per_cu);
}

}  // namespace skr
