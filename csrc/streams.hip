// Stream utilities: CU-masked auxiliary streams.
//
// The backward scans of the recurrent layers are latency-bound chains of
// small launches that use a fraction of the chip at any moment, while their
// weight-gradient GEMMs are throughput work that only needs the per-step
// saves of steps already processed. The framework issues those GEMMs in
// chunks on an auxiliary stream while the scan continues. An unrestricted
// library GEMM would occupy every CU with long-running workgroups and stretch
// each scan step; a stream created with a CU mask confines it to a subset
// (hipExtStreamCreateWithCUMask), so the scan keeps the rest of the chip.
//
// The mask selects every `stride`-th CU starting at `first` (bit i of the
// mask = logical CU i), i.e. a spread-out subset of count/stride CUs.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <vector>

extern "C" {

// Creates a stream restricted to CUs {first, first+stride, ...} below n_cu.
// Returns 0 and writes the stream handle to *out, or a HIP error code.
int skr_stream_create_cumask(int n_cu, int first, int stride, void** out) {
    if (n_cu <= 0 || stride <= 0 || first < 0 || out == nullptr) return -1;
    std::vector<uint32_t> mask((n_cu + 31) / 32, 0u);
    int set = 0;
    for (int i = first; i < n_cu; i += stride) {
        mask[i / 32] |= 1u << (i % 32);
        ++set;
    }
    if (set == 0) return -2;
    hipStream_t s = nullptr;
    hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data());
    if (e != hipSuccess) return (int)e;
    *out = (void*)s;
    return 0;
}

int skr_stream_destroy(void* s) { return (int)hipStreamDestroy((hipStream_t)s); }

}  // extern "C"
