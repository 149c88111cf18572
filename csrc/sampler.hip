// On-device MDN sampler (reference capability R14, model.py:187-264).
//
// One wave per batch row. From the head output z [B, 3 + 6M] it draws a
// stroke (csrc/mdn_sample.h, shared with the fused decoder), then writes
// (a) the sampled stroke row into the output sequence and (b) the next
// decoder input -- so an N-step decode loop never returns to the host
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
#include "mdn_sample.h"

namespace {

__global__ __launch_bounds__(64) void mdn_sample_kernel(const float* __restrict__ z, int64_t ldz, int M, int mode,
                                                        float temp, int greedy, int fix_pen, const int64_t* seed,
                                                        uint32_t step, float* __restrict__ out_row, int64_t ld_out,
                                                        float* __restrict__ next_x, int64_t ld_next,
                                                        int* __restrict__ done, float* __restrict__ params) {
    const int b = blockIdx.x, lane = threadIdx.x;
    const uint32_t key = skr::hash_key(*seed, 0x5A3Du, step);
    const skr::MdnDraw d = skr::mdn_sample_wave(z + b * ldz, M, mode, temp, greedy, fix_pen, key, (uint32_t)b, step);
    if (lane != 0) return;
    const bool was_done = done[b] != 0;
    float* o = out_row + b * ld_out;
    if (was_done) {
        // finished rows emit end-of-sketch padding
        for (int k = 0; k < 5; ++k) o[k] = 0.f;
        o[mode == 1 ? 4 : 3] = 1.f;
    } else {
        for (int k = 0; k < 5; ++k) o[k] = d.row[k];
    }
    float* nx = next_x + b * ld_next;
    for (int k = 0; k < 5; ++k) nx[k] = d.row[k];
    const int stop_col = mode == 1 ? 4 : 3;  // p3 | eoc
    if (d.pidx + 2 == stop_col) done[b] = 1;
    if (params) {
        float* p = params + b * 4;
        p[0] = (float)d.idx;
        p[1] = (float)d.pidx;
        p[2] = d.s1;
        p[3] = d.s2;
    }
}

// Same, with z given as the sum of `nslab` split-K partial slabs of a head
// GEMM without bias (csrc/skinny_gemm.hip, z = h @ W_out in slabs) plus the
// bias. One 256-thread workgroup per row: wave w folds the slabs s = w mod 4
// of every column with independent (unrolled, clamped) loads, the four
// partial rows meet in LDS, then wave 0 samples.
__global__ __launch_bounds__(256) void mdn_sample_slabs_kernel(const float* __restrict__ zs, int64_t ldz, int nslab,
                                                               int64_t slab, const float* __restrict__ bias, int nout,
                                                               int M, int mode, float temp, int greedy, int fix_pen,
                                                               const int64_t* seed, uint32_t step, int row0,
                                                               float* __restrict__ out_row, int64_t ld_out,
                                                               float* __restrict__ next_x, int64_t ld_next,
                                                               int* __restrict__ done) {
    __shared__ float part[4][256];
    __shared__ float zrow[256];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    skr::fold_head_slabs(zs, ldz, nslab, slab, bias, nout, b, part, zrow);
    if (w != 0) return;
    const uint32_t key = skr::hash_key(*seed, 0x5A3Du, step);
    const skr::MdnDraw d = skr::mdn_sample_wave(zrow, M, mode, temp, greedy, fix_pen, key, (uint32_t)(row0 + b), step);
    if (lane != 0) return;
    const int stop_col = mode == 1 ? 4 : 3;  // p3 | eoc
    float* o = out_row + b * ld_out;
    const bool was_done = done[b] != 0;
    for (int k = 0; k < 5; ++k) o[k] = was_done ? (k == stop_col ? 1.f : 0.f) : d.row[k];
    float* nx = next_x + b * ld_next;
    for (int k = 0; k < 5; ++k) nx[k] = d.row[k];
    if (d.pidx + 2 == stop_col) done[b] = 1;
}

}  // namespace

SKR_API int skr_mdn_sample_slabs(const float* zs, int64_t ldz, int nslab, int64_t slab, const float* bias, int B,
                                 int M, int mode, float temp, int greedy, int fix_pen, const int64_t* seed,
                                 uint32_t step, int row0, float* out_row, int64_t ld_out, float* next_x,
                                 int64_t ld_next, int* done, hipStream_t s) {
    if (M < 1 || M > 32 || nslab < 1) return -2;
    if (B <= 0) return 0;
    hipLaunchKernelGGL(mdn_sample_slabs_kernel, dim3(B), dim3(256), 0, s, zs, ldz, nslab, slab, bias, 3 + 6 * M, M,
                       mode, temp, greedy, fix_pen, seed, step, row0, out_row, ld_out, next_x, ld_next, done);
    return SKR_CHECK_LAUNCH();
}

SKR_API int skr_mdn_sample(const float* z, int64_t ldz, int B, int M, int mode, float temp, int greedy, int fix_pen,
                           const int64_t* seed, uint32_t step, float* out_row, int64_t ld_out, float* next_x,
                           int64_t ld_next, int* done, float* params, hipStream_t s) {
    if (M < 1 || M > 32) return -2;
    if (B <= 0) return 0;
    hipLaunchKernelGGL(mdn_sample_kernel, dim3(B), dim3(64), 0, s, z, ldz, M, mode, temp, greedy, fix_pen, seed, step,
                       out_row, ld_out, next_x, ld_next, done, params);
    return SKR_CHECK_LAUNCH();
}
