// Decode-step hyper cell with the previous stroke's sampler folded in
// (sample/hyper_step.py, four launches per stroke).
//
// The HyperLSTM decode step (reference per-stroke loop model.py:213-249,
// sample_sketch in sketch_rnn's sample code) is a chain of dependent,
// latency-bound launches. Stroke t needs x_t, which is sampled from the
// head of h_{t-1}; the head GEMM h_{t-1} W_out needs nothing the step's own
// recurrent GEMMs do not also read, so it rides in the same grouped skinny
// GEMM launch as h W_h and [h | hh] W_y (csrc/skinny_gemm.hip), and the
// sampler of stroke t-1 runs at the top of THIS kernel:
//
//   workgroup b (one row, 256 threads):
//     1. (sampling on) fold the head's split-K slabs + bias (mdn_sample.h
//        fold_head_slabs), wave 0 draws the stroke (mdn_sample_wave: the same
//        keyed hash draws as skr_mdn_sample_slabs, so a stroke is the same
//        whichever kernel samples it), lane 0 writes out[b][t-1], done[b]
//        and x[b]; the 5 values meet the rest of the workgroup in LDS;
//        (sampling off) x[b] is read (t == 0, or teacher-forced steps);
//     2. the hyper LayerNorm cell (cell_fwd_body.h) with its x-projection
//        formed in-register from x (zp + x . w5, the per-sketch z part zp
//        precomputed once).
//
// Stroke chain: [R_main, R_hyp, head(h_{t-1})] GEMM -> this kernel ->
// hyper_mod (csrc/hyper_mod.hip, decode inputs) -> main cell (MOD 3); after
// the last stroke one head GEMM + skr_mdn_sample_slabs.
#include "cell_fwd_body.h"
#include "mdn_sample.h"

struct DecodeSample {
    int active;                        // 0: x is an input (no sampling)
    const float* zs; int64_t ldz; int nslab; int64_t slab;   // head slabs [nslab][B][ldz]
    const float* bias; int nout;
    int M, mode; float temp; int greedy, fix_pen;
    const int64_t* seed; uint32_t step; int row0;            // hash key (global row = row0 + b)
    float* out_row; int64_t ld_out;    // out[b] = stroke of step `step` (row stride ld_out)
    int* done;                         // [B] eos reached
};

namespace {

template <int NS>
__global__ __launch_bounds__(256) void decode_hyper_cell(const FwdArgs a, const DecodeSample s, float* __restrict__ x,
                                                         const float* __restrict__ w5, int64_t ldw5) {
    __shared__ float part[4][256];
    __shared__ float zrow[256];
    __shared__ float xr[8];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (s.active) {
        skr::fold_head_slabs(s.zs, s.ldz, s.nslab, s.slab, s.bias, s.nout, b, part, zrow);
        if (w == 0) {
            const uint32_t key = skr::hash_key(*s.seed, 0x5A3Du, s.step);
            const skr::MdnDraw d =
                skr::mdn_sample_wave(zrow, s.M, s.mode, s.temp, s.greedy, s.fix_pen, key, (uint32_t)(s.row0 + b), s.step);
            if (lane == 0) {
                const int stop_col = s.mode == 1 ? 4 : 3;   // p3 | eoc
                float* o = s.out_row + b * s.ld_out;
                const bool was_done = s.done[b] != 0;
                for (int k = 0; k < 5; ++k) {
                    o[k] = was_done ? (k == stop_col ? 1.f : 0.f) : d.row[k];
                    x[b * 5 + k] = d.row[k];
                    xr[k] = d.row[k];
                }
                if (d.pidx + 2 == stop_col) s.done[b] = 1;
            }
        }
    } else if (tid < 5) {
        xr[tid] = x[b * 5 + tid];
    }
    __syncthreads();
    cell_fwd_body<256, 1, NS, true, 0>(a, 0, b, 1, xr, w5, ldw5);
}

}  // namespace

// a: the hyper cell's forward args (LayerNorm, H <= 256, one workgroup per
// row: a.cluster <= 1; a.xp = the per-sketch z projection zp [B][ld_xp]),
// s: the sampler of the previous stroke (s->active == 0: x [B][5] is read),
// x [B][5] fp32 (in/out), w5 [5][ldw5] fp32 stroke rows of the hyper cell's
// input weights (column offset applied by the caller, like a.xp).
SKR_API int skr_decode_hyper_cell(const FwdArgs* a, const DecodeSample* s, float* x, const float* w5, int64_t ldw5,
                                  hipStream_t st) {
    if (a->B <= 0) return 0;
    if (a->H > 256 || a->cluster > 1 || a->ln_g == nullptr || x == nullptr || w5 == nullptr) return -2;
    if (s->active && (s->nout > 256 || s->M > 64 || s->nslab < 1 || s->zs == nullptr || s->done == nullptr ||
                      s->out_row == nullptr || s->seed == nullptr))
        return -3;
    const dim3 grid(a->B), blk(256);
    switch (a->R_nslab) {
        case 1: hipLaunchKernelGGL(decode_hyper_cell<1>, grid, blk, 0, st, *a, *s, x, w5, ldw5); break;
        case 2: hipLaunchKernelGGL(decode_hyper_cell<2>, grid, blk, 0, st, *a, *s, x, w5, ldw5); break;
        case 4: hipLaunchKernelGGL(decode_hyper_cell<4>, grid, blk, 0, st, *a, *s, x, w5, ldw5); break;
        case 8: hipLaunchKernelGGL(decode_hyper_cell<8>, grid, blk, 0, st, *a, *s, x, w5, ldw5); break;
        default: hipLaunchKernelGGL(decode_hyper_cell<0>, grid, blk, 0, st, *a, *s, x, w5, ldw5); break;
    }
    return SKR_CHECK_LAUNCH();
}

SKR_API int skr_decode_sample_size() { return (int)sizeof(DecodeSample); }
