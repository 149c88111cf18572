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
//     2. the hyper LayerNorm cell (cell_fwd_body.h's arithmetic) with its
//        x-projection formed in-register from x (zp + x . w5, the per-sketch
//        z part zp precomputed once); its global loads are issued before 1.
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

// One row per workgroup, unit u = threadIdx.x (H <= 256). Every global load of
// the cell (R slabs, z projection, stroke weights, LayerNorm parameters,
// c) is issued BEFORE the sampler prologue -- none depends on the sampled
// stroke -- so its latency overlaps the head-slab fold and the draw. The
// arithmetic is cell_fwd_body<256, 1, NS, true, 0>'s (csrc/cell_fwd_body.h)
// with the x-projection formed from the stroke, term for term.
template <int NS>
__global__ __launch_bounds__(256) void decode_hyper_cell(const FwdArgs a, const DecodeSample s, float* __restrict__ x,
                                                         const float* __restrict__ w5, int64_t ldw5) {
    __shared__ float part[4][256];
    __shared__ float zrow[256];
    __shared__ float xr[8];
    __shared__ float red[4 * 8];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int H = a.H;
    const bool on = tid < H;
    const int u = on ? tid : H - 1;
    // ---- the cell's loads (clamped, never predicated)
    float zp[4], wv[4][5], rv[4], lg[4], lb[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int col = q * H + u;
        zp[q] = a.xp[b * a.ld_xp + col];
#pragma unroll
        for (int k = 0; k < 5; ++k) wv[q][k] = w5[k * ldw5 + col];
        rv[q] = slab_sum<NS>(a.R, b * a.ld_R + col, a.R_nslab, a.R_slab);
        lg[q] = a.ln_g[col];
        lb[q] = a.ln_b[col];
    }
    const float lcg = a.lnc_g[u], lcb = a.lnc_b[u];
    const float cp = a.c_prev[(int64_t)b * H + u];
    // ---- stroke t-1: fold + draw (or the given x)
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
    lds_barrier();
    // ---- gates: xp + x . w5 (skr_bproj_fwd's order) + R, LayerNorm per gate block
    float g[4], st[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        float xv = zp[q];
#pragma unroll
        for (int k = 0; k < 5; ++k) xv += xr[k] * wv[q][k];
        g[q] = xv + rv[q];
        const float v = on ? g[q] : 0.f;
        st[q] = v;
        st[4 + q] = v * v;
    }
    block_sum<8, 4>(st, red);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float mean = st[q] / (float)H;
        const float var = fmaxf(st[4 + q] / (float)H - mean * mean, 0.f);
        const float rs = rsqrtf(var + kLnEps);
        g[q] = ((g[q] - mean) * rs) * lg[q] + lb[q];
    }
    const float i = cell_sig(g[0]), tj = cell_tanh(g[1]), f = cell_sig(g[2] + a.forget_bias), o = cell_sig(g[3]);
    const float cn = on ? cp * f + i * tj : 0.f;     // (no dropout at inference)
    float s2[2] = {cn, cn * cn};
    block_sum<2, 4>(s2, red);
    const float mean = s2[0] / (float)H;
    const float var = fmaxf(s2[1] / (float)H - mean * mean, 0.f);
    const float rc = rsqrtf(var + kLnEps);
    const float h = cell_tanh(((cn - mean) * rc) * lcg + lcb) * o;
    if (!on) return;
    const int64_t ro = (int64_t)b * H + u;
    a.h_out[ro] = h;
    a.c_carry[ro] = cn;
    if (a.lp_kind == 1) ((__hip_bfloat16*)a.h_lp)[b * a.ld_lp + u] = to_bf16(h);
    else if (a.lp_kind == 2) ((float*)a.h_lp)[b * a.ld_lp + u] = h;
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
    if (a->H > 256 || a->cluster > 1 || a->ln_g == nullptr || x == nullptr || w5 == nullptr || a->keep < 1.0f ||
        a->reset != nullptr || a->xhat != nullptr || a->act != nullptr || a->c_carry == nullptr)
        return -2;
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
