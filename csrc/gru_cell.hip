// Fused GRU and vanilla-RNN cell steps (forward + backward) for gfx950:
// the reference's `--model gru` / `--model rnn` layers (model.py:16-23,
// TF GRUCell / BasicRNNCell semantics, sketch_rnn_amd/models/cells.py),
// with the same eoc state reset to the batch-initial state (model.py:82-92).
//
// GRU step t (input projections hoisted out of the scan):
//   [r, u] = sig(xg + h @ W_gh)            xg = x @ W_gx + b_g
//   c      = tanh(xc + (r*h) @ W_ch)       xc = x @ W_cx + b_c
//   h'     = u*h + (1-u)*c ;  carry = reset ? init : h'
// The candidate's GEMM operand r*h depends on the gate GEMM, so a step is
// GEMM -> gates kernel -> GEMM -> output kernel; the backward mirrors it
// (output-side kernel -> GEMM -> gate-side kernel -> GEMM). RNN step:
// h' = tanh(xp + h @ W_h), one GEMM + one kernel each way.
//
// Every GEMM result arrives as split-K partial slabs (csrc/skinny_gemm.hip)
// summed while loading; all loads of a thread are issued before first use.
// Elementwise: grid (ceil(H/256), B), one hidden unit per thread.
#include "common.h"

namespace {

using namespace skr;

struct Slabs {
    const float* p;
    int64_t ld;
    int n;
    int64_t slab;
    __device__ __forceinline__ float at(int b, int u) const {
        return p ? slab_sum<0>(p, (int64_t)b * ld + u, n, slab) : 0.f;
    }
};

__device__ __forceinline__ void store_lp(void* dst, int kind, int64_t i, float v) {
    if (kind == 1) ((__hip_bfloat16*)dst)[i] = to_bf16(v);
    else if (kind == 2) ((float*)dst)[i] = v;
}

}  // namespace

// ---- argument blocks (mirrored by sketch_rnn_amd/ops/_hipapi.py) ------------------------
struct GruFwdArgs {
    int B, H;
    const float* xg; int64_t ld_xg;            // [B, 2H] (GRU) | xp [B, H] (RNN)
    const float* Rg; int64_t ld_Rg; int Rg_nslab; int64_t Rg_slab;
    const float* xc; int64_t ld_xc;            // [B, H] (GRU)
    const float* Rc; int64_t ld_Rc; int Rc_nslab; int64_t Rc_slab;
    const float* h_prev;                       // [B, H] carried h (fp32)
    const float* reset; const float* init_h;
    float* ru;                                 // [B, 2H] sig(r), sig(u)
    void* rh_lp; int64_t ld_rh; int rh_kind;   // GEMM operand r*h: 1 bf16, 2 fp32
    float* cand;                               // [B, H] candidate (GRU) | h' (RNN)
    float* h_out;                              // [B, H] cell output
    float* h_carry;                            // [B, H]
    void* h_lp; int64_t ld_lp; int lp_kind;    // next step's GEMM operand
};

struct GruBwdArgs {
    int B, H;
    const float* dh_out;                       // [B, H] loss grad into h'_t (or null)
    const float* dh_elem;                      // [B, H] elementwise part of the carried grad (or null)
    const float* dhg; int64_t ld_dhg; int dhg_nslab; int64_t dhg_slab;  // GEMM part of the carried grad
    const float* ru; const float* cand; const float* h_prev;
    const float* reset;
    float* dinit_h;                            // reset rows accumulate the carried grad (or null)
    float* dh_tot;                             // [B, H] total grad into h'_t
    float* dpc; void* dpc_lp; int dpc_kind;    // [B, H] grad of the candidate pre-activation (RNN: of h pre-act)
    const float* drh; int64_t ld_drh; int drh_nslab; int64_t drh_slab;  // dpc @ W_ch^T slabs
    float* dpg; void* dpg_lp; int dpg_kind;    // [B, 2H] grad of the gate pre-activations
    float* dh_elem_out;                        // [B, H] -> next (earlier) step's dh_elem
};

namespace {

// dh' = dh_out + (reset ? 0 : carried), carried = dh_elem + GEMM slabs
__device__ __forceinline__ float total_dh(const GruBwdArgs& a, int b, int u, int64_t ro, bool r) {
    const float carried = (a.dh_elem ? a.dh_elem[ro] : 0.f) +
                          Slabs{a.dhg, a.ld_dhg, a.dhg_nslab, a.dhg_slab}.at(b, u);
    if (r && a.dinit_h) a.dinit_h[ro] += carried;
    return (a.dh_out ? a.dh_out[ro] : 0.f) + (r ? 0.f : carried);
}

__global__ __launch_bounds__(256) void gru_fwd_gates(const GruFwdArgs a) {
    const int b = blockIdx.y, u = blockIdx.x * 256 + threadIdx.x, H = a.H;
    if (u >= H) return;
    const Slabs R{a.Rg, a.ld_Rg, a.Rg_nslab, a.Rg_slab};
    const float xr = a.xg[b * a.ld_xg + u], xu = a.xg[b * a.ld_xg + H + u];
    const float rr = R.at(b, u), ru = R.at(b, H + u);
    const float h = a.h_prev[(int64_t)b * H + u];
    const float r = sigmoidf_(xr + rr), z = sigmoidf_(xu + ru);
    a.ru[(int64_t)b * 2 * H + u] = r;
    a.ru[(int64_t)b * 2 * H + H + u] = z;
    store_lp(a.rh_lp, a.rh_kind, (int64_t)b * a.ld_rh + u, r * h);
}

__global__ __launch_bounds__(256) void gru_fwd_out(const GruFwdArgs a) {
    const int b = blockIdx.y, u = blockIdx.x * 256 + threadIdx.x, H = a.H;
    if (u >= H) return;
    const bool rs = a.reset != nullptr && a.reset[b] != 0.f;
    const int64_t ro = (int64_t)b * H + u;
    const float xc = a.xc[b * a.ld_xc + u];
    const float rc = Slabs{a.Rc, a.ld_Rc, a.Rc_nslab, a.Rc_slab}.at(b, u);
    const float z = a.ru[(int64_t)b * 2 * H + H + u];
    const float h = a.h_prev[ro];
    const float c = tanhf(xc + rc);
    const float hn = z * h + (1.f - z) * c;
    a.cand[ro] = c;
    a.h_out[ro] = hn;
    const float hc = rs ? a.init_h[ro] : hn;
    a.h_carry[ro] = hc;
    store_lp(a.h_lp, a.lp_kind, (int64_t)b * a.ld_lp + u, hc);
}

// backward, output side: dh' -> dpc (-> GEMM dpc @ W_ch^T)
__global__ __launch_bounds__(256) void gru_bwd_out(const GruBwdArgs a) {
    const int b = blockIdx.y, u = blockIdx.x * 256 + threadIdx.x, H = a.H;
    if (u >= H) return;
    const bool rs = a.reset != nullptr && a.reset[b] != 0.f;
    const int64_t ro = (int64_t)b * H + u;
    const float z = a.ru[(int64_t)b * 2 * H + H + u];
    const float c = a.cand[ro];
    const float dh = total_dh(a, b, u, ro, rs);
    a.dh_tot[ro] = dh;
    const float dpc = dh * (1.f - z) * (1.f - c * c);
    a.dpc[ro] = dpc;
    store_lp(a.dpc_lp, a.dpc_kind, ro, dpc);
}

// backward, gate side: d(r*h) -> dpg (-> GEMM dpg @ W_gh^T) and the elementwise carried grad
__global__ __launch_bounds__(256) void gru_bwd_gates(const GruBwdArgs a) {
    const int b = blockIdx.y, u = blockIdx.x * 256 + threadIdx.x, H = a.H;
    if (u >= H) return;
    const int64_t ro = (int64_t)b * H + u;
    const float drh = Slabs{a.drh, a.ld_drh, a.drh_nslab, a.drh_slab}.at(b, u);
    const float r = a.ru[(int64_t)b * 2 * H + u], z = a.ru[(int64_t)b * 2 * H + H + u];
    const float h = a.h_prev[ro], c = a.cand[ro], dh = a.dh_tot[ro];
    const float dr = drh * h * r * (1.f - r);
    const float dz = dh * (h - c) * z * (1.f - z);
    a.dpg[(int64_t)b * 2 * H + u] = dr;
    a.dpg[(int64_t)b * 2 * H + H + u] = dz;
    store_lp(a.dpg_lp, a.dpg_kind, (int64_t)b * 2 * H + u, dr);
    store_lp(a.dpg_lp, a.dpg_kind, (int64_t)b * 2 * H + H + u, dz);
    a.dh_elem_out[ro] = dh * z + drh * r;
}

// vanilla RNN: h' = tanh(xp + R)
__global__ __launch_bounds__(256) void rnn_fwd(const GruFwdArgs a) {
    const int b = blockIdx.y, u = blockIdx.x * 256 + threadIdx.x, H = a.H;
    if (u >= H) return;
    const bool rs = a.reset != nullptr && a.reset[b] != 0.f;
    const int64_t ro = (int64_t)b * H + u;
    const float hn = tanhf(a.xg[b * a.ld_xg + u] + Slabs{a.Rg, a.ld_Rg, a.Rg_nslab, a.Rg_slab}.at(b, u));
    a.cand[ro] = hn;
    a.h_out[ro] = hn;
    const float hc = rs ? a.init_h[ro] : hn;
    a.h_carry[ro] = hc;
    store_lp(a.h_lp, a.lp_kind, (int64_t)b * a.ld_lp + u, hc);
}

__global__ __launch_bounds__(256) void rnn_bwd(const GruBwdArgs a) {
    const int b = blockIdx.y, u = blockIdx.x * 256 + threadIdx.x, H = a.H;
    if (u >= H) return;
    const bool rs = a.reset != nullptr && a.reset[b] != 0.f;
    const int64_t ro = (int64_t)b * H + u;
    const float hn = a.cand[ro];
    const float dh = total_dh(a, b, u, ro, rs);
    const float dp = dh * (1.f - hn * hn);
    a.dpc[ro] = dp;
    store_lp(a.dpc_lp, a.dpc_kind, ro, dp);
}

template <typename K, typename A>
int launch(K k, const A& a, hipStream_t s) {
    if (a.B <= 0) return 0;
    hipLaunchKernelGGL(k, dim3((a.H + 255) / 256, a.B), dim3(256), 0, s, a);
    return SKR_CHECK_LAUNCH();
}

}  // namespace

// phase: 0 = GRU gates, 1 = GRU output, 2 = RNN
SKR_API int skr_gru_fwd(const GruFwdArgs* a, int phase, hipStream_t s) {
    switch (phase) {
        case 0: return launch(gru_fwd_gates, *a, s);
        case 1: return launch(gru_fwd_out, *a, s);
        case 2: return launch(rnn_fwd, *a, s);
        default: return -2;
    }
}

// phase: 0 = GRU output side, 1 = GRU gate side, 2 = RNN
SKR_API int skr_gru_bwd(const GruBwdArgs* a, int phase, hipStream_t s) {
    switch (phase) {
        case 0: return launch(gru_bwd_out, *a, s);
        case 1: return launch(gru_bwd_gates, *a, s);
        case 2: return launch(rnn_bwd, *a, s);
        default: return -2;
    }
}

SKR_API int skr_gru_fwd_args_size() { return (int)sizeof(GruFwdArgs); }
SKR_API int skr_gru_bwd_args_size() { return (int)sizeof(GruBwdArgs); }
