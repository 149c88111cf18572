// Row-per-workgroup LayerNorm-LSTM cell kernels (forward and backward step):
// one workgroup owns one batch row, each thread V contiguous hidden units.
//
// Why: the clustered cell kernels (csrc/lstm_cell.hip) split a wide row over
// C workgroups and exchange the LayerNorm statistics in-launch through
// tagged global slots -- about 3 us per exchange on MI355X, two per
// backward step -- and load every operand as a scalar (2-4 bytes per lane:
// one vector-memory instruction per unit per operand). At the HyperLSTM
// shapes (H = 2048 main cell, H = 256 hyper cell, B = 100) the step is then
// bound by exchange latency and instruction issue, not bytes. Here every
// statistic is a workgroup reduction (DPP + LDS, no global exchange) and
// every operand is a 16-byte (fp32 x4, bf16 x8) or 8-byte (bf16 x4) vector
// load, all issued before the first use. A row block of 100 workgroups
// leaves CUs idle, but each one streams its row with few instructions.
//
// Semantics: identical expressions to cell_fwd_body / cell_bwd with LN
// (csrc/cell_fwd_body.h, csrc/lstm_cell.hip) -- LayerNorm over each gate
// block and over c (var = E[x^2] - mean^2, clamped, eps kLnEps), forget
// bias, stateless recurrent dropout on tanh(j) keyed by (seed, stream, step,
// b*H + u), the HyperLSTM modulation g = xh*ax + R*ah + bh + bias (MOD 3:
// precomputed by csrc/hyper_mod.hip with per-tile statistics). Reference
// cell: /root/reference model.py:19-27 (LayerNormLSTM / HyperLSTM cells
// inside the static unroll of model.py:66-95); no eoc resets on these paths
// (the VAE decoders), so `reset` must be null.
#include <cstdlib>

#include "row_cell.h"

namespace {

using namespace skr;

// ---- forward / backward step kernels (bodies: csrc/row_cell.h) -----------------------
template <int NT, int V, int MOD, int DS>
__global__ __launch_bounds__(NT) void row_fwd(const FwdArgs a) {
    row_fwd_body<NT, V, MOD, DS>(a, blockIdx.x);
}

template <int NT, int V, bool MOD, int DO>
__global__ __launch_bounds__(NT) void row_bwd(const BwdArgs a) {
    row_bwd_body<NT, V, MOD, DO>(a, blockIdx.x);
}

// ---- dispatch --------------------------------------------------------------------------
template <typename A>
using KernelT = void (*)(const A);


// Units per thread: 4 (rows up to 2048 units: <= 512 threads, no AGPR spill
// in the backward), 8 for wider rows.
int pick_v(int H) { return H > 2048 ? 8 : 4; }

#define SKR_ROW_GEOMS(X) X(64, 4) X(128, 4) X(256, 4) X(512, 4) X(256, 8) X(512, 8)

template <int MOD, int DS>
KernelT<FwdArgs> fwd_kernel(int nt, int v) {
#define SKR_ROW_CASE(NT_, V_) if (nt == NT_ && v == V_) return row_fwd<NT_, V_, MOD, DS>;
    SKR_ROW_GEOMS(SKR_ROW_CASE)
#undef SKR_ROW_CASE
    return nullptr;
}
template <bool MOD, int DO>
KernelT<BwdArgs> bwd_kernel(int nt, int v) {
#define SKR_ROW_CASE(NT_, V_) if (nt == NT_ && v == V_) return row_bwd<NT_, V_, MOD, DO>;
    SKR_ROW_GEOMS(SKR_ROW_CASE)
#undef SKR_ROW_CASE
    return nullptr;
}

}  // namespace

// Shape / layout support of the row kernels for a row of H units: 0 if
// supported, else the code the launchers return.
SKR_API int skr_row_supported(int H) {
    if (H < 256 || H % 256 != 0) return -2;
    const int v = pick_v(H), nt = H / v;
    return nt <= 512 ? 0 : -2;   // (1024-thread variants would spill at their 128-VGPR cap)
}

// Forward step. mod 0: g = xp + sum of R slabs; 3: precomputed g + per-tile
// statistics (csrc/hyper_mod.hip). LayerNorm cells only, no resets, bf16 or
// fp32 next-step operand (lp_kind 1 / 2); every pointer 16-byte aligned and
// every stride a multiple of 8 elements.
SKR_API int skr_row_fwd_step(const FwdArgs* args, int mod, hipStream_t s) {
    const FwdArgs& a = *args;
    if (a.B <= 0) return 0;
    if (skr_row_supported(a.H) != 0) return -2;
    const int rc = row_fwd_check(a, mod);
    if (rc) return rc;
    const int v = pick_v(a.H), nt = a.H / v;
    KernelT<FwdArgs> k = nullptr;
    if (mod == 3) k = fwd_kernel<3, 1>(nt, v);
    else if (a.R_nslab <= 1) k = fwd_kernel<0, 1>(nt, v);
    else if (a.R_nslab <= 2) k = fwd_kernel<0, 2>(nt, v);
    else if (a.R_nslab <= 4) k = fwd_kernel<0, 4>(nt, v);
    else k = fwd_kernel<0, 8>(nt, v);
    if (k == nullptr) return -2;
    hipLaunchKernelGGL(k, dim3(a.B), dim3(nt), 0, s, a);
    return SKR_CHECK_LAUNCH();
}

// Backward step. mod 0: LN-LSTM / hyper cell; 2: HyperLSTM main cell (bf16
// vec, bf16 R copy r_lp, bf16 dxp / dvec; vec_bias may be null = zero).
SKR_API int skr_row_bwd_step(const BwdArgs* args, int mod, hipStream_t s) {
    const BwdArgs& a = *args;
    if (a.B <= 0) return 0;
    if (skr_row_supported(a.H) != 0) return -2;
    const int rc = row_bwd_check(a, mod);
    if (rc) return rc;
    const int v = pick_v(a.H), nt = a.H / v;
    const bool wide = a.dh_out != nullptr && a.dho_nslab > 1;   // split-K dh_out (the hyper cell's dvec path)
    KernelT<BwdArgs> k = mod == 2 ? (wide ? bwd_kernel<true, 32>(nt, v) : bwd_kernel<true, 1>(nt, v))
                                  : (wide ? bwd_kernel<false, 32>(nt, v) : bwd_kernel<false, 1>(nt, v));
    if (k == nullptr) return -2;
    hipLaunchKernelGGL(k, dim3(a.B), dim3(nt), 0, s, a);
    return SKR_CHECK_LAUNCH();
}
