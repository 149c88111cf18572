// Argument blocks of the fused LSTM-family cell kernels (csrc/lstm_cell.hip;
// a row runs on `cluster` workgroups). Mirrored field for field by
// sketch_rnn_amd/ops/_hipapi.py (size-checked at load).
#pragma once
#include "common.h"

namespace skr {

constexpr float kLnEps = 1e-3f;

struct FwdArgs {
    int B, H;
    int grp_rows;                      // rows per parameter group (0: one group)
    const float* xp; int64_t ld_xp;    // [B, 4H]: x-projection (+bias unless MOD)
    const float* R;  int64_t ld_R;     // [B, 4H]: h_prev @ W_h (fp32)
    int R_nslab; int64_t R_slab;       // R is the sum of R_nslab split-K partial slabs
    const void* vec; int64_t vec_gs; int64_t vec_ld;   // MOD: element (k,b,u) at k*gs + b*ld + u (mod 1 fp32, 2 bf16)
    const float* vec_bias;             // MOD: [12, H] added to vec (required)
    const float* bias;                 // MOD: [4H]
    const float* c_prev;               // [B, H]
    const float* ln_g; const float* ln_b; const float* lnc_g; const float* lnc_b;
    const float* reset;                // [B] or null
    const float* init_h; const float* init_c;
    float forget_bias, keep;
    const int64_t* seed; uint32_t stream, step;
    float* h_out;                      // [B, H]
    float* c_out;                      // [B, H]
    float* act;                        // [B, 4H] sig(i), tanh(j), sig(f+fb), sig(o)
    float* xhat;                       // LN: [B, 4H]
    float* rstd;                       // LN: [B, 5]
    float* chat;                       // LN: [B, H]
    float* h_carry;                    // [B, H]
    void* h_lp; int64_t ld_lp; int lp_kind;  // 0: none, 1: bf16, 2: fp32
    float* c_carry;                    // [B, H]
    // rows split over `cluster` workgroups (LayerNorm statistics exchanged in-launch)
    int cluster;                       // <= 1: one workgroup per row
    uint64_t* part;                    // [2][B][cluster][16] tagged partial statistics (zeroed per sequence)
    int* err;                          // set to 1 if a cluster wait timed out
    __hip_bfloat16* r_lp;              // MOD: bf16 copy of the summed R ([B, ld_R]) for the backward, or null
    // MOD 3 (HyperLSTM main cell after csrc/hyper_mod.hip): the gate
    // pre-activations g [B, 4H] and per-tile LayerNorm partial sums
    // [B][4][gstat_tiles][2] are precomputed -- no statistics exchange for
    // the gates; xp / R / vec / bias are not read
    const float* gpre; const float* gstats; int gstat_tiles;
    // LN saves in bf16 (xhat / chat buffers hold __hip_bfloat16; the forward
    // itself runs on the fp32 values, like a bf16 activation save)
    int save_lp;
    // MX-fp8 copy of the carried h (csrc/mx8_gemm.hip operand; null: none):
    // e4m3 bytes [B, ld_q8] and one E8M0 scale per 32 units in the
    // [B][4][H/128] layout (H % 128 == 0)
    uint8_t* h_q8; int64_t ld_q8; uint8_t* h_qs;
};

struct BwdArgs {
    int B, H;
    int grp_rows;
    const float* dh_out;               // [B, H] or null
    int dho_nslab; int64_t dho_slab;
    const float* dh_rec;               // [B, H] (grad into carried h_t) or null
    int64_t ld_dh_rec;
    int dhr_nslab; int64_t dhr_slab;
    const float* dh_rec2;              // second split-K source of the carried-h grad (added) or null
    int64_t ld_dh_rec2;
    int dhr2_nslab; int64_t dhr2_slab;
    float* dc_rec;                     // [B, H] in: grad into carried c_t; out: into carried c_{t-1}
    const float* act; const float* c_new; const float* c_prev;
    const float* xhat; const float* rstd; const float* chat;
    const float* ln_g; const float* lnc_g; const float* lnc_b;
    const float* xp; int64_t ld_xp;    // MOD: xh
    const float* R;  int64_t ld_R;     // MOD: R
    int R_nslab; int64_t R_slab;
    const void* vec; int64_t vec_gs; int64_t vec_ld;   // MOD (mod 1 fp32, 2 bf16)
    const float* vec_bias;
    const float* reset;
    float keep; const int64_t* seed; uint32_t stream, step;
    float* dG; int64_t ld_dG;          // non-MOD: d(preact) [B, 4H]; MOD: dR = dg*ah
    void* dG_lp; int64_t ld_dG_lp; int dG_lp_kind;  // bf16 copy of dG for the next GEMM (1) or none (0)
    void* dxp; int64_t ld_dxp; int dxp_kind;  // MOD: dxh = dg*ax (1 bf16, 2 fp32)
    void* dvec; int dvec_kind;         // MOD: same layout as vec; 1 bf16, 2 fp32
    float* dlny;                       // LN: [B, 4H] grad wrt LN-all output (for gamma/beta)
    float* dlncy;                      // LN: [B, H]  grad wrt LN(c) output
    float* dinit_h; float* dinit_c;    // [B, H] accumulated on reset rows (or null)
    int cluster; uint64_t* part; int* err;
    // LN: the gate activations are recomputed from xhat (the forward does not
    // store them): act = sig/tanh(xhat * ln_g + ln_b (+ forget_bias on f))
    const float* ln_b; float forget_bias;
    const __hip_bfloat16* r_lp;        // MOD: R from the forward's bf16 copy (stride ld_R) instead of the slabs
    int save_lp;                       // LN: xhat / chat read and dlny / dlncy written as bf16
    int xp_lp;                         // MOD: xp (xh) stored as bf16 (the fused-modulation training path)
};

// Gate / cell activations of the LSTM-family cell kernels: the hardware
// exp2 + reciprocal forms (common.h sigmoid_fast / tanh_fast, ~1e-7 absolute
// error, a few VALU ops instead of ~25-45 for expf + IEEE division / tanhf);
// -DSKR_EXACT_ACT builds the IEEE forms (A/B and numerics experiments).
#ifdef SKR_EXACT_ACT
__device__ __forceinline__ float cell_sig(float x) { return sigmoidf_(x); }
__device__ __forceinline__ float cell_tanh(float x) { return tanhf(x); }
#else
__device__ __forceinline__ float cell_sig(float x) { return sigmoid_fast(x); }
__device__ __forceinline__ float cell_tanh(float x) { return tanh_fast(x); }
#endif

// hyper modulation vectors: MOD 1 fp32, MOD 2 bf16
template <int MOD>
__device__ __forceinline__ float ldvec(const void* v, int64_t i) {
    if constexpr (MOD == 2) return __bfloat162float(((const __hip_bfloat16*)v)[i]);
    else return ((const float*)v)[i];
}

// LN saves: fp32 or (lp) bf16 element i. The load is branch-free (one
// dword load + selects): the cells issue every load up front, and a branch
// between two loads would split that batch.
__device__ __forceinline__ float ld_save(const void* p, int64_t i, bool lp) {
    const int64_t off = lp ? (i << 1) : (i << 2);
    const uint32_t w = *(const uint32_t*)((const char*)p + (off & ~(int64_t)3));
    return __uint_as_float(lp ? ((off & 2) ? (w & 0xffff0000u) : (w << 16)) : w);
}
__device__ __forceinline__ void st_save(void* p, int64_t i, float v, bool lp) {
    if (lp) ((__hip_bfloat16*)p)[i] = __float2bfloat16(v);
    else ((float*)p)[i] = v;
}

__device__ __forceinline__ float dropout_mult(bool on, uint32_t key, int64_t idx, float keep) {
    if (!on) return 1.f;
    return hash_uniform(key, (uint32_t)idx) < keep ? 1.0f / keep : 0.f;
}

}  // namespace skr
