// Fused LSTM step for small hidden sizes (H = 256 / 512, no LayerNorm):
// the recurrent GEMM and the cell update in ONE launch per time step.
//
// At H <= 512 the per-step work is tiny (the bidirectional encoder: 2 x
// [100 x 512] x [512 x 2048]) and a GEMM launch + a cell launch are both
// latency-bound; fusing removes one launch, the fp32 partial slabs and their
// round trip through memory. A workgroup owns 16 hidden units x 32 rows of
// one direction: it stages h_{t-1}[32 rows, H] and the 64 matching columns
// of W_h (4 gates x 16 units) in LDS with global_load_lds_dwordx4 (rows XOR-
// swizzled by (row & 15) on the source address), each of the 4 waves
// computes one gate's [32 x 16] tile with v_mfma_f32_16x16x32_bf16, the
// tiles meet in LDS and every thread finishes the cell for 2 (row, unit)
// pairs -- the inputs of that epilogue (x-projection, c_{t-1}) are loaded
// before the GEMM so their latency hides under it.
//
// Semantics and saves are identical to csrc/lstm_cell.hip (plain LSTM path):
// forget bias, stateless dropout on tanh(j) keyed (seed, stream, step,
// row*H + u), eoc reset of the carried state, bf16 copy of the carried h for
// the next step. Grid (H/16, ceil(B/32), nd).
#include <cstdlib>

#include "lstm_args.h"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

}  // namespace

struct FusedFwdArgs {
    int B, H, nd;                           // B rows per group, nd groups (encoder directions)
    const __hip_bfloat16* A; int64_t lda;   // h_{t-1} operand, [nd*B, H]
    const __hip_bfloat16* WT; int64_t w_gs; // B^T of W_h per group: [4H, H], group stride w_gs
    const float* xp; int64_t ld_xp;         // [nd*B, 4H] input projection (+ bias)
    const float* c_prev;                    // [nd*B, H]
    const float* reset;                     // [nd*B] or null
    const float* init_h; const float* init_c;
    float forget_bias, keep;
    const int64_t* seed; uint32_t stream, step;
    float* h_out; float* c_out; float* act; // act [nd*B, 4H]
    float* h_carry; float* c_carry;
    __hip_bfloat16* h_next; int64_t ld_next;
};

// Backward step t: dh_rec = dG_{t+1} @ W_h^T (K = 4H) fused with the cell
// backward of step t. Operands are read straight from L2 into MFMA fragments
// (no LDS staging: K is split over the NW waves and each wave streams only
// its slice); the NW partial tiles are summed in LDS by the epilogue.
struct FusedBwdArgs {
    int B, H, nd;
    const __hip_bfloat16* dG_next; int64_t ld_dgn;  // bf16 dG of step t+1 [nd*B, 4H], null at t = T-1
    const __hip_bfloat16* W; int64_t w_gs;          // W_h per group [H, 4H], group stride w_gs
    const float* dh_extra;                          // [nd*B, H] added to dh_rec (dh_T at t = T-1) or null
    const float* dh_out;                            // [nd*B, H] or null
    float* dc_rec;                                  // [nd*B, H] in: dc from step t+1, out: dc into step t-1
    const float* act; const float* c_new; const float* c_prev;
    const float* reset;
    float keep; const int64_t* seed; uint32_t stream, step;
    float* dG; __hip_bfloat16* dG_lp;               // [nd*B, 4H]
    float* dinit_h; float* dinit_c;                 // [nd*B, H] accumulated on reset rows (or null)
};

namespace {

using namespace skr;

constexpr int RB = 32, UB = 16;   // rows x units per workgroup

template <int H>
__global__ __launch_bounds__(256) void lstm_fused_fwd(const FusedFwdArgs a) {
    constexpr int CPR = H / 8;                 // 16-byte chunks per K-row
    constexpr int ROWS_PER_G = 64 / CPR;       // rows one glds wave-instruction covers
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __hip_bfloat16* As = (__hip_bfloat16*)smem;            // [RB][H]
    __hip_bfloat16* Ws = As + RB * H;                       // [4*UB][H]
    float* gates = (float*)(Ws + 4 * UB * H);               // [4][RB][UB]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int grp = blockIdx.z, rb = blockIdx.y * RB, u0 = blockIdx.x * UB;
    const int B = a.B;
    const int64_t row0 = (int64_t)grp * B;

    // ---- stage h_{t-1} rows and the 64 W columns (glds, swizzled on the source)
    {
        const int sub = lane / CPR, ch = lane % CPR;
        for (int r = w * ROWS_PER_G; r < RB; r += 4 * ROWS_PER_G) {
            const int row = r + sub;
            const int src = min(rb + row, B - 1);
            const __hip_bfloat16* g = a.A + (row0 + src) * a.lda + ((ch ^ (row & 15)) * 8);
            __builtin_amdgcn_global_load_lds((const void*)g, (__attribute__((address_space(3))) void*)(As + r * H),
                                             16, 0, 0);
        }
        const __hip_bfloat16* Wg = a.WT + grp * a.w_gs;
        for (int r = w * ROWS_PER_G; r < 4 * UB; r += 4 * ROWS_PER_G) {
            const int row = r + sub;                         // row = q*16 + unit
            const int n = (row / UB) * a.H + u0 + (row % UB);
            const __hip_bfloat16* g = Wg + (int64_t)n * H + ((ch ^ (row & 15)) * 8);
            __builtin_amdgcn_global_load_lds((const void*)g, (__attribute__((address_space(3))) void*)(Ws + r * H),
                                             16, 0, 0);
        }
    }
    // ---- epilogue inputs, loaded before the GEMM (2 (row, unit) pairs per thread)
    const bool keep_on = a.keep < 1.0f;
    const uint32_t key = keep_on ? hash_key(*a.seed, a.stream, a.step) : 0u;
    float xv[2][4], cp[2];
    int br[2], uu[2];
    bool on[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int p = tid + 256 * k, r = p / UB;
        uu[k] = p % UB;
        on[k] = rb + r < B;
        br[k] = (int)row0 + min(rb + r, B - 1);
        const int u = u0 + uu[k];
#pragma unroll
        for (int q = 0; q < 4; ++q) xv[k][q] = a.xp[(int64_t)br[k] * a.ld_xp + q * a.H + u];
        cp[k] = a.c_prev[(int64_t)br[k] * a.H + u];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();

    // ---- wave w: gate w, [32 rows x 16 units], K = H
    const int fr = lane & 15, fq = lane >> 4;
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll 4
    for (int ks = 0; ks < H / 32; ++ks) {
        const int c = ks * 4 + fq;
        const int wrow = w * UB + fr;
        const bf16x8 bfr = *(const bf16x8*)(&Ws[wrow * H + ((c ^ (wrow & 15)) * 8)]);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int arow = 16 * i + fr;
            const bf16x8 af = *(const bf16x8*)(&As[arow * H + ((c ^ (arow & 15)) * 8)]);
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc[i], 0, 0, 0);
        }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) gates[(w * RB + 16 * i + fq * 4 + e) * UB + fr] = acc[i][e];
    lds_barrier();

    // ---- cell update for this thread's 2 (row, unit) pairs
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        if (!on[k]) continue;
        const int p = tid + 256 * k, r = p / UB;
        const int b = br[k], u = u0 + uu[k];
        float g[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) g[q] = gates[(q * RB + r) * UB + uu[k]] + xv[k][q];
        const float i = sigmoidf_(g[0]), tj = tanhf(g[1]), f = sigmoidf_(g[2] + a.forget_bias), o = sigmoidf_(g[3]);
        const int64_t ro = (int64_t)b * a.H + u;
        const float m = dropout_mult(keep_on, key, ro, a.keep);
        const float cn = cp[k] * f + i * tj * m;
        const float h = tanhf(cn) * o;
        float* ap = a.act + (int64_t)b * 4 * a.H + u;
        ap[0] = i;
        ap[a.H] = tj;
        ap[2 * a.H] = f;
        ap[3 * a.H] = o;
        a.c_out[ro] = cn;
        a.h_out[ro] = h;
        const bool rs = a.reset != nullptr && a.reset[b] != 0.f;
        const float hc = rs ? a.init_h[ro] : h;
        if (a.h_carry != nullptr) a.h_carry[ro] = hc;   // (== h_out without resets: callers skip it)
        a.c_carry[ro] = rs ? a.init_c[ro] : cn;
        a.h_next[(int64_t)b * a.ld_next + u] = to_bf16(hc);
    }
}

// NW waves split K = 4H (each streams K/NW straight from L2 into MFMA
// fragments, loop fully unrolled so all of a wave's loads are in flight
// before its first MFMA); the NW partial tiles meet in LDS; each of the
// 64*NW threads finishes 512/(64*NW) (row, unit) pairs.
template <int H, int NW>
__global__ __launch_bounds__(64 * NW) void lstm_fused_bwd(const FusedBwdArgs a) {
    constexpr int K = 4 * H, KW = K / NW;   // K per wave
    constexpr int NTH = 64 * NW, P = RB * UB / NTH;
    __shared__ float red[NW][RB][UB + 1];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int grp = blockIdx.z, rb = blockIdx.y * RB, u0 = blockIdx.x * UB;
    const int B = a.B;
    const int64_t row0 = (int64_t)grp * B;
    const bool keep_on = a.keep < 1.0f;
    const uint32_t key = keep_on ? hash_key(*a.seed, a.stream, a.step) : 0u;

    // ---- epilogue inputs first (P (row, unit) pairs per thread)
    float ac[P][4], cx[P], cp[P], dcc[P], dho[P], dhx[P];
    int br[P], uu[P];
    bool on[P], rs[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const int p = tid + NTH * k, r = p / UB;
        uu[k] = p % UB;
        on[k] = rb + r < B;
        br[k] = (int)row0 + min(rb + r, B - 1);
        const int64_t ro = (int64_t)br[k] * H + u0 + uu[k];
#pragma unroll
        for (int q = 0; q < 4; ++q) ac[k][q] = a.act[(int64_t)br[k] * K + q * H + u0 + uu[k]];
        cx[k] = a.c_new[ro];
        cp[k] = a.c_prev[ro];
        dcc[k] = a.dc_rec[ro];
        dho[k] = a.dh_out ? a.dh_out[ro] : 0.f;
        dhx[k] = a.dh_extra ? a.dh_extra[ro] : 0.f;
        rs[k] = a.reset != nullptr && a.reset[br[k]] != 0.f;
    }

    // ---- dh_rec tile [32 rows x 16 units], this wave's K slice
    const int fr = lane & 15, fq = lane >> 4;
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    if (a.dG_next != nullptr) {
        const __hip_bfloat16* wp = a.W + grp * a.w_gs + (int64_t)(u0 + fr) * K + w * KW + fq * 8;
        const __hip_bfloat16* ap0 = a.dG_next + (row0 + min(rb + fr, B - 1)) * a.ld_dgn + w * KW + fq * 8;
        const __hip_bfloat16* ap1 = a.dG_next + (row0 + min(rb + 16 + fr, B - 1)) * a.ld_dgn + w * KW + fq * 8;
        constexpr int NK = KW / 32;
        bf16x8 bfr[NK], a0[NK], a1[NK];
#pragma unroll
        for (int ks = 0; ks < NK; ++ks) {
            bfr[ks] = *(const bf16x8*)(wp + ks * 32);
            a0[ks] = *(const bf16x8*)(ap0 + ks * 32);
            a1[ks] = *(const bf16x8*)(ap1 + ks * 32);
        }
#pragma unroll
        for (int ks = 0; ks < NK; ++ks) {
            acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[ks], bfr[ks], acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[ks], bfr[ks], acc[1], 0, 0, 0);
        }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) red[w][16 * i + fq * 4 + e][fr] = acc[i][e];
    __syncthreads();

    // ---- cell backward (plain LSTM path of csrc/lstm_cell.hip cell_bwd)
#pragma unroll
    for (int k = 0; k < P; ++k) {
        if (!on[k]) continue;
        const int p = tid + NTH * k, r = p / UB;
        const int b = br[k], u = u0 + uu[k];
        const int64_t ro = (int64_t)b * H + u;
        float dhc = dhx[k];
#pragma unroll
        for (int v = 0; v < NW; ++v) dhc += red[v][r][uu[k]];
        const float dh = dho[k] + (rs[k] ? 0.f : dhc);
        float dc = rs[k] ? 0.f : dcc[k];
        if (rs[k] && a.dinit_h) {
            a.dinit_h[ro] += dhc;
            a.dinit_c[ro] += dcc[k];
        }
        const float i = ac[k][0], tj = ac[k][1], f = ac[k][2], o = ac[k][3];
        const float t = tanhf(cx[k]);
        const float dout = dh * t;
        dc += dh * o * (1.f - t * t);
        const float m = dropout_mult(keep_on, key, ro, a.keep);
        float dy[4];
        dy[0] = dc * tj * m * i * (1.f - i);
        dy[1] = dc * i * m * (1.f - tj * tj);
        dy[2] = dc * cp[k] * f * (1.f - f);
        dy[3] = dout * o * (1.f - o);
        a.dc_rec[ro] = dc * f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            a.dG[(int64_t)b * K + q * H + u] = dy[q];
            a.dG_lp[(int64_t)b * K + q * H + u] = to_bf16(dy[q]);
        }
    }
}

template <int H>
int launch_bwd(const FusedBwdArgs& a, hipStream_t s) {
    const dim3 grid(H / UB, (a.B + RB - 1) / RB, a.nd);
    hipLaunchKernelGGL((lstm_fused_bwd<H, 8>), grid, dim3(512), 0, s, a);   // 8 waves (4 measured slower)
    return SKR_CHECK_LAUNCH();
}

template <int H>
int launch(const FusedFwdArgs& a, hipStream_t s) {
    const size_t lds = (size_t)(RB + 4 * UB) * H * 2 + 4 * RB * UB * 4;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)lstm_fused_fwd<H>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        attr = true;
    }
    hipLaunchKernelGGL(lstm_fused_fwd<H>, dim3(H / UB, (a.B + RB - 1) / RB, a.nd), dim3(256), lds, s, a);
    return SKR_CHECK_LAUNCH();
}

}  // namespace

SKR_API int skr_lstm_fused_fwd(const FusedFwdArgs* a, hipStream_t s) {
    if (a->B <= 0) return 0;
    if ((a->lda % 8) || (((uintptr_t)a->A | (uintptr_t)a->WT) & 15)) return -3;
    switch (a->H) {
        case 256: return launch<256>(*a, s);
        case 512: return launch<512>(*a, s);
        default: return -2;
    }
}

SKR_API int skr_lstm_fused_bwd(const FusedBwdArgs* a, hipStream_t s) {
    if (a->B <= 0) return 0;
    if ((a->dG_next && (a->ld_dgn % 8)) || (((uintptr_t)a->dG_next | (uintptr_t)a->W) & 15)) return -3;
    switch (a->H) {
        case 256: return launch_bwd<256>(*a, s);
        case 512: return launch_bwd<512>(*a, s);
        default: return -2;
    }
}

SKR_API int skr_lstm_fused_fwd_args_size() { return (int)sizeof(FusedFwdArgs); }
SKR_API int skr_lstm_fused_bwd_args_size() { return (int)sizeof(FusedBwdArgs); }
