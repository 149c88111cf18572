// HyperLSTM modulation step (forward), one launch per time step:
//
//   zd    = hh_t @ W_z                                               [B, 12 E]
//   vec   = bf16(zd) @ W_a + q (+ the main bias in the shift block)  [B, 12 H]
//   g     = xh * vec_x + R * vec_h + vec_b                           [B, 4 H]
//   stats = per (row, gate, 32-unit tile): sum g, sum g^2
//
// Reference recurrence: /root/reference model.py:66-95 (static unroll);
// HyperLSTM semantics: sketch_rnn_amd/models/cells.py hyper_lstm_step.
//
// Why fused: the main cell's LayerNorm needs row statistics over all 2048
// units of each gate, so as its own kernel it spends one in-launch exchange
// between the workgroups of a row on them (~3 us per step). This kernel
// already owns every (row, unit) of the gate pre-activations it produces, so
// it emits per-tile partial sums (64 tiles per gate); the main cell
// (csrc/cell_fwd_body.h, MOD 3) sums them while loading -- one exchange per
// step fewer -- and reads the finished g (32 KB per row) instead of x-proj,
// the R slabs and the modulation vectors (144 KB per row).
// The saves the backward needs are written here too: the x and h blocks of
// vec (bf16, q folded in: the backward cell runs with a zero vec_bias) and
// the bf16 summed R.
//
// The hyper-norm projections run unfolded, as in the model (and the oracle,
// models/cells.py hyper_lstm_step): z = hh @ W_z + b_z, vec = z @ W_a. With
// b_z @ W_a = q added in fp32, vec = bf16(hh @ W_z) @ W_a + q. Per step that
// streams W_z (196 KB, L2-resident: every workgroup of a gate reads the same
// slice) and W_a (1.5 MB) instead of the folded P = W_z W_a (12.6 MB, a
// different slice per workgroup), at the same MFMA count per wave.
//
// Tiling: workgroup (gate q, 32-unit tile u0) -> 4 x 64 = 256 workgroups of
// 384 threads. Wave w works on k-block kb = q + 4 (w / 2) (x, h, shift
// modulation of gate q): it computes the embedding half e = 16 (w % 2)..+15
// of zd_kb for all rows (W_z fragments in VGPRs, hh staged once in LDS),
// the pair of waves of a block swaps halves through LDS, then the wave forms
// vec for units u0 + 16 (w % 2)..+15 (K = 32: one MFMA per row tile).
// v_mfma_f32_16x16x32_bf16: lane l holds A[row l & 15][k 8 (l >> 4)..+7],
// B[k 8 (l >> 4)..+7][col l & 15]; C: col l & 15, rows 4 (l >> 4) + i.
//
// The x-/h-block vectors are saved for the backward (bf16, q folded in), and
// (zsave) z = zd + b_z in fp32 for the W_a / W_z gradients (by the u0 = 0
// workgroup of each gate).
#include "common.h"

namespace {

using namespace skr;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int HH = 256, NTH = 384, TU = 32;      // hyper units (K), threads, units per tile
constexpr int MAXB = 128, NRT = MAXB / 16;
constexpr int EP = 32, ZS = EP + 8;               // embedding padded to one MFMA K step; sZ row stride

__device__ __forceinline__ int sw(int row, int chunk) { return row * HH + ((chunk ^ (row & 15)) << 3); }

__device__ __forceinline__ uint32_t pack_bf(float a, float b) {
    return (uint32_t)__bfloat16_as_ushort(__float2bfloat16(a)) |
           ((uint32_t)__bfloat16_as_ushort(__float2bfloat16(b)) << 16);
}

}  // namespace

// Decode-step inputs (sample/hyper_step.py, csrc/decode_step.hip): hh from
// the hyper cell's fp32 output (the fp8 decode keeps no bf16 copy of it) and
// the main x-projection formed here from the sampled stroke x [B][5]:
// xh[b][n] = zp[b][n] + sum_k x[b][k] w5[k][n]. Null members: the training
// sequence's inputs (bf16 hh operand, precomputed xh).
struct ModDecode {
    const float* hh32;
    const float* x5;
    const float* w5; int64_t ldw5;
    const float* zp; int64_t ldzp;
};

namespace {

template <int NS>
__global__ __launch_bounds__(NTH) void hyper_mod_fwd(const ModDecode dec, const __hip_bfloat16* __restrict__ hh, int64_t ld_hh,
                                                     const __hip_bfloat16* __restrict__ WzT,   // [12][EP][HH]
                                                     const __hip_bfloat16* __restrict__ WaT,   // [12][H][EP]
                                                     const float* __restrict__ bz, int E,      // [12 E]
                                                     float* __restrict__ zsave,                // [B][12 E] or null
                                                     const float* __restrict__ qb,             // [12H]
                                                     const float* __restrict__ xh,             // [B][4H]
                                                     const float* __restrict__ R, int64_t r_slab,   // [NS][B][4H]
                                                     __hip_bfloat16* __restrict__ vec,          // [B][12H]
                                                     float* __restrict__ gout,                  // [B][4H]
                                                     __hip_bfloat16* __restrict__ rlp,          // [B][4H] or null
                                                     float* __restrict__ stats,                 // [B][4][H/TU][2]
                                                     int B, int H) {
    __shared__ __attribute__((aligned(16))) __hip_bfloat16 sA[MAXB * HH];   // 56 KB
    __shared__ __attribute__((aligned(16))) float sV[6][MAXB][16];          // 42 KB
    __shared__ __attribute__((aligned(16))) __hip_bfloat16 sZ[3][MAXB * ZS]; // 26 KB
    const int q = blockIdx.y, u0 = blockIdx.x * TU, ntile = H / TU;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const int G = 4 * H, NV = 12 * H;
    // ---- every global load up front: this wave's W_z fragments (block kb,
    // embeddings 16 half .. +15) and W_a fragment (units u0 + 16 half ..), the
    // epilogue's x-projection and R slabs (thread -> rows rg, rg + 48, rg + 96;
    // units u0 + 4 ug .. +3), and hh for the LDS stage
    const int jb = w >> 1, half = w & 1, kb = q + 4 * jb;
    const int vcol = kb * H + u0 + 16 * half;       // first modulation column of tile w
    bf16x8 zf[8];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
        zf[ks] = *(const bf16x8*)(WzT + ((int64_t)kb * EP + 16 * half + fr) * HH + 32 * ks + 8 * fq);
    const bf16x8 waf = *(const bf16x8*)(WaT + (int64_t)(vcol + fr) * EP + 8 * fq);
    const float qv = qb[vcol + fr];
    constexpr int RPT = (MAXB + NTH / 8 - 1) / (NTH / 8);    // rows per thread (3)
    const int rg = tid >> 3, ug = tid & 7, ul = 4 * ug;
    f32x4 x4[RPT], r4[RPT];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const int rr = min(rg + k * (NTH / 8), B - 1);
        const int64_t go = (int64_t)rr * G + q * H + u0 + ul;
        if (dec.x5 != nullptr) {
            const int col = q * H + u0 + ul;
            f32x4 v = *(const f32x4*)(dec.zp + rr * dec.ldzp + col);
#pragma unroll
            for (int k5 = 0; k5 < 5; ++k5) v += dec.x5[rr * 5 + k5] * *(const f32x4*)(dec.w5 + k5 * dec.ldw5 + col);
            x4[k] = v;
        } else {
            x4[k] = *(const f32x4*)(xh + go);
        }
        r4[k] = *(const f32x4*)(R + go);
#pragma unroll
        for (int sl = 1; sl < NS; ++sl) {
            const f32x4 t = *(const f32x4*)(R + sl * r_slab + go);
            r4[k] += t;
        }
    }
    constexpr int NPC = MAXB * (HH / 8), SPT = (NPC + NTH - 1) / NTH;   // 16-byte hh pieces (per thread: 10)
    bf16x8 hv[SPT];
#pragma unroll
    for (int k = 0; k < SPT; ++k) {
        const int i = min(tid + k * NTH, NPC - 1), r = i / (HH / 8), c = i % (HH / 8);
        if (dec.hh32 != nullptr) {
            const float* src = dec.hh32 + (int64_t)min(r, B - 1) * HH + 8 * c;
            const f32x4 lo = *(const f32x4*)src, hi = *(const f32x4*)(src + 4);
            hv[k] = bf16x8{(__bf16)lo[0], (__bf16)lo[1], (__bf16)lo[2], (__bf16)lo[3],
                           (__bf16)hi[0], (__bf16)hi[1], (__bf16)hi[2], (__bf16)hi[3]};
        } else {
            hv[k] = *(const bf16x8*)(hh + (int64_t)min(r, B - 1) * ld_hh + 8 * c);
        }
    }
#pragma unroll
    for (int k = 0; k < SPT; ++k) {
        const int i = tid + k * NTH, r = i / (HH / 8), c = i % (HH / 8);
        if (i >= NPC) break;
        if (r >= B) hv[k] = bf16x8{};
        *(bf16x8*)(sA + sw(r, c)) = hv[k];
    }
    __syncthreads();
    f32x4 acc[NRT];
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt) acc[rt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
#pragma unroll
        for (int rt = 0; rt < NRT; ++rt) {
            const bf16x8 a = *(const bf16x8*)(sA + sw(16 * rt + fr, 4 * ks + fq));
            acc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, zf[ks], acc[rt], 0, 0, 0);
        }
    // zd (this wave's 16 embeddings of block kb) -> bf16 -> LDS; z = zd + b_z saved in fp32
    const int e = 16 * half + fr;
    const bool zs = zsave != nullptr && blockIdx.x == 0 && e < E;
    const float bze = zs ? bz[kb * E + e] : 0.f;
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = 16 * rt + 4 * fq + i;
            sZ[jb][row * ZS + e] = __float2bfloat16(acc[rt][i]);
            if (zs && row < B) zsave[(int64_t)row * 12 * E + kb * E + e] = acc[rt][i] + bze;
        }
    __syncthreads();                 // both halves of every block's zd
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt) {
        const bf16x8 a = *(const bf16x8*)(&sZ[jb][(16 * rt + fr) * ZS + 8 * fq]);
        acc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, waf, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    }
    // modulation vectors (+ q) -> bf16 -> LDS: the epilogue needs all three
    // blocks of a unit in one thread. The bf16-rounded value is what the
    // backward will read, so g is formed from it too.
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
        for (int i = 0; i < 4; ++i)
            sV[w][16 * rt + 4 * fq + i][fr] = __bfloat162float(__float2bfloat16(acc[rt][i] + qv));
    __syncthreads();
    // ---- epilogue (no loads left): 8 threads per row (lanes 8k..8k+7)
    const int ch = ul >> 4, cu = ul & 15;          // column tile half, column inside it
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const int r = rg + k * (NTH / 8);
        if (r >= ((B + 7) & ~7)) break;            // uniform over each 8-lane row group and each wave
        const bool on = r < B;
        const int rr = on ? r : B - 1;
        float g[4], s1 = 0.f, s2 = 0.f;
        float vx[4], vh[4], vb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            vx[i] = sV[0 + ch][rr][cu + i];
            vh[i] = sV[2 + ch][rr][cu + i];
            vb[i] = sV[4 + ch][rr][cu + i];
            g[i] = x4[k][i] * vx[i] + r4[k][i] * vh[i] + vb[i];
            s1 += g[i];
            s2 += g[i] * g[i];
        }
        s1 += __shfl_xor(s1, 1, 64);
        s2 += __shfl_xor(s2, 1, 64);
        s1 += __shfl_xor(s1, 2, 64);
        s2 += __shfl_xor(s2, 2, 64);
        s1 += __shfl_xor(s1, 4, 64);
        s2 += __shfl_xor(s2, 4, 64);
        if (on) {
            const int64_t go = (int64_t)rr * G + q * H + u0 + ul;
            *(f32x4*)(gout + go) = f32x4{g[0], g[1], g[2], g[3]};
            if (rlp) *(u32x2*)(rlp + go) = u32x2{pack_bf(r4[k][0], r4[k][1]), pack_bf(r4[k][2], r4[k][3])};
            const int64_t vo = (int64_t)rr * NV + u0 + ul;
            if (vec) {   // (null at inference)
                *(u32x2*)(vec + vo + q * H) = u32x2{pack_bf(vx[0], vx[1]), pack_bf(vx[2], vx[3])};
                *(u32x2*)(vec + vo + (4 + q) * H) = u32x2{pack_bf(vh[0], vh[1]), pack_bf(vh[2], vh[3])};
            }
            // (the shift block 8..11 is not stored: the backward reads only
            // the x and h modulations -- d(shift) = dg needs no saved value)
            if (ug == 0) {
                float* sp = stats + (((int64_t)rr * 4 + q) * ntile + blockIdx.x) * 2;
                sp[0] = s1;
                sp[1] = s2;
            }
        }
    }
}

}  // namespace

// hh [B][Hh] bf16 rows (stride ld_hh), WzT [12][32][Hh] bf16 (W_z^T per block,
// embeddings past E zero), WaT [12][H][32] bf16 (W_a per block, unit-major,
// embeddings past E zero), bz [12E] fp32, qb [12H] fp32 (b_z @ W_a, with the
// main bias added to blocks 8..11), xh [B][4H] fp32, R = sum of nslab fp32
// slabs [B][4H] (stride r_slab); outputs vec [B][12H] bf16 (blocks 0..7
// written; null at inference), g [B][4H] fp32, rlp [B][4H] bf16 (or null), stats [B][4][H/32][2]
// fp32, zsave [B][12E] fp32 (or null).
SKR_API int skr_hyper_mod_fwd(const void* hh, int64_t ld_hh, const void* WzT, const void* WaT, const float* bz,
                              int E, float* zsave, const float* qb, const float* xh, const float* R, int64_t r_slab,
                              int nslab, void* vec, float* g, void* rlp, float* stats, int B, int H, int Hh,
                              const ModDecode* dec, hipStream_t s) {
    const ModDecode dz = dec ? *dec : ModDecode{};
    if (dz.x5 && (((uintptr_t)dz.w5 | (uintptr_t)dz.zp) & 15 || dz.ldw5 % 4 || dz.ldzp % 4)) return -4;
    if (dz.hh32 && ((uintptr_t)dz.hh32 & 15)) return -4;
    if (B <= 0) return 0;
    if (B > MAXB || Hh != HH || H % TU != 0 || E < 1 || E > EP) return -2;
    if (((uintptr_t)hh | (uintptr_t)WzT | (uintptr_t)WaT | (uintptr_t)xh | (uintptr_t)R | (uintptr_t)vec |
         (uintptr_t)g | (uintptr_t)rlp) & 15 || (ld_hh % 8) || (r_slab % 4))
        return -4;
    const dim3 grid(H / TU, 4);
    const auto* a = (const __hip_bfloat16*)hh;
    const auto* wz = (const __hip_bfloat16*)WzT;
    const auto* wa = (const __hip_bfloat16*)WaT;
    auto* v = (__hip_bfloat16*)vec;
    auto* rl = (__hip_bfloat16*)rlp;
#define SKR_HM(NS_) hipLaunchKernelGGL(hyper_mod_fwd<NS_>, grid, dim3(NTH), 0, s, dz, a, ld_hh, wz, wa, bz, E, zsave, qb, \
                                       xh, R, r_slab, v, g, rl, stats, B, H)
    switch (nslab) {
        case 1: SKR_HM(1); break;
        case 2: SKR_HM(2); break;
        case 4: SKR_HM(4); break;
        default: return -3;
    }
#undef SKR_HM
    return SKR_CHECK_LAUNCH();
}
