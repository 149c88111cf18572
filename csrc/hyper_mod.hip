// HyperLSTM modulation step (forward), one launch per time step:
//
//   vec   = hh_t @ P + q (+ the main bias in the shift block)       [B, 12 H]
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
// Tiling: workgroup (gate q, 32-unit tile u0) -> 4 x 64 = 256 workgroups of
// 384 threads. Wave w owns MFMA column tile w: k-block q + 4 (w / 2) (x, h,
// shift modulation of gate q), units u0 + 16 (w % 2) .. +15; its P
// fragments (8 k-steps, K = Hh = 256) live in VGPRs; hh (all rows, bf16) is
// staged once in LDS (XOR-swizzled rows). v_mfma_f32_16x16x32_bf16: lane l
// holds A[row l & 15][k 8 (l >> 4)..+7], B[k 8 (l >> 4)..+7][col l & 15];
// C: col l & 15, rows 4 (l >> 4) + i.
//
// (Round 4 measured an unfolded variant -- vec = bf16(hh W_z) W_a + q on two
// MFMA stages, W_z L2-resident instead of the 12.6 MB folded P -- at 12.9 vs
// 10.2 us per step, with a slower backward; profiles/r4/unfold_ab.txt.)
#include "cell_fwd_body.h"
#include "handoff.h"
#include "row_cell.h"

namespace {

using namespace skr;

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int HH = 256, NTH = 384, TU = 32;      // hyper units (K), threads, units per tile
constexpr int MAXB = 128;                        // rows (16-row MFMA tiles: NRT <= 8)

__device__ __forceinline__ int sw(int row, int chunk) { return row * HH + ((chunk ^ (row & 15)) << 3); }

__device__ __forceinline__ uint32_t pack_bf(float a, float b) {
    return (uint32_t)__bfloat16_as_ushort(__float2bfloat16(a)) |
           ((uint32_t)__bfloat16_as_ushort(__float2bfloat16(b)) << 16);
}

}  // namespace

// Decode-step inputs (sample/hyper_step.py, csrc/decode_step.hip): the main
// x-projection formed here from the sampled stroke x [B][5]:
// xh[b][n] = zp[b][n] + sum_k x[b][k] w5[k][n] (skr_bproj_fwd's order). Null
// members: the training sequence's input (precomputed xh).
struct ModDecode {
    int xh_bf16;                              // training: the precomputed xh is bf16 [B][4H] (not decode)
    const float* x5;
    const float* w5; int64_t ldw5;
    const float* zp; int64_t ldzp;
    int probe;                                // timing probe (skr_hyper_mod_set_probe; 0 = off), set by the host
};

namespace {

// One modulation tile: gate q, hidden units [TU tile, +TU), row block z.
// NRT: 16-row tiles staged and multiplied (rows up to 16 NRT; a B = 100 launch
// pays for 112 rows, not MAXB). SC1: g and the partial sums are read by
// workgroups of the SAME launch (hyper_mod_chain): write-through stores.
// WAITHH (hyper_cell_mod): hh is written by workgroups of the SAME launch --
// every other load is issued first, then the tile waits on the launch's
// arrival counter (wcnt >= wtarget) and reads hh with sc1 loads.
template <int NS, int NRT, bool SC1, bool WAITHH = false>
__device__ __forceinline__ void mod_block(ModDecode dec, const __hip_bfloat16* __restrict__ hh, int64_t ld_hh,
                                          const float* __restrict__ xh, const float* __restrict__ R, int64_t r_slab,
                                          __hip_bfloat16* __restrict__ vec, float* __restrict__ gout,
                                          __hip_bfloat16* __restrict__ rlp, float* __restrict__ stats, int B, int H,
                                          const int q, const int tile, const int z, const bf16x8 (&pf)[8],
                                          const float qv, const uint32_t* wcnt = nullptr, uint32_t wtarget = 0,
                                          int* werr = nullptr);

// One modulation tile: gate q, hidden units [TU tile, +TU), row blocks z0,
// z0 + zs, ... of B rows (the P fragments loaded once for all of them).
template <int NS, int NRT, bool SC1, bool WAITHH = false>
__device__ __forceinline__ void mod_tile(ModDecode dec, const __hip_bfloat16* __restrict__ hh, int64_t ld_hh,
                                         const __hip_bfloat16* __restrict__ PlT,   // [12H][HH]
                                         const float* __restrict__ qb,             // [12H]
                                         const float* __restrict__ xh,             // [B][4H]
                                         const float* __restrict__ R, int64_t r_slab,   // [NS][B][4H]
                                         __hip_bfloat16* __restrict__ vec,          // [B][12H]
                                         float* __restrict__ gout,                  // [B][4H]
                                         __hip_bfloat16* __restrict__ rlp,          // [B][4H] or null
                                         float* __restrict__ stats,                 // [B][4][H/TU][2]
                                         int B, int H, const int q, const int tile, const int z0, const int zs,
                                         const uint32_t* wcnt = nullptr, uint32_t wtarget = 0, int* werr = nullptr) {
    const int u0 = tile * TU;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const int vcol = (q + 4 * (w >> 1)) * H + u0 + 16 * (w & 1);   // first modulation column of tile w
    bf16x8 pf[8];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) pf[ks] = *(const bf16x8*)(PlT + (int64_t)(vcol + fr) * HH + 32 * ks + 8 * fq);
    const float qv = qb[vcol + fr];
    const int nblk = (B + MAXB - 1) / MAXB;
    // (consecutive blocks reuse the LDS: the next block's hh stage is written
    // after this block's MFMAs -- every wave passed this block's second
    // barrier -- and its vectors after the next block's first barrier)
    for (int z = z0; z < nblk; z += zs)
        mod_block<NS, NRT, SC1, WAITHH>(dec, hh, ld_hh, xh, R, r_slab, vec, gout, rlp, stats, B, H, q, tile, z, pf, qv,
                                        wcnt, wtarget, werr);
}

// Row block z of a modulation tile (B > MAXB: the wide decode): rows
// r0 .. r0 + MAXB - 1.
template <int NS, int NRT, bool SC1, bool WAITHH>
__device__ __forceinline__ void mod_block(ModDecode dec, const __hip_bfloat16* __restrict__ hh, int64_t ld_hh,
                                          const float* __restrict__ xh, const float* __restrict__ R, int64_t r_slab,
                                          __hip_bfloat16* __restrict__ vec, float* __restrict__ gout,
                                          __hip_bfloat16* __restrict__ rlp, float* __restrict__ stats, int B, int H,
                                          const int q, const int tile, const int z, const bf16x8 (&pf)[8],
                                          const float qv, const uint32_t* wcnt, uint32_t wtarget, int* werr) {
    constexpr int MB = 16 * NRT;
    {
        const int r0 = z * MAXB;
        B = min(MAXB, B - r0);
        const int64_t G4 = (int64_t)r0 * 4 * H;
        if (hh) hh += (int64_t)r0 * ld_hh;
        if (dec.x5) {
            dec.x5 += (int64_t)r0 * 5;
            dec.zp += (int64_t)r0 * dec.ldzp;
        }
        if (xh) xh = dec.xh_bf16 ? (const float*)(const void*)((const __hip_bfloat16*)(const void*)xh + G4) : xh + G4;
        R += G4;
        gout += G4;
        if (rlp) rlp += G4;
        if (vec) vec += (int64_t)r0 * 12 * H;
        stats += (int64_t)r0 * 4 * (H / TU) * 2;
    }
    // (hh and the modulation vectors in one overlaid 64 KB buffer -- two
    // workgroups per CU, 130 VGPRs instead of 248 -- measured slower: the wide
    // decode's launch 64.2 vs 60.9 us, profiles/r6/dec2_kernels_bf16.txt)
    __shared__ __attribute__((aligned(16))) __hip_bfloat16 sA[MB * HH];     // <= 64 KB
    __shared__ __attribute__((aligned(16))) float sV[6][MB][16];            // <= 48 KB
    const int u0 = tile * TU, ntile = H / TU;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const int G = 4 * H, NV = 12 * H;
    // ---- every global load up front (the P fragments: mod_tile): the
    // epilogue's x-projection and R slabs (thread -> rows rg, rg + 48, rg + 96;
    // units u0 + 4 ug .. +3), and hh for the LDS stage
    constexpr int RPT = (MB + NTH / 8 - 1) / (NTH / 8);      // rows per thread (<= 3)
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
        } else if (dec.xh_bf16) {
            const uint2 u = *(const uint2*)((const __hip_bfloat16*)(const void*)xh + go);
            x4[k] = f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                          __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)};
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
    if (dec.probe == 1) return;                 // (timing probe: dispatch + the P fragments only)
    constexpr int NPC = MB * (HH / 8), SPT = (NPC + NTH - 1) / NTH;     // 16-byte hh pieces per thread
    bf16x8 hv[SPT];
    if constexpr (WAITHH) {   // hh from the rows of this launch: after their arrival, sc1 loads
        if (wcnt != nullptr) {   // (three workgroup barriers per block on every path: hyper_cell_mod's row wave)
            if (dec.probe == 8) chain_wait<8>(wcnt, wtarget, werr);
            else chain_wait<1>(wcnt, wtarget, werr);
        } else {
            __syncthreads();
        }
        const __amdgpu_buffer_rsrc_t hr = rsrc(hh, (int64_t)B * ld_hh * 2);
#pragma unroll
        for (int k = 0; k < SPT; ++k) {
            const int i = min(tid + k * NTH, NPC - 1), r = i / (HH / 8), c = i % (HH / 8);
            hv[k] = ld_sc1(hr, (uint32_t)(((int64_t)min(r, B - 1) * ld_hh + 8 * c) * 2));
        }
    } else {
#pragma unroll
        for (int k = 0; k < SPT; ++k) {
            const int i = min(tid + k * NTH, NPC - 1), r = i / (HH / 8), c = i % (HH / 8);
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
    if (dec.probe == 2) {                       // (timing probe: every load and the LDS stage, no MFMA / epilogue)
        float t = (float)pf[0][0] + __bfloat162float(sA[tid]);
#pragma unroll
        for (int k = 0; k < RPT; ++k) t += x4[k][0] + r4[k][0];
        if (t == 1.2345e-30f) gout[tid] = t;
        return;
    }
    f32x4 acc[NRT];
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt) acc[rt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
#pragma unroll
        for (int rt = 0; rt < NRT; ++rt) {
            const bf16x8 a = *(const bf16x8*)(sA + sw(16 * rt + fr, 4 * ks + fq));
            acc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pf[ks], acc[rt], 0, 0, 0);
        }
    if (dec.probe == 3) {                       // (timing probe: loads + MFMA, no vector stage / epilogue)
        float t = 0.f;
#pragma unroll
        for (int rt = 0; rt < NRT; ++rt) t += acc[rt][0];
#pragma unroll
        for (int k = 0; k < RPT; ++k) t += x4[k][0] + r4[k][0];
        if (t == 1.2345e-30f) gout[tid] = t;
        return;
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
    const __amdgpu_buffer_rsrc_t gr = rsrc(gout, (int64_t)B * G * 4);
    const __amdgpu_buffer_rsrc_t sr = rsrc(stats, (int64_t)B * 4 * ntile * 8);
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
            if constexpr (SC1) st_sc1(gr, (uint32_t)(go * 4), u32x4{__float_as_uint(g[0]), __float_as_uint(g[1]),
                                                                     __float_as_uint(g[2]), __float_as_uint(g[3])});
            else *(f32x4*)(gout + go) = f32x4{g[0], g[1], g[2], g[3]};
            if (rlp) *(u32x2*)(rlp + go) = u32x2{pack_bf(r4[k][0], r4[k][1]), pack_bf(r4[k][2], r4[k][3])};
            const int64_t vo = (int64_t)rr * NV + u0 + ul;
            if (vec) {   // (null at inference)
                *(u32x2*)(vec + vo + q * H) = u32x2{pack_bf(vx[0], vx[1]), pack_bf(vx[2], vx[3])};
                *(u32x2*)(vec + vo + (4 + q) * H) = u32x2{pack_bf(vh[0], vh[1]), pack_bf(vh[2], vh[3])};
            }
            // (the shift block 8..11 is not stored: the backward reads only
            // the x and h modulations -- d(shift) = dg needs no saved value)
            if (ug == 0) {
                const int64_t so = (((int64_t)rr * 4 + q) * ntile + tile) * 2;
                if constexpr (SC1) {
                    st_sc1_f32(sr, (uint32_t)(so * 4), s1);
                    st_sc1_f32(sr, (uint32_t)(so * 4 + 4), s2);
                } else {
                    stats[so] = s1;
                    stats[so + 1] = s2;
                }
            }
        }
    }
}

template <int NS, int NRT>
__global__ __launch_bounds__(NTH) void hyper_mod_fwd(ModDecode dec, const __hip_bfloat16* __restrict__ hh, int64_t ld_hh,
                                                     const __hip_bfloat16* __restrict__ PlT, const float* __restrict__ qb,
                                                     const float* __restrict__ xh, const float* __restrict__ R,
                                                     int64_t r_slab, __hip_bfloat16* __restrict__ vec,
                                                     float* __restrict__ gout, __hip_bfloat16* __restrict__ rlp,
                                                     float* __restrict__ stats, int B, int H) {
    if (dec.probe == 4) return;   // (timing probe: dispatch only)
    mod_tile<NS, NRT, false>(dec, hh, ld_hh, PlT, qb, xh, R, r_slab, vec, gout, rlp, stats, B, H, blockIdx.y, blockIdx.x,
                             blockIdx.z, gridDim.z);
}

// ---- chained launch: the modulation tiles + the main LayerNorm cell rows -----------------
// Every workgroup first runs its modulation tile (gate q, 32 units: all rows,
// one row block), stores g and the tile partial sums write-through and
// arrives on the launch's counter; workgroups [0, B C) then run the main cell
// of row b = id / C over units [c H / C, (c + 1) H / C), c = id % C: the loads
// that do not depend on the tiles (c_prev, the LayerNorm parameters) are
// issued before the wait, g and the partial sums are read with sc1 loads
// after it. Every workgroup arrives before any waits, so the launch needs all
// of its workgroups resident at once (the host checks the grid against the
// occupancy API; the waits are bounded and set *err).
// Arithmetic: cell_fwd_body MOD 3 (csrc/cell_fwd_body.h) with NT = NTH
// threads and UPT units per thread (per-thread unit u = base + k NTH + tid).
__device__ __forceinline__ float pick4(const float (&v)[4], int i) {
    return i == 0 ? v[0] : i == 1 ? v[1] : i == 2 ? v[2] : v[3];
}

template <int UPT>
__device__ __forceinline__ void main_rows(const FwdArgs& a, const int b, const int c, const int C,
                                          const uint32_t* cnt, uint32_t target, int* err) {
    constexpr int NT = NTH, NW = NT / 64;
    __shared__ float lds[NW * 8];
    __shared__ float mine[8];
    __shared__ float all[kMaxCluster * 8];
    const int tid = threadIdx.x, H = a.H, per = H / C, base = c * per;
    const bool keep_on = a.keep < 1.0f;
    const uint32_t key = keep_on ? hash_key(*a.seed, a.stream, a.step) : 0u;
    const bool r = a.reset != nullptr && a.reset[b] != 0.f;
    const bool save = a.xhat != nullptr;
    // ---- loads that do not depend on this launch's tiles
    float cp[UPT], lg[UPT][4], lb[UPT][4], lcg[UPT], lcb[UPT];
    bool on[UPT];
    int uc[UPT];
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
        const int u = base + k * NT + tid;
        on[k] = u < base + per;
        uc[k] = min(u, base + per - 1);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            lg[k][q] = a.ln_g[q * H + uc[k]];
            lb[k][q] = a.ln_b[q * H + uc[k]];
        }
        cp[k] = a.c_prev[(int64_t)b * H + uc[k]];
        lcg[k] = a.lnc_g[uc[k]];
        lcb[k] = a.lnc_b[uc[k]];
    }
    chain_wait<1>(cnt, target, err);
    // ---- g and the row's per-tile partial sums (stored by other workgroups of this launch)
    const __amdgpu_buffer_rsrc_t gr = rsrc(a.gpre + (int64_t)b * 4 * H, (int64_t)4 * H * 4);
    const __amdgpu_buffer_rsrc_t sr = rsrc(a.gstats + (int64_t)b * 4 * a.gstat_tiles * 2, (int64_t)a.gstat_tiles * 32);
    float g[UPT][4];
#pragma unroll
    for (int k = 0; k < UPT; ++k)
#pragma unroll
        for (int q = 0; q < 4; ++q) g[k][q] = ld_sc1_f32(gr, (uint32_t)((q * H + uc[k]) * 4));
    float s[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) s[q] = 0.f;
    for (int i = tid; i < 4 * a.gstat_tiles; i += NT) {
        const int gq = i / a.gstat_tiles;
        const float v1 = ld_sc1_f32(sr, (uint32_t)(i * 8)), v2 = ld_sc1_f32(sr, (uint32_t)(i * 8 + 4));
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (q == gq) {
                s[q] += v1;
                s[4 + q] += v2;
            }
        }
    }
    block_sum<8, NW>(s, lds);
    float mean[4], rs[4], xs[UPT][4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        mean[q] = s[q] / (float)H;
        rs[q] = rsqrtf(fmaxf(s[4 + q] / (float)H - mean[q] * mean[q], 0.f) + kLnEps);
    }
#pragma unroll
    for (int k = 0; k < UPT; ++k)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            xs[k][q] = (g[k][q] - mean[q]) * rs[q];
            g[k][q] = xs[k][q] * lg[k][q] + lb[k][q];
        }
    if (save && c == 0 && tid < 4) a.rstd[b * 5 + tid] = pick4(rs, tid);
    // ---- cell
    float cn[UPT], og[UPT], s2[2] = {0.f, 0.f};
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
        const int64_t ro = (int64_t)b * H + base + k * NT + tid;
        const float i = cell_sig(g[k][0]);
        const float tj = cell_tanh(g[k][1]);
        const float f = cell_sig(g[k][2] + a.forget_bias);
        og[k] = cell_sig(g[k][3]);
        const float m = dropout_mult(keep_on, key, ro, a.keep);
        cn[k] = on[k] ? cp[k] * f + i * tj * m : 0.f;
        s2[0] += cn[k];
        s2[1] += cn[k] * cn[k];
    }
    row_sum<2, NW>(s2, lds, mine, all, a.part + (int64_t)a.B * C * kSlots, a.err, a.step + 1, b, c, C);
    const float mc = s2[0] / (float)H;
    const float rc = rsqrtf(fmaxf(s2[1] / (float)H - mc * mc, 0.f) + kLnEps);
    if (save && c == 0 && tid == 0) a.rstd[b * 5 + 4] = rc;
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
        if (!on[k]) continue;
        const int u = base + k * NT + tid;
        const int64_t ro = (int64_t)b * H + u;
        const float ch = (cn[k] - mc) * rc;
        const float h = cell_tanh(ch * lcg[k] + lcb[k]) * og[k];
        if (save) {
            st_save(a.chat, ro, ch, a.save_lp);
#pragma unroll
            for (int q = 0; q < 4; ++q) st_save(a.xhat, (int64_t)b * 4 * H + q * H + u, xs[k][q], a.save_lp);
        }
        if (a.c_out != nullptr) a.c_out[ro] = cn[k];
        a.h_out[ro] = h;
        const float hc = r ? a.init_h[ro] : h;
        if (a.h_carry != nullptr) a.h_carry[ro] = hc;
        a.c_carry[ro] = r ? a.init_c[ro] : cn[k];
        if (a.lp_kind == 1) ((__hip_bfloat16*)a.h_lp)[b * a.ld_lp + u] = to_bf16(hc);
        else if (a.lp_kind == 2) ((float*)a.h_lp)[b * a.ld_lp + u] = hc;
    }
}

template <int NS, int NRT, int UPT>
__global__ __launch_bounds__(NTH) void hyper_mod_chain(const __hip_bfloat16* __restrict__ hh, int64_t ld_hh,
                                                       const __hip_bfloat16* __restrict__ PlT, const float* __restrict__ qb,
                                                       const float* __restrict__ xh, int xh_bf16, const float* __restrict__ R,
                                                       int64_t r_slab, __hip_bfloat16* __restrict__ vec,
                                                       __hip_bfloat16* __restrict__ rlp, const FwdArgs cell, const int C,
                                                       const ChainSync cs) {
    const int id = blockIdx.x, H = cell.H, ntile = H / TU;
    if (id == 0) chain_rotate(cs.counters, cs.n, cs.k);
    ModDecode dec{};
    dec.xh_bf16 = xh_bf16;
    mod_tile<NS, NRT, true>(dec, hh, ld_hh, PlT, qb, xh, R, r_slab, vec, const_cast<float*>(cell.gpre), rlp,
                            const_cast<float*>(cell.gstats), cell.B, H, id / ntile, id % ntile, 0, 1);
    chain_arrive(cs.counters + cs.k);
    if (id >= cell.B * C) return;
    main_rows<UPT>(cell, id / C, id % C, C, cs.counters + cs.k, (uint32_t)gridDim.x, cs.err);
}

// ---- chained launch: the hyper cell rows + the modulation tiles --------------------------
// One workgroup per modulation tile (gate q, 32 units), as hyper_mod_fwd, plus
// a seventh wave. In workgroups b < B that wave runs the hyper LayerNorm cell
// of row b (csrc/row_cell.h row_fwd_body, one wave of Hh / 4 lanes: its block
// sums need no barrier), stores the bf16 hh row write-through, drains and
// adds 1 to the launch's arrival counter; then (every workgroup) it joins
// the tile's three workgroup barriers and ends. The six tile waves issue
// every load that does not depend on hh -- the P fragments (12.6 MB over
// the chip: 4.8 of the separate launch's 10.9 us, scripts/micro/hm_probe.py),
// the x-projection and the R slabs -- then wait for all B rows and read hh
// with sc1 loads. Rows never wait before they arrive and every workgroup is
// one per CU (LDS), so the waits cannot starve a row of residency. One launch
// per forward step instead of the hyper cell + modulation pair.
// Measured and NOT adopted (ops.hyper.CELL_MOD, default off): 28.2 us per
// launch against 4.9 + 10.9 for the pair (vae_large 26.2 vs 23.65 ms/step,
// profiles/r6/cm2/); probes: tiles that do not wait 24.9 us, no rows 13.5 --
// the one-wave row takes ~11 us inside the launch, where the clustered hyper
// cell spends 4.9 on four 256-thread workgroups per row. (Run by wave 0 of
// the tile instead: 20.8 us, its row serialised before the wave's own P
// fetch; inside the tile after the loads are in flight: 122 VGPRs spilled.)
constexpr int NTH_HCM = NTH + 64;

template <int NS, int NRT>
__global__ __launch_bounds__(NTH_HCM) void hyper_cell_mod(const FwdArgs hc, const __hip_bfloat16* __restrict__ PlT,
                                                          const float* __restrict__ qb, const float* __restrict__ xh,
                                                          int xh_bf16, const float* __restrict__ R, int64_t r_slab,
                                                          __hip_bfloat16* __restrict__ vec, float* __restrict__ gout,
                                                          __hip_bfloat16* __restrict__ rlp, float* __restrict__ stats,
                                                          int H, const ChainSync cs, const int probe) {
    const int id = blockIdx.x, B = hc.B, ntile = H / TU;
    if (id == 0) chain_rotate(cs.counters, cs.n, cs.k);
    // (timing probes, skr_hyper_mod_set_probe; outputs WRONG: 5 the tiles do not
    // wait, 6 no rows and no wait; 8: poll period 8 s_sleep units -- correct)
    if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= NTH) {   // the row wave
        if (id < B && probe != 6) {
            row_fwd_body<HH / 4, 4, 0, 4, false, true>(hc, id, nullptr, 0, nullptr, NTH);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (threadIdx.x == NTH)
                __hip_atomic_fetch_add(cs.counters + cs.k, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();   // the tile's barriers: after the wait, the hh stage, the vector stage
        __syncthreads();
        __syncthreads();
        return;
    }
    ModDecode dec{};
    dec.xh_bf16 = xh_bf16;
    dec.probe = probe == 8 ? 8 : 0;
    mod_tile<NS, NRT, false, true>(dec, (const __hip_bfloat16*)hc.h_lp, hc.ld_lp, PlT, qb, xh, R, r_slab, vec, gout,
                                   rlp, stats, B, H, id / ntile, id % ntile, 0, 1,
                                   (probe == 5 || probe == 6) ? nullptr : cs.counters + cs.k, (uint32_t)B, cs.err);
}

}  // namespace

static int g_hm_zgrid = 0;   // row blocks in parallel (0: all); skr_hyper_mod_set_zgrid
static int g_hm_probe = 0;   // timing probe of skr_hyper_mod_fwd (the outputs are WRONG while set)

// Timing probes (scripts/micro/hm_probe.py): 0 off, 1 each row block returns
// at once (dispatch + P fragment loads), 2 after every load and the hh LDS
// stage, 3 after the MFMAs (no vector stage, epilogue or stores), 4 every
// workgroup returns at entry (dispatch only). Returns the previous setting.
SKR_API int skr_hyper_mod_set_probe(int p) {
    const int prev = g_hm_probe;
    if (p >= 0) g_hm_probe = p;
    return prev;
}

// A/B hook: parallel row blocks of the wide (B > 128) launches; 0 = one
// workgroup per row block. Returns the previous setting.
SKR_API int skr_hyper_mod_set_zgrid(int zg) {
    const int prev = g_hm_zgrid;
    if (zg >= 0) g_hm_zgrid = zg;
    return prev;
}

// hh [B][Hh] bf16 rows (stride ld_hh), PlT [12H][Hh] bf16, qb [12H] fp32
// (q, with the main bias added to blocks 8..11), xh [B][4H] fp32, R = sum of
// nslab fp32 slabs [B][4H] (stride r_slab), outputs vec [B][12H] bf16 (blocks
// 0..7 written; null at inference), g [B][4H] fp32, rlp [B][4H] bf16 (or
// null), stats [B][4][H/32][2] fp32. dec: decode-step inputs (ModDecode) or
// null. B > 128: 128-row blocks over gridDim.z (the last one partial).
SKR_API int skr_hyper_mod_fwd(const void* hh, int64_t ld_hh, const void* PlT, const float* qb, const float* xh,
                              const float* R, int64_t r_slab, int nslab, void* vec, float* g, void* rlp,
                              float* stats, int B, int H, int Hh, const ModDecode* dec, hipStream_t s) {
    ModDecode dz = dec ? *dec : ModDecode{};
    dz.probe = g_hm_probe;
    if (dz.x5 && (((uintptr_t)dz.w5 | (uintptr_t)dz.zp) & 15 || dz.ldw5 % 4 || dz.ldzp % 4)) return -4;
    if ((dz.x5 == nullptr && xh == nullptr) || hh == nullptr) return -3;
    if (B <= 0) return 0;
    if (B > 8 * MAXB || Hh != HH || H % TU != 0) return -2;
    if (((uintptr_t)hh | (uintptr_t)PlT | (uintptr_t)xh | (uintptr_t)R | (uintptr_t)vec | (uintptr_t)g |
         (uintptr_t)rlp) & 15 || (ld_hh % 8) || (r_slab % 4))
        return -4;
    // row blocks: gridDim.z of them in parallel, each workgroup walking
    // blocks z, z + gridDim.z, ... with its P fragments loaded once
    const int nblk = (B + MAXB - 1) / MAXB;
    const dim3 grid(H / TU, 4, g_hm_zgrid > 0 ? (nblk < g_hm_zgrid ? nblk : g_hm_zgrid) : nblk);
    const auto* a = (const __hip_bfloat16*)hh;
    const auto* p = (const __hip_bfloat16*)PlT;
    auto* v = (__hip_bfloat16*)vec;
    auto* rl = (__hip_bfloat16*)rlp;
    const int nrt = B <= 32 ? 2 : B <= 64 ? 4 : B <= 112 ? 7 : 8;
    if (nslab != 1 && nslab != 2 && nslab != 4) return -3;
#define SKR_HM(NS_, NRT_) \
    hipLaunchKernelGGL((hyper_mod_fwd<NS_, NRT_>), grid, dim3(NTH), 0, s, dz, a, ld_hh, p, qb, xh, R, r_slab, v, g, rl, stats, B, H)
#define SKR_HM_NS(NRT_) \
    do { if (nslab == 1) SKR_HM(1, NRT_); else if (nslab == 2) SKR_HM(2, NRT_); else SKR_HM(4, NRT_); } while (0)
    switch (nrt) {
        case 2: SKR_HM_NS(2); break;
        case 4: SKR_HM_NS(4); break;
        case 7: SKR_HM_NS(7); break;
        default: SKR_HM_NS(8); break;
    }
#undef SKR_HM_NS
#undef SKR_HM
    return SKR_CHECK_LAUNCH();
}

// Chained modulation step + main LayerNorm cell (hyper_mod_chain above): the
// modulation operands as skr_hyper_mod_fwd (training layout: xh precomputed,
// fp32 or bf16), cell = the MOD-3 main-cell arguments (gpre / gstats = this
// launch's g and partial-sum outputs) with cell->cluster = C workgroups per
// row. One row block (B <= 128) and B C <= 4 H / 32 rows' workgroups.
// Returns -2 / -3 / -4 when the shape is not taken (callers keep the two
// launches), -8 when the grid cannot be resident at once.
SKR_API int skr_hyper_mod_chain(const void* hh, int64_t ld_hh, const void* PlT, const float* qb, const float* xh,
                                int xh_bf16, const float* R, int64_t r_slab, int nslab, void* vec, void* rlp,
                                const skr::FwdArgs* cell, const ChainSync* cs, hipStream_t s) {
    if (cell == nullptr || cs == nullptr || cs->counters == nullptr || cs->err == nullptr || cs->n < 2 || cs->k < 0 ||
        cs->k >= cs->n)
        return -6;
    const skr::FwdArgs& a = *cell;
    const int B = a.B, H = a.H, C = a.cluster > 1 ? a.cluster : 1;
    if (B <= 0) return 0;
    if (B > MAXB || H % TU != 0 || xh == nullptr || hh == nullptr || a.gpre == nullptr || a.gstats == nullptr ||
        a.gstat_tiles != H / TU || a.h_q8 != nullptr || a.r_lp != nullptr || a.ln_g == nullptr || a.grp_rows > 0)
        return -3;
    if (nslab != 1 && nslab != 2 && nslab != 4) return -3;
    if (H % C != 0 || (C > 1 && (a.part == nullptr || a.err == nullptr)) || C > kMaxCluster) return -3;
    const int per = H / C, upt = (per + NTH - 1) / NTH;
    const int grid = 4 * (H / TU);
    if (B * C > grid) return -2;
    if (((uintptr_t)hh | (uintptr_t)PlT | (uintptr_t)xh | (uintptr_t)R | (uintptr_t)vec | (uintptr_t)a.gpre |
         (uintptr_t)rlp) & 15 || (ld_hh % 8) || (r_slab % 4))
        return -4;
    const auto* ap = (const __hip_bfloat16*)hh;
    const auto* pp = (const __hip_bfloat16*)PlT;
    auto* v = (__hip_bfloat16*)vec;
    auto* rl = (__hip_bfloat16*)rlp;
    const int nrt = B <= 32 ? 2 : B <= 64 ? 4 : B <= 112 ? 7 : 8;
    const void* k = nullptr;
#define SKR_HC_PICK(NS_, NRT_, UPT_) if (nslab == NS_ && nrt == NRT_ && upt == UPT_) k = (const void*)hyper_mod_chain<NS_, NRT_, UPT_>
#define SKR_HC_NRT(NS_, UPT_) SKR_HC_PICK(NS_, 2, UPT_); SKR_HC_PICK(NS_, 4, UPT_); SKR_HC_PICK(NS_, 7, UPT_); SKR_HC_PICK(NS_, 8, UPT_)
#define SKR_HC_UPT(NS_) SKR_HC_NRT(NS_, 2); SKR_HC_NRT(NS_, 3); SKR_HC_NRT(NS_, 6)
    SKR_HC_UPT(1);
    SKR_HC_UPT(2);
    SKR_HC_UPT(4);
#undef SKR_HC_UPT
#undef SKR_HC_NRT
#undef SKR_HC_PICK
    if (k == nullptr) return -2;
    // every workgroup waits on every other one: all must be resident at once
    if (!grid_fits(k, NTH, 0, grid, 1)) return -8;
    void* args[] = {(void*)&ap, (void*)&ld_hh, (void*)&pp, (void*)&qb, (void*)&xh, (void*)&xh_bf16, (void*)&R,
                    (void*)&r_slab, (void*)&v, (void*)&rl, (void*)&a, (void*)&C, (void*)cs};
    if (hipLaunchKernel(k, dim3(grid), dim3(NTH), args, 0, s) != hipSuccess) return -1;
    return SKR_CHECK_LAUNCH();
}

// Hyper cell step + modulation step in one launch (hyper_cell_mod). hc: the
// hyper LayerNorm cell (H = 256 units, mod 0: xp + the R slabs, bf16 h_lp =
// the tiles' hh operand, no resets); the modulation operands as
// skr_hyper_mod_fwd with the training layout (xh precomputed). 65 <= B <= 128.
// Returns -2 / -3 / -4 when not taken (the caller runs the two launches).
SKR_API int skr_hyper_cell_mod(const FwdArgs* hc, const void* PlT, const float* qb, const float* xh, int xh_bf16,
                               const float* R, int64_t r_slab, int nslab, void* vec, float* g, void* rlp, float* stats,
                               int H, const ChainSync* cs, hipStream_t s) {
    if (hc == nullptr || cs == nullptr || cs->counters == nullptr || cs->n < 2 || cs->k < 0 || cs->k >= cs->n ||
        cs->err == nullptr)
        return -6;
    const FwdArgs& a = *hc;
    const int B = a.B;
    if (B < 65 || B > MAXB || a.H != HH || H % TU != 0 || a.lp_kind != 1 || a.h_lp == nullptr || a.grp_rows > 0 ||
        a.R_nslab < 1 || xh == nullptr)
        return -2;
    const int rc = row_fwd_check(a, 0);
    if (rc) return rc;
    if (((uintptr_t)a.h_lp | (uintptr_t)PlT | (uintptr_t)xh | (uintptr_t)R | (uintptr_t)vec | (uintptr_t)g |
         (uintptr_t)rlp) & 15 || (a.ld_lp % 8) || (r_slab % 4))
        return -4;
    if (nslab != 1 && nslab != 2 && nslab != 4) return -3;
    const int grid = 4 * (H / TU);
    if (grid < B) return -2;   // (every row needs a host workgroup)
    const auto* p = (const __hip_bfloat16*)PlT;
    auto* v = (__hip_bfloat16*)vec;
    auto* rl = (__hip_bfloat16*)rlp;
#define SKR_HCM(NS_, NRT_) \
    hipLaunchKernelGGL((hyper_cell_mod<NS_, NRT_>), dim3(grid), dim3(NTH_HCM), 0, s, a, p, qb, xh, xh_bf16, R, r_slab, v, \
                       g, rl, stats, H, *cs, g_hm_probe)
#define SKR_HCM_NS(NRT_) \
    do { if (nslab == 1) SKR_HCM(1, NRT_); else if (nslab == 2) SKR_HCM(2, NRT_); else SKR_HCM(4, NRT_); } while (0)
    if (B <= 112) SKR_HCM_NS(7);
    else SKR_HCM_NS(8);
#undef SKR_HCM_NS
#undef SKR_HCM
    return SKR_CHECK_LAUNCH();
}
