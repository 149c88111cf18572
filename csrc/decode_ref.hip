// Fused whole-sketch decoder for the reference model (SURVEY K13 + K14;
// reference sampling loop model.py:187-264 around the single-step decoder
// model.py:9-11, 66-99): ONE launch generates every stroke of B sketches --
// per step both LSTM layers, the MDN head and the sampler -- with no host
// round trip and no kernel boundary between strokes.
//
// Roles (per row block of RB = 16*MTW sketches, 2*16 + 1 workgroups):
//   layer l, unit block wu (16 hidden units = 64 gate columns): keeps its
//     columns of [W_in; W_h] in LDS for the whole decode (K = H for layer 0,
//     whose K = 5 input projection x(t) @ W_x runs in fp32 in the epilogue;
//     K = 2H for layer 1, whose input is layer 0's output), c and the
//     carried h in VGPRs; bf16 MFMA (v_mfma_f32_16x16x32_bf16), fp32 cell.
//   head: keeps W_out^T (padded to a multiple of 16 rows) in LDS, computes
//     z = h_top @ W_out + b for its RB rows with MFMA into LDS, then one wave
//     per row draws the stroke (csrc/mdn_sample.h, bit-identical with the
//     stand-alone sampler kernel) and writes it as the next input x(t+1).
// Critical path per stroke: head(t-1) -> layer 0 epilogue (t) -> layer 1
// (t) -> head (t): three in-launch hand-offs (csrc/handoff.h). Layer 0's
// recurrent MFMAs for step t only need h0(t-1), so they run while the head
// is still sampling x(t).
//
// Reference step semantics (sampling feeds one step at a time with the
// previous state as `initial_state`): if the fed input x(t) has eoc set,
// every layer's carried state stays the fed-in state (model.py:82-92 with
// T = 1); the head sees the pre-reset output. The first input is x(0) from
// the host (zeros for the reference). Finished rows (eoc drawn) emit
// end-of-sketch padding while the recurrence keeps running, exactly as
// GraphDecoder + csrc/sampler.hip do. `forced` = teacher forcing: x(t) is
// read from `xin` for every t (numerics tests against the step oracle).
#include <algorithm>

#include "handoff.h"
#include "mdn_sample.h"

struct DecLayer {
    const __hip_bfloat16* WT;            // [4H][K] B^T: row n = [W_in[:, n] | W_h[:, n]] (layer 0: W_h[:, n])
    const float* bias;                   // [4H]
    const float* h0; const float* c0;    // [B][H] initial state
    __hip_bfloat16* hbuf;                // [N+1][B][H] carried h (next step's operand); hbuf[0] = h0 (host)
    __hip_bfloat16* hup;                 // [N][B][H] pre-reset output (input of the layer above / the head)
    float* hT; float* cT;                // [B][H] final carried state, or null
};

struct DecArgs {
    int N, B, L, H, mtw, nrb, M, nout, noutp, mode, greedy, fix_pen, forced;
    int row0;                            // global index of row 0 (sampler hash: batches split over launches)
    float temp, forget_bias;
    DecLayer ly[2];
    const float* Wx0;                    // [5][4H] layer-0 input weights (fp32)
    const __hip_bfloat16* WoT;           // [noutp][H] head weights^T (rows >= nout zero)
    const float* bo;                     // [nout]
    float* xin;                          // [N+1][B][8] fed inputs (x(0) from the host; forced: all from the host)
    float* out;                          // [B][N][5] strokes (finished rows: end-of-sketch padding)
    int* done;                           // [B], zeroed by the host
    float* zout;                         // [N][B][nout] head outputs, or null
    const int64_t* seed;
    uint32_t* flags;                     // [nrb][kFlagStride] epochs (zeroed per launch)
    int* err;
};

namespace {

using namespace skr;

constexpr int kH = 256;          // hidden units (the reference default rnn_size)
constexpr int U = 16;            // hidden units per layer workgroup
constexpr int NTHR = 512;        // 8 waves
constexpr int kFlagStride = 64;  // flag words per row block: [layer 0 | layer 1 | head]
constexpr int kXLd = 8;          // floats per fed-input row

// nrows x K of a row-major bf16 matrix into LDS, 16-byte chunks of LDS row r
// XOR-swizzled by (r & 15). GATE: LDS row r = gate (r >> 4), unit u0 + (r & 15)
// of a [4H][K] matrix; otherwise LDS row r = source row r.
template <bool GATE>
__device__ void stage(__hip_bfloat16* lds, const __hip_bfloat16* src, int nrows, int K, int u0) {
    const int cpr = K / 8;
    for (int i = threadIdx.x; i < nrows * cpr; i += NTHR) {
        const int r = i / cpr, c = i - r * cpr;
        const int sr = GATE ? (r >> 4) * kH + u0 + (r & 15) : r;
        const bf16x8 v = *(const bf16x8*)(src + (int64_t)sr * K + c * 8);
        *(bf16x8*)(lds + r * K + ((c ^ (r & 15)) * 8)) = v;
    }
}

__device__ __forceinline__ bf16x8 frag(const __hip_bfloat16* lds, int row, int K, int chunk) {
    return *(const bf16x8*)(lds + row * K + ((chunk ^ (row & 15)) * 8));
}

// ---------------------------------------------------------------------------------
// one LSTM layer's unit block
// ---------------------------------------------------------------------------------
template <int MTW, int KIN>
__device__ void layer_body(const DecArgs& a, int l, int rb, int wu, unsigned char* smem) {
    constexpr int H = kH, K = KIN + H, KS = 8 / MTW, KP = K / KS, NKS = KP / 32, NW = H / U, RB = 16 * MTW;
    const DecLayer& P = a.ly[l];
    __hip_bfloat16* Ws = (__hip_bfloat16*)smem;                        // [64][K]
    f32x4* part = (f32x4*)(smem + 64 * K * 2);                         // [KS][MTW][4][64]
    __hip_bfloat16* hx = (__hip_bfloat16*)(part + KS * MTW * 4 * 64);  // [MTW][16][16]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int mt = w % MTW, kp = w / MTW;
    const int fr = lane & 15, fq = lane >> 4;
    const int B = a.B, N = a.N;
    const int u0 = wu * U;
    const int row_t0 = rb * RB + mt * 16;       // first row of this wave's tile
    const bool tile_on = row_t0 < B;

    stage<true>(Ws, P.WT, 64, K, u0);
    __syncthreads();

    uint32_t* fl = a.flags + (int64_t)rb * kFlagStride;
    uint32_t* my_flags = fl + l * NW;
    const uint32_t* in_flags = fl + (l > 0 ? l - 1 : 0) * NW;
    const uint32_t* head_flag = fl + a.L * NW;
    const int64_t hbytes = (int64_t)N * B * H * 2;
    const __amdgpu_buffer_rsrc_t r_h = rsrc(P.hbuf, hbytes + (int64_t)B * H * 2);
    const __amdgpu_buffer_rsrc_t r_up = rsrc(P.hup, hbytes);
    const __amdgpu_buffer_rsrc_t r_in = rsrc(KIN > 0 ? a.ly[l > 0 ? l - 1 : 0].hup : P.hup, hbytes);
    const __amdgpu_buffer_rsrc_t r_x = rsrc(a.xin, (int64_t)(N + 1) * B * kXLd * 4);

    // epilogue lanes: K-slice-0 waves; lane holds rows row_t0 + 4fq + e, unit u0 + fr
    const bool epi = kp == 0 && tile_on;
    const int u = u0 + fr;
    int brow[4];
    bool bon[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int r = row_t0 + 4 * fq + e;
        bon[e] = epi && r < B;
        brow[e] = min(r, B - 1);
    }
    float c[4], hc[4], bias[4], wx[5][4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        c[e] = epi ? P.c0[(int64_t)brow[e] * H + u] : 0.f;
        hc[e] = epi ? P.h0[(int64_t)brow[e] * H + u] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        bias[q] = P.bias[q * H + u];
#pragma unroll
        for (int i = 0; i < 5; ++i) wx[i][q] = KIN == 0 ? a.Wx0[i * 4 * H + q * H + u] : 0.f;
    }
    const int arow = min(row_t0 + fr, B - 1);   // A-fragment row of this lane (clamped)
    bool ok = true;

    for (int t = 0; t < N; ++t) {
        f32x4 acc[4] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f},
                        f32x4{0.f, 0.f, 0.f, 0.f}};
        if (tile_on) {
            const int k0 = kp * KP;
            const bool from_in = KIN > 0 && k0 < KIN;
            if (from_in) ok = ok && wait_flags(in_flags, NW, (uint32_t)(t + 1), a.err);
            else if (t > 0) ok = ok && wait_flags(my_flags, NW, (uint32_t)t, a.err);
            const int kc = from_in ? k0 : k0 - KIN;
            const uint32_t base = (uint32_t)(((int64_t)t * B + arow) * H * 2);
            bf16x8 af[NKS];
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks)
                af[ks] = ld_sc1(from_in ? r_in : r_h, base + (uint32_t)((kc + ks * 32 + fq * 8) * 2));
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                const int chunk = (k0 + ks * 32) / 8 + fq;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks], frag(Ws, q * 16 + fr, K, chunk), acc[q],
                                                                     0, 0, 0);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) part[((kp * MTW + mt) * 4 + q) * 64 + lane] = acc[q];
        }
        __syncthreads();
        if (epi) {
            // fed input x(t): drawn by the head at step t-1 (layer 1 reads it
            // after layer 0's hand-off of step t, which came after that draw)
            if (KIN == 0 && !a.forced && t > 0) ok = ok && wait_flags(head_flag, 1, (uint32_t)t, a.err);
            float xv[4][5];
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int i = 0; i < 5; ++i)
                    xv[e][i] = (KIN == 0 || i == 3)
                                   ? ld_sc1_f32(r_x, (uint32_t)((((int64_t)t * B + brow[e]) * kXLd + i) * 4))
                                   : 0.f;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                f32x4 s = part[(mt * 4 + q) * 64 + lane];
#pragma unroll
                for (int p = 1; p < KS; ++p) s += part[((p * MTW + mt) * 4 + q) * 64 + lane];
                acc[q] = s;
            }
            float hn[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float g[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    float v = acc[q][e] + bias[q];
                    if (KIN == 0) {
#pragma unroll
                        for (int i = 0; i < 5; ++i) v += xv[e][i] * wx[i][q];
                    }
                    g[q] = v;
                }
                const float ig = sigmoidf_(g[0]), tj = tanhf(g[1]), fg = sigmoidf_(g[2] + a.forget_bias);
                const float og = sigmoidf_(g[3]);
                const float cn = c[e] * fg + ig * tj;
                hn[e] = tanhf(cn) * og;
                const bool r = xv[e][3] > 0.f;   // eoc fed: the carried state stays the fed-in state
                c[e] = r ? c[e] : cn;
                hc[e] = r ? hc[e] : hn[e];
            }
            // carried h -> hbuf[t+1], pre-reset h -> hup[t]: transposed through
            // LDS so each store is 16 contiguous bytes (8 units of one row)
            __hip_bfloat16* hw = hx + mt * 256;
#pragma unroll
            for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
                for (int e = 0; e < 4; ++e) hw[(4 * fq + e) * 16 + fr] = to_bf16(pass == 0 ? hc[e] : hn[e]);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (lane < 32) {
                    const int r = lane >> 1, hf = lane & 1;
                    if (row_t0 + r < B) {
                        const u32x4 v = *(const u32x4*)(hw + r * 16 + hf * 8);
                        const int64_t off = ((int64_t)(t + 1 - pass) * B + row_t0 + r) * H + u0 + hf * 8;
                        st_sc1(pass == 0 ? r_h : r_up, (uint32_t)(off * 2), v);
                    }
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
        }
        publish(my_flags + wu, (uint32_t)(t + 1));
    }
    if (epi && P.hT != nullptr) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            if (!bon[e]) continue;
            P.hT[(int64_t)brow[e] * H + u] = hc[e];
            P.cT[(int64_t)brow[e] * H + u] = c[e];
        }
    }
    (void)ok;
}

// ---------------------------------------------------------------------------------
// MDN head + sampler of a row block
// ---------------------------------------------------------------------------------
template <int MTW>
__device__ void head_body(const DecArgs& a, int rb, unsigned char* smem) {
    constexpr int H = kH, RB = 16 * MTW, NKS = H / 32, NW = H / U, CW = 8 / MTW;
    const int noutp = a.noutp, NT = noutp / 16, ldz = noutp + 4;
    __hip_bfloat16* Wo = (__hip_bfloat16*)smem;                  // [noutp][H]
    float* zs = (float*)(smem + (int64_t)noutp * H * 2);         // [RB][ldz]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const int B = a.B, N = a.N, M = a.M, nout = a.nout;
    const int stop_col = a.mode == 1 ? 4 : 3;

    stage<false>(Wo, a.WoT, noutp, H, 0);
    __syncthreads();

    uint32_t* fl = a.flags + (int64_t)rb * kFlagStride;
    const uint32_t* top_flags = fl + (a.L - 1) * NW;
    uint32_t* my_flag = fl + a.L * NW;
    const int64_t hbytes = (int64_t)N * B * H * 2;
    const __amdgpu_buffer_rsrc_t r_top = rsrc(a.ly[a.L - 1].hup, hbytes);
    const __amdgpu_buffer_rsrc_t r_x = rsrc(a.xin, (int64_t)(N + 1) * B * kXLd * 4);
    // wave w: row tile w % MTW, column tiles w / MTW, + CW, + 2 CW, ...
    const int mt = w % MTW, j0 = w / MTW;
    const int row_t0 = rb * RB + mt * 16;
    const bool tile_on = row_t0 < B;
    const int arow = min(row_t0 + fr, B - 1);
    const int64_t seed = *a.seed;
    constexpr int RPW = RB / 8;         // sampled rows per wave: w, w + 8, ...
    bool fin[RPW];                      // row finished (eoc drawn): emits padding from the next step
#pragma unroll
    for (int k = 0; k < RPW; ++k) fin[k] = false;
    bool ok = true;

    for (int t = 0; t < N; ++t) {
        if (tile_on) {
            ok = ok && wait_flags(top_flags, NW, (uint32_t)(t + 1), a.err);
            bf16x8 af[NKS];
            const uint32_t base = (uint32_t)(((int64_t)t * B + arow) * H * 2);
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) af[ks] = ld_sc1(r_top, base + (uint32_t)((ks * 32 + fq * 8) * 2));
            for (int j = j0; j < NT; j += CW) {
                f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ks = 0; ks < NKS; ++ks)
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks], frag(Wo, j * 16 + fr, H, ks * 4 + fq), acc,
                                                                  0, 0, 0);
                const int col = j * 16 + fr;
                const float bv = col < nout ? a.bo[col] : 0.f;
#pragma unroll
                for (int e = 0; e < 4; ++e) zs[(mt * 16 + 4 * fq + e) * ldz + col] = acc[e] + bv;
            }
        }
        __syncthreads();
        const uint32_t key = hash_key(seed, 0x5A3Du, (uint32_t)t);
        MdnDraw dr[RPW];
#pragma unroll
        for (int k = 0; k < RPW; ++k) {
            const int r = w + 8 * k, b = rb * RB + r;
            if (b >= B) continue;   // wave-uniform
            const float* zr = zs + r * ldz;
            dr[k] = mdn_sample_wave(zr, M, a.mode, a.temp, a.greedy, a.fix_pen, key, (uint32_t)(a.row0 + b),
                                    (uint32_t)t);
            if (!a.forced && lane < 5) {
                const float v = lane == 0 ? dr[k].row[0] : lane == 1 ? dr[k].row[1] : lane == 2 ? dr[k].row[2]
                              : lane == 3 ? dr[k].row[3] : dr[k].row[4];
                st_sc1_f32(r_x, (uint32_t)((((int64_t)(t + 1) * B + b) * kXLd + lane) * 4), v);
            }
            if (a.zout != nullptr)
                for (int c = lane; c < nout; c += 64) a.zout[((int64_t)t * B + b) * nout + c] = zr[c];
        }
        publish(my_flag, (uint32_t)(t + 1));
        // outputs no workgroup of this launch reads: stored after the hand-off
#pragma unroll
        for (int k = 0; k < RPW; ++k) {
            const int b = rb * RB + w + 8 * k;
            if (b >= B || lane != 0) continue;
            float* o = a.out + ((int64_t)b * N + t) * 5;
#pragma unroll
            for (int c = 0; c < 5; ++c) o[c] = fin[k] ? (c == stop_col ? 1.f : 0.f) : dr[k].row[c];
            fin[k] = fin[k] || dr[k].pidx + 2 == stop_col;
        }
    }
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
        const int b = rb * RB + w + 8 * k;
        if (b < B && lane == 0) a.done[b] = fin[k] ? 1 : 0;
    }
    (void)ok;
}

template <int MTW>
__global__ __launch_bounds__(NTHR) void decode_ref_kernel(const DecArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int NW = kH / U;
    const int per = a.L * NW + 1;
    const int rb = blockIdx.x / per, role = blockIdx.x - rb * per;
    if (role == a.L * NW) {
        head_body<MTW>(a, rb, smem);
    } else if (role >= NW) {
        layer_body<MTW, kH>(a, 1, rb, role - NW, smem);
    } else {
        layer_body<MTW, 0>(a, 0, rb, role, smem);
    }
}

inline size_t layer_lds(int K, int mtw) {
    return (size_t)64 * K * 2 + (size_t)(8 / mtw) * mtw * 4 * 64 * 16 + (size_t)mtw * 256 * 2;
}
inline size_t head_lds(int noutp, int mtw) { return (size_t)noutp * kH * 2 + (size_t)16 * mtw * (noutp + 4) * 4; }

template <int MTW>
int launch(const DecArgs& a, hipStream_t s) {
    const size_t lds = std::max(layer_lds(a.L == 2 ? 2 * kH : kH, MTW), head_lds(a.noutp, MTW));
    const int grid = a.nrb * (a.L * (kH / U) + 1);
    auto kern = decode_ref_kernel<MTW>;
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
            hipSuccess)
            return -9;
        attr = true;
    }
    if (!grid_fits((const void*)kern, NTHR, lds, grid)) return -8;
    const int nflags = a.nrb * kFlagStride;
    hipLaunchKernelGGL(zero_flags, dim3((nflags + 255) / 256), dim3(256), 0, s, a.flags, nflags);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NTHR), lds, s, a);
    return SKR_CHECK_LAUNCH();
}

}  // namespace

// Rows per row block: 16 * mtw (mtw 1 or 2). Returns 0 on success, < 0 on a
// rejected shape (-2 geometry, -4 nrb, -6 missing buffers, -8 grid not
// co-resident, -11 offsets past 32 bits).
SKR_API int skr_decode_ref(const DecArgs* a, hipStream_t s) {
    if (a->N <= 0 || a->B <= 0) return 0;
    if (a->H != kH || a->L < 1 || a->L > 2 || (a->mtw != 1 && a->mtw != 2)) return -2;
    if (a->M < 1 || a->M > 32 || a->nout != 3 + 6 * a->M || a->noutp != (a->nout + 15) / 16 * 16) return -2;
    if (a->nrb != (a->B + 16 * a->mtw - 1) / (16 * a->mtw)) return -4;
    if (a->flags == nullptr || a->err == nullptr || a->xin == nullptr || a->out == nullptr || a->done == nullptr ||
        a->seed == nullptr)
        return -6;
    if ((int64_t)(a->N + 1) * a->B * kH * 2 > 0x7fffffffLL || (int64_t)(a->N + 1) * a->B * kXLd * 4 > 0x7fffffffLL)
        return -11;
    return a->mtw == 1 ? launch<1>(*a, s) : launch<2>(*a, s);
}

SKR_API int skr_decode_ref_args_size() { return (int)sizeof(DecArgs); }
