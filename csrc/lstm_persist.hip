// Persistent LSTM sequence kernels (plain LSTM, bf16 MFMA operands, fp32
// state): ONE launch runs a whole sequence -- every time step of up to two
// stacked layers (or two independent directions) -- instead of one launch
// per layer per step.
//
// Why: at the shapes of the reference config (2 x 256 LSTM, B = 100,
// T = 300) and the VAE encoder (bidirectional 512, B = 100, T = 250) a step
// is ~50-200 MFLOP; the per-step launch chain (launch gap + re-staging W_h
// from L2 + a cold epilogue) costs 6-10 us per layer-step on MI355X while
// the math is well under 1 us. Here each workgroup keeps its slice of the
// weights in LDS for the whole sequence, its slice of the cell state c in
// VGPRs, and only the bf16 hidden state (forward) or bf16 gate gradient
// (backward) travels between workgroups, once per step.
//
// Tiling: a workgroup owns U = 16 hidden units x 16*MTW batch rows of one
// (layer, direction). Forward: it holds the 64 gate columns of its units
// (4 gates x 16) of [W_in; W_h] (K = H, or 2H for a layer whose input is
// the layer below, computed in-kernel rather than hoisted) in LDS; the
// 8 waves split the work as MTW row tiles x KS = 8/MTW K-slices, each wave
// accumulating its [16 rows x 64 columns] with v_mfma_f32_16x16x32_bf16,
// partial tiles summed through LDS. The cell epilogue runs in the MFMA
// accumulator layout: a lane of a K-slice-0 wave holds all four gates of
// 4 (row, unit) cells, so c lives in that lane's registers for all T steps.
// Backward: the workgroup holds rows u0..u0+15 of W_h (and of the layer
// above's W_in) -- dh = dG_{t+1} @ W_h^T (+ dG_above_t @ W_in_above^T) --
// and the cell backward again runs in registers with dc carried in VGPRs.
//
// Hand-off between workgroups (CDNA4 guide, Guideline 16, the first row of
// the "measured hand-offs" table): the producer stores its payload
// write-through (buffer_store ... sc1), every storing wave drains
// (s_waitcnt vmcnt(0)), a workgroup barrier, then ONE lane stores the
// workgroup's epoch (t + 1) into its flag word with an sc1 store. A consumer
// wave polls the NW flag words of its row block with sc1 loads (one lane per
// flag, bounded spin with s_sleep) and then reads the payload with sc1
// buffer loads only -- no agent-scope acquire needed, no atomics, no
// counter fan-in. Flags are per (layer, direction, row block, producer) so
// only the workgroups that exchange data wait on each other. A timed-out
// wait sets *err (the host raises) and poisons the launch so every other
// wait returns at once: the grid always drains.
//
// Co-residency: every workgroup must be resident (they spin on each other);
// the launcher checks the grid against the occupancy API and refuses a grid
// that does not fit.
//
// (A LayerNorm-LSTM variant -- both LayerNorms' row statistics exchanged
// in-launch, two hand-offs per step each way -- was built and measured
// slower than the per-step clustered cells on vae_layernorm, 11.50 vs 10.34
// ms/step, and removed in round 5; the LayerNorm-LSTM runs on
// csrc/lstm_cell.hip.)
//
// Reference semantics: model.py:19-23 (BasicLSTMCell, forget bias 1),
// model.py:66-95 (static unroll with the eoc state reset: the carried state
// of a row whose input has eoc set is replaced by the batch-initial state);
// recurrent dropout on tanh(j) keyed like csrc/lstm_cell.hip.
#include "handoff.h"
#include "lstm_args.h"

namespace {

using namespace skr;

constexpr int U = 16;               // hidden units per workgroup
constexpr int NTHR = 512;           // 8 waves
constexpr int kFlagStride = 64;     // u32 flag words per (layer, group, row block)

}  // namespace

// Spin bound of this file's hand-off waits (polls; kHandoffSpinLimit, ~seconds).
// The failure-path test lowers it (skr_persist_set_spin_limit) so that a
// co-running occupancy hog outlives it: the wait times out, sets *err and
// the launch drains (tests/test_dp_concurrency_gpu.py).
__device__ unsigned g_persist_spin_limit = kHandoffSpinLimit;

struct PFwdLayer {
    const __hip_bfloat16* WT; int64_t w_gs;  // [nd][4H][K] B^T: row n = [W_in[:, n] | W_h[:, n]], K = kin + H
    int kin;                                  // 0: input projection hoisted into xp; H: input = layer below
    const float* xp; int64_t xp_ts, xp_ld;    // xp[t*ts + row*ld + n] (+bias); ts = ld = 0: a bias vector
    const float* c0;                          // [nd*B][H]
    const float* init_h; const float* init_c; // reset targets [nd*B][H] (read iff reset)
    __hip_bfloat16* hlp;                      // [nd][T+1][B][H] carried h (next step's operand); [:, 0] = h0 (host)
    __hip_bfloat16* hup;                      // [T][nd*B][H] pre-reset h for the layer above, or null
    float* h_out;                             // [T][nd*B][H] or null
    float* c_out;                             // [T][nd*B][H] pre-reset c
    float* c_carry;                           // [T+1][nd*B][H] carried c (index t+1) or null (no resets)
    float* act;                               // [T][nd*B][4H] sig(i), tanh(j), sig(f+fb), sig(o)
    float* hT; float* cT;                     // [nd*B][H] final carried state (fp32)
    float keep; uint32_t stream;
    float* h_last;                            // [B][nd*H] h at each row's last valid step (needs tlen), the
                                              // directions side by side (the encoder's [h_fw | h_bw]), or null
};

struct PFwdArgs {
    int T, B, nd, L, H, nrb;                  // nrb row blocks of 16*MTW rows per group
    PFwdLayer ly[2];
    const float* reset;                       // [T][nd*B] or null
    float forget_bias;
    const int64_t* seed;
    uint32_t* flags;                          // [L][nd][nrb][kFlagStride] epochs (zeroed per launch)
    int* err;
    const int* tlen;                          // [B] valid lengths (L = 1) or null, see row_block_steps
};

struct PBwdLayer {
    const __hip_bfloat16* Wr; int64_t wr_gs;  // [nd][H][4H] W_h (row u = unit): B^T of dG @ W_h^T
    const __hip_bfloat16* Wu;                 // [H][4H] W_in of the layer above (rows = this layer's units) or null
    const float* dh_out;                      // [T][nd*B][H] grad of this layer's outputs (top layer) or null
    const float* dhT; const float* dcT;       // [nd*B][H] grads into the final carried state, or null
    const float* act; const float* c_out; const float* c_carry; const float* c0;
    __hip_bfloat16* dg_lp;                    // [nd][T][B][4H] bf16 dG (published)
    float* dg;                                // [T][nd*B][4H] fp32 dG or null
    float* dh0; float* dc0;                   // [nd*B][H] grads into the initial state
    float* dinit_h; float* dinit_c;           // [nd*B][H] grads into the reset targets (with resets)
    float keep; uint32_t stream;
    const float* dh_last;                     // [B][nd*H] grad of h_last (added at each row's last step) or null
};

struct PBwdArgs {
    int T, B, nd, L, H, nrb;
    PBwdLayer ly[2];
    const float* reset;
    const int64_t* seed;
    uint32_t* flags;
    int* err;
    const int* tlen;                          // as PFwdArgs::tlen (the same lengths as the forward)
};

namespace {

// Stage nrows x K of a row-major bf16 matrix into LDS with the 16-byte
// chunks of LDS row r XOR-swizzled by (r & 15) (conflict-free ds_read_b128 of
// MFMA fragments). GATE: LDS row r = gate (r >> 4), unit u0 + (r & 15) of a
// [4H][K] matrix; otherwise LDS row r = source row u0 + r.
template <bool GATE>
__device__ void stage_rows(__hip_bfloat16* lds, const __hip_bfloat16* src, int64_t ld, int nrows, int K, int H,
                           int u0) {
    const int cpr = K / 8;
    for (int i = threadIdx.x; i < nrows * cpr; i += NTHR) {
        const int r = i / cpr, c = i - r * cpr;
        const int sr = GATE ? (r >> 4) * H + u0 + (r & 15) : u0 + r;
        const bf16x8 v = *(const bf16x8*)(src + (int64_t)sr * ld + c * 8);
        *(bf16x8*)(lds + r * K + ((c ^ (r & 15)) * 8)) = v;
    }
}

__device__ __forceinline__ bf16x8 lds_frag(const __hip_bfloat16* lds, int row, int K, int chunk) {
    return *(const bf16x8*)(lds + row * K + ((chunk ^ (row & 15)) * 8));
}

// Steps a row block runs. With per-row valid lengths (the VAE encoder: rows
// are padded past their length, both directions read only steps < length,
// like TF's dynamic_rnn with sequence_length) a row block stops after the
// longest of its rows: Te = max(min(len, T)) over its rows (>= 1). Row blocks
// never wait on each other, so each keeps its own bound; the tails t >= Te
// of the tensors read after the launch (top outputs, the carried-h operand of
// the weight-gradient GEMM, dG) are zero-filled so those products stay exact.
// The final carried state (hT, cT) is the state after step Te - 1.
__device__ __forceinline__ int row_block_steps(const int* tlen, int T, int B, int rb, int rows) {
    if (tlen == nullptr) return T;
    int te = 1;
    const int r1 = min(B, (rb + 1) * rows);
    for (int r = rb * rows; r < r1; ++r) te = max(te, min(tlen[r], T));
    return te;
}

// Last valid step of row r: the one whose h the encoder reads (h[len - 1],
// len clamped to [1, T] like the gather it replaces).
__device__ __forceinline__ int row_last_step(const int* tlen, int T, int r) {
    return tlen == nullptr ? T - 1 : max(min(tlen[r], T), 1) - 1;
}

// =====================================================================================
// forward
// =====================================================================================
template <int H, int MTW, int KIN>
__device__ void fwd_body(const PFwdArgs& a, int l, int g, int rb, int wu, unsigned char* smem) {
    constexpr int K = KIN + H, KS = 8 / MTW, KP = K / KS, NKS = KP / 32, NW = H / U;
    const PFwdLayer& P = a.ly[l];
    __hip_bfloat16* Ws = (__hip_bfloat16*)smem;                       // [64][K]
    f32x4* part = (f32x4*)(smem + 64 * K * 2);                        // [KS][MTW][4][64]
    __hip_bfloat16* hx = (__hip_bfloat16*)(part + KS * MTW * 4 * 64); // [MTW][16][16]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int mt = w % MTW, kp = w / MTW;
    const int fr = lane & 15, fq = lane >> 4;
    const int B = a.B, nB = a.nd * B, T = a.T;
    const int u0 = wu * U;
    const int row_t0 = rb * 16 * MTW + mt * 16;        // first row (within the group) of this wave's tile
    const bool tile_on = row_t0 < B;
    const int64_t grow0 = (int64_t)g * B;              // group's first global row

    stage_rows<true>(Ws, P.WT + g * P.w_gs, K, 64, K, H, u0);
    __syncthreads();

    // carried h is direction-major ([nd][T+1][B][H]): a direction's rows are
    // contiguous per step, so the weight-gradient GEMM reads each direction
    // as one [T*B, H] matrix without a copy (nd == 1: the plain [T+1][B][H])
    __hip_bfloat16* const hl = P.hlp + (int64_t)g * (T + 1) * B * H;
    const __amdgpu_buffer_rsrc_t r_h = rsrc(hl, (int64_t)(T + 1) * B * H * 2);
    const PFwdLayer* Pb = l > 0 ? &a.ly[l - 1] : nullptr;
    const __hip_bfloat16* in_base = (KIN > 0) ? (Pb->hup != nullptr ? Pb->hup : Pb->hlp + (int64_t)nB * H) : nullptr;
    const __amdgpu_buffer_rsrc_t r_in = rsrc(KIN > 0 ? (const void*)in_base : (const void*)P.hlp,
                                             (int64_t)(T + 1) * nB * H * 2);
    uint32_t* my_flags = a.flags + (((int64_t)l * a.nd + g) * a.nrb + rb) * kFlagStride;
    const uint32_t* in_flags = l > 0 ? a.flags + (((int64_t)(l - 1) * a.nd + g) * a.nrb + rb) * kFlagStride : nullptr;

    // epilogue lanes: K-slice-0 waves; lane holds rows row_t0 + 4fq + e, unit u0 + fr
    const bool epi = kp == 0 && tile_on;
    const int u = u0 + fr;
    int brow[4];
    bool bon[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int r = row_t0 + 4 * fq + e;
        bon[e] = epi && r < B;
        brow[e] = (int)grow0 + min(r, B - 1);
    }
    float c[4];
    int tlast[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        c[e] = epi ? P.c0[(int64_t)brow[e] * H + u] : 0.f;
        tlast[e] = row_last_step(a.tlen, T, brow[e] - (int)grow0);
    }
    const bool keep_on = P.keep < 1.0f;
    // A-fragment row of this lane (clamped) within its tile
    const int arow = (int)grow0 + min(row_t0 + fr, B - 1);
    bool ok = true;
    const int Te = row_block_steps(a.tlen, T, B, rb, 16 * MTW);

    for (int t = 0; t < Te; ++t) {
        // ---- epilogue inputs of step t (independent of the recurrence: issued before the wait)
        float xv[4][4], rs[4], ih[4], ic[4];
        if (epi) {
            const float* xb = P.xp + (int64_t)t * P.xp_ts;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
#pragma unroll
                for (int q = 0; q < 4; ++q) xv[e][q] = xb[(int64_t)brow[e] * P.xp_ld + q * H + u];
                rs[e] = a.reset != nullptr ? a.reset[(int64_t)t * nB + brow[e]] : 0.f;
                ih[e] = a.reset != nullptr ? P.init_h[(int64_t)brow[e] * H + u] : 0.f;
                ic[e] = a.reset != nullptr ? P.init_c[(int64_t)brow[e] * H + u] : 0.f;
            }
        }
        // ---- wait for the operands of this wave's K slice
        f32x4 acc[4] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f},
                        f32x4{0.f, 0.f, 0.f, 0.f}};
        if (tile_on) {
            const int k0 = kp * KP;
            const bool from_in = KIN > 0 && k0 < KIN;
            if (from_in) ok = ok && wait_flags(in_flags, NW, (uint32_t)(t + 1), a.err, g_persist_spin_limit);
            else if (t > 0) ok = ok && wait_flags(my_flags, NW, (uint32_t)t, a.err, g_persist_spin_limit);
            // A fragments: row arow, columns k0 + ks*32 + fq*8 (sc1: written by other workgroups)
            bf16x8 af[NKS];
            const int kc = from_in ? k0 : k0 - KIN;     // column within the source matrix
            const uint32_t base = from_in ? (uint32_t)(((int64_t)t * nB + arow) * H * 2)
                                          : (uint32_t)(((int64_t)t * B + (arow - grow0)) * H * 2);
            const __amdgpu_buffer_rsrc_t rr = from_in ? r_in : r_h;
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) af[ks] = ld_sc1(rr, base + (uint32_t)((kc + ks * 32 + fq * 8) * 2));
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                const int chunk = (k0 + ks * 32) / 8 + fq;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks], lds_frag(Ws, q * 16 + fr, K, chunk),
                                                                     acc[q], 0, 0, 0);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) part[((kp * MTW + mt) * 4 + q) * 64 + lane] = acc[q];
        }
        __syncthreads();
        // ---- cell update in registers (K-slice-0 waves)
        float hc[4], hn[4], cn[4], av[4][4];
        if (epi) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                f32x4 s = part[(mt * 4 + q) * 64 + lane];
#pragma unroll
                for (int p = 1; p < KS; ++p) s += part[((p * MTW + mt) * 4 + q) * 64 + lane];
                acc[q] = s;
            }
        }
        if (epi) {
            const uint32_t key = keep_on ? hash_key(*a.seed, P.stream, (uint32_t)t) : 0u;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float gi = acc[0][e] + xv[e][0], gj = acc[1][e] + xv[e][1];
                const float gf = acc[2][e] + xv[e][2], go = acc[3][e] + xv[e][3];
                const float i = sigmoidf_(gi), tj = tanhf(gj), f = sigmoidf_(gf + a.forget_bias), o = sigmoidf_(go);
                const float m = dropout_mult(keep_on, key, (int64_t)brow[e] * H + u, P.keep);
                cn[e] = c[e] * f + i * tj * m;
                hn[e] = tanhf(cn[e]) * o;
                av[e][0] = i; av[e][1] = tj; av[e][2] = f; av[e][3] = o;
                const bool r = rs[e] != 0.f;
                hc[e] = r ? ih[e] : hn[e];
                c[e] = r ? ic[e] : cn[e];
            }
            // carried h (bf16) -> next step's operand: transpose through LDS so
            // each store is 16 contiguous bytes (8 units of one row)
            __hip_bfloat16* hw = hx + mt * 256;
#pragma unroll
            for (int e = 0; e < 4; ++e) hw[(4 * fq + e) * 16 + fr] = to_bf16(hc[e]);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane < 32) {
                const int r = lane >> 1, hf = lane & 1;
                if (row_t0 + r < B) {
                    const u32x4 v = *(const u32x4*)(hw + r * 16 + hf * 8);
                    const int64_t off = ((int64_t)(t + 1) * B + row_t0 + r) * H + u0 + hf * 8;
                    st_sc1(r_h, (uint32_t)(off * 2), v);
                }
            }
            if (P.hup != nullptr) {   // pre-reset h for the layer above
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
                for (int e = 0; e < 4; ++e) hw[(4 * fq + e) * 16 + fr] = to_bf16(hn[e]);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (lane < 32) {
                    const int r = lane >> 1, hf = lane & 1;
                    if (row_t0 + r < B) {
                        const u32x4 v = *(const u32x4*)(hw + r * 16 + hf * 8);
                        const int64_t off = ((int64_t)t * nB + grow0 + row_t0 + r) * H + u0 + hf * 8;
                        st_sc1(rsrc(P.hup, (int64_t)T * nB * H * 2), (uint32_t)(off * 2), v);
                    }
                }
            }
        }
        publish(my_flags + wu, (uint32_t)(t + 1));
        // ---- saves for the backward (plain stores, drained off the critical path)
        if (epi) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (!bon[e]) continue;
                const int64_t ro = (int64_t)brow[e] * H + u;
                const int64_t so = (int64_t)t * nB * H + ro;
                float* ap = P.act + (int64_t)t * nB * 4 * H + (int64_t)brow[e] * 4 * H + u;
#pragma unroll
                for (int q = 0; q < 4; ++q) ap[q * H] = av[e][q];
                P.c_out[so] = cn[e];
                if (P.c_carry != nullptr) P.c_carry[so + (int64_t)nB * H] = c[e];
                if (P.h_out != nullptr) P.h_out[so] = hn[e];
                if (P.h_last != nullptr && t == tlast[e])
                    P.h_last[(int64_t)(brow[e] - grow0) * a.nd * H + g * H + u] = hn[e];
                if (t == Te - 1) {
                    P.hT[ro] = hc[e];
                    P.cT[ro] = c[e];
                }
            }
        }
    }
    // tails past the row block's last step: zero top outputs and carried-h
    // operand rows (plain stores; nothing in this launch reads them)
    if (epi && Te < T) {
        for (int t = Te; t < T; ++t) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (!bon[e]) continue;
                const int64_t ro = (int64_t)brow[e] * H + u;
                hl[((int64_t)(t + 1) * B + (brow[e] - grow0)) * H + u] = to_bf16(0.f);
                if (P.h_out != nullptr) P.h_out[(int64_t)t * nB * H + ro] = 0.f;
            }
        }
    }
    (void)ok;
}

template <int H, int MTW>
__global__ __launch_bounds__(NTHR) void lstm_persist_fwd(const PFwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int NW = H / U;
    const int per_l = a.nd * a.nrb * NW;
    int bid = blockIdx.x;
    const int l = bid / per_l;
    bid -= l * per_l;
    const int g = bid / (a.nrb * NW);
    bid -= g * a.nrb * NW;
    const int rb = bid / NW, wu = bid % NW;
    if constexpr (H == 256) {
        if (a.ly[l].kin != 0) {
            fwd_body<H, MTW, H>(a, l, g, rb, wu, smem);
            return;
        }
    }
    fwd_body<H, MTW, 0>(a, l, g, rb, wu, smem);
}

// =====================================================================================
// backward (reverse time)
// =====================================================================================
template <int H, int MTW, bool UP>
__device__ void bwd_body(const PBwdArgs& a, int l, int g, int rb, int wu, unsigned char* smem) {
    constexpr int G = 4 * H, KS = 8 / MTW, KP = G / KS, NKS = KP / 32, NW = H / U;
    constexpr int NCH = NKS > 8 ? 8 : NKS;     // k-steps per load batch
    const PBwdLayer& P = a.ly[l];
    __hip_bfloat16* Wr = (__hip_bfloat16*)smem;                          // [16][G]
    __hip_bfloat16* Wu = Wr + 16 * G;                                    // [16][G] (UP)
    f32x4* part = (f32x4*)(smem + (UP ? 2 : 1) * 16 * G * 2);            // [KS][MTW][2][64]
    __hip_bfloat16* gx = (__hip_bfloat16*)(part + KS * MTW * 2 * 64);    // [MTW][4][16][16]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int mt = w % MTW, kp = w / MTW;
    const int fr = lane & 15, fq = lane >> 4;
    const int B = a.B, nB = a.nd * B, T = a.T;
    const int u0 = wu * U;
    const int row_t0 = rb * 16 * MTW + mt * 16;
    const bool tile_on = row_t0 < B;
    const int64_t grow0 = (int64_t)g * B;

    stage_rows<false>(Wr, P.Wr + g * P.wr_gs, G, 16, G, H, u0);
    if (UP) stage_rows<false>(Wu, P.Wu, G, 16, G, H, u0);
    __syncthreads();

    // bf16 dG is direction-major ([nd][T][B][4H], like the carried h)
    __hip_bfloat16* const gl = P.dg_lp + (int64_t)g * T * B * G;
    const __amdgpu_buffer_rsrc_t r_g = rsrc(gl, (int64_t)T * B * G * 2);
    const __amdgpu_buffer_rsrc_t r_up = rsrc(UP ? (const void*)a.ly[l + 1].dg_lp : (const void*)P.dg_lp,
                                             (int64_t)T * nB * G * 2);
    uint32_t* my_flags = a.flags + (((int64_t)l * a.nd + g) * a.nrb + rb) * kFlagStride;
    const uint32_t* up_flags = UP ? a.flags + (((int64_t)(l + 1) * a.nd + g) * a.nrb + rb) * kFlagStride : nullptr;

    const bool epi = kp == 0 && tile_on;
    const int u = u0 + fr;
    int brow[4];
    bool bon[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int r = row_t0 + 4 * fq + e;
        bon[e] = epi && r < B;
        brow[e] = (int)grow0 + min(r, B - 1);
    }
    float dcr[4], dih[4], dic[4], dhl[4];
    int tlast[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        dcr[e] = (epi && P.dcT != nullptr) ? P.dcT[(int64_t)brow[e] * H + u] : 0.f;
        dih[e] = dic[e] = 0.f;
        tlast[e] = row_last_step(a.tlen, T, brow[e] - (int)grow0);
        dhl[e] = (epi && P.dh_last != nullptr) ? P.dh_last[(int64_t)(brow[e] - grow0) * a.nd * H + g * H + u] : 0.f;
    }
    const bool keep_on = P.keep < 1.0f;
    const int arow = (int)grow0 + min(row_t0 + fr, B - 1);
    bool ok = true;
    const int Te = row_block_steps(a.tlen, T, B, rb, 16 * MTW);

    // t = Te-1 .. 0 are cell steps; t = -1 only forms dh0 = dG_0 @ W_h^T
    for (int t = Te - 1; t >= -1; --t) {
        float ac[4][4], cnw[4], cpv[4], dho[4], rs[4];
        if (epi && t >= 0) {
            const int64_t so = (int64_t)t * nB * H;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int64_t ro = (int64_t)brow[e] * H + u;
                const float* ap = P.act + (int64_t)t * nB * G + (int64_t)brow[e] * G + u;
#pragma unroll
                for (int q = 0; q < 4; ++q) ac[e][q] = ap[q * H];
                cnw[e] = P.c_out[so + ro];
                cpv[e] = t == 0 ? P.c0[ro] : (P.c_carry != nullptr ? P.c_carry[so + ro] : P.c_out[so - (int64_t)nB * H + ro]);
                dho[e] = ((!UP && P.dh_out != nullptr) ? P.dh_out[so + ro] : 0.f) + (t == tlast[e] ? dhl[e] : 0.f);
                rs[e] = a.reset != nullptr ? a.reset[(int64_t)t * nB + brow[e]] : 0.f;
            }
        }
        f32x4 accr = {0.f, 0.f, 0.f, 0.f}, accu = {0.f, 0.f, 0.f, 0.f};
        if (tile_on) {
            const int k0 = kp * KP;
            // dG_l[t+1] @ W_h^T (own layer, previous reverse step)
            if (t < Te - 1) {
                ok = ok && wait_flags(my_flags, NW, (uint32_t)(T - 1 - t), a.err, g_persist_spin_limit);
                const uint32_t base = (uint32_t)(((int64_t)(t + 1) * B + (arow - grow0)) * G * 2);
#pragma unroll
                for (int kb = 0; kb < NKS; kb += NCH) {
                    bf16x8 af[NCH];
#pragma unroll
                    for (int j = 0; j < NCH; ++j) af[j] = ld_sc1(r_g, base + (uint32_t)((k0 + (kb + j) * 32 + fq * 8) * 2));
#pragma unroll
                    for (int j = 0; j < NCH; ++j)
                        accr = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[j], lds_frag(Wr, fr, G, (k0 + (kb + j) * 32) / 8 + fq),
                                                                       accr, 0, 0, 0);
                }
            }
            // dG_{l+1}[t] @ W_in_{l+1}^T (layer above, same step)
            if (UP && t >= 0) {
                ok = ok && wait_flags(up_flags, NW, (uint32_t)(T - t), a.err, g_persist_spin_limit);
                const uint32_t base = (uint32_t)(((int64_t)t * nB + arow) * G * 2);
#pragma unroll
                for (int kb = 0; kb < NKS; kb += NCH) {
                    bf16x8 af[NCH];
#pragma unroll
                    for (int j = 0; j < NCH; ++j) af[j] = ld_sc1(r_up, base + (uint32_t)((k0 + (kb + j) * 32 + fq * 8) * 2));
#pragma unroll
                    for (int j = 0; j < NCH; ++j)
                        accu = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[j], lds_frag(Wu, fr, G, (k0 + (kb + j) * 32) / 8 + fq),
                                                                       accu, 0, 0, 0);
                }
            }
            part[((kp * MTW + mt) * 2 + 0) * 64 + lane] = accr;
            if (UP) part[((kp * MTW + mt) * 2 + 1) * 64 + lane] = accu;
        }
        __syncthreads();
        if (t < 0) {   // dh0 = dG_0 @ W_h^T (no cell step)
            if (epi) {
                f32x4 s = part[(mt * 2) * 64 + lane];
#pragma unroll
                for (int p = 1; p < KS; ++p) s += part[((p * MTW + mt) * 2) * 64 + lane];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (!bon[e]) continue;
                    const int64_t ro = (int64_t)brow[e] * H + u;
                    P.dh0[ro] = T > 0 ? s[e] : (P.dhT ? P.dhT[ro] : 0.f);
                    P.dc0[ro] = dcr[e];
                    if (P.dinit_h != nullptr) {
                        P.dinit_h[ro] = dih[e];
                        P.dinit_c[ro] = dic[e];
                    }
                }
            }
            break;
        }
        float dy[4][4];
        f32x4 sr = {0.f, 0.f, 0.f, 0.f}, su = {0.f, 0.f, 0.f, 0.f};
        if (epi) {
            sr = part[(mt * 2) * 64 + lane];
#pragma unroll
            for (int p = 1; p < KS; ++p) sr += part[((p * MTW + mt) * 2) * 64 + lane];
            if (UP) {
                su = part[(mt * 2 + 1) * 64 + lane];
#pragma unroll
                for (int p = 1; p < KS; ++p) su += part[((p * MTW + mt) * 2 + 1) * 64 + lane];
            }
        }
        if (epi) {
            const uint32_t key = keep_on ? hash_key(*a.seed, P.stream, (uint32_t)t) : 0u;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int64_t ro = (int64_t)brow[e] * H + u;
                float dhr = sr[e];
                if (t == Te - 1) dhr = P.dhT != nullptr ? P.dhT[ro] : 0.f;
                const bool r = rs[e] != 0.f;
                const float dh = (UP ? su[e] : dho[e]) + (r ? 0.f : dhr);
                float dc = r ? 0.f : dcr[e];
                if (r) {
                    dih[e] += dhr;
                    dic[e] += dcr[e];
                }
                const float i = ac[e][0], tj = ac[e][1], f = ac[e][2], o = ac[e][3];
                const float th = tanhf(cnw[e]);
                dc += dh * o * (1.f - th * th);
                const float m = dropout_mult(keep_on, key, ro, P.keep);
                dy[e][0] = dc * tj * m * i * (1.f - i);
                dy[e][1] = dc * i * m * (1.f - tj * tj);
                dy[e][2] = dc * cpv[e] * f * (1.f - f);
                dy[e][3] = dh * th * o * (1.f - o);
                dcr[e] = dc * f;
            }
            // publish bf16 dG: [row][q*H + u0 .. u0+15] through LDS (16-byte stores)
            __hip_bfloat16* gw = gx + mt * 1024;
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int q = 0; q < 4; ++q) gw[(q * 16 + 4 * fq + e) * 16 + fr] = to_bf16(dy[e][q]);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int s = lane + 64 * k;            // 128 16-byte pieces: (q, row, half)
                const int q = s >> 5, r = (s >> 1) & 15, hf = s & 1;
                if (row_t0 + r < B) {
                    const u32x4 v = *(const u32x4*)(gw + (q * 16 + r) * 16 + hf * 8);
                    const int64_t off = ((int64_t)t * B + row_t0 + r) * G + q * H + u0 + hf * 8;
                    st_sc1(r_g, (uint32_t)(off * 2), v);
                }
            }
        }
        publish(my_flags + wu, (uint32_t)(T - t));
        if (epi && P.dg != nullptr) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (!bon[e]) continue;
                float* dp = P.dg + (int64_t)t * nB * G + (int64_t)brow[e] * G + u;
#pragma unroll
                for (int q = 0; q < 4; ++q) dp[q * H] = dy[e][q];
            }
        }
    }
    // dG tails past the row block's last step: zero (read by the weight /
    // input-projection gradients after the launch)
    if (epi && Te < T) {
        for (int t = Te; t < T; ++t) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (!bon[e]) continue;
                const int64_t go = (int64_t)t * nB * G + (int64_t)brow[e] * G + u;           // fp32 dG: [T][nd*B][4H]
                const int64_t gb = ((int64_t)t * B + (brow[e] - grow0)) * G + u;      // bf16 dG: direction-major
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    gl[gb + q * H] = to_bf16(0.f);
                    if (P.dg != nullptr) P.dg[go + q * H] = 0.f;
                }
            }
        }
    }
    (void)ok;
}

template <int H, int MTW>
__global__ __launch_bounds__(NTHR) void lstm_persist_bwd(const PBwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int NW = H / U;
    const int per_l = a.nd * a.nrb * NW;
    int bid = blockIdx.x;
    const int l = bid / per_l;
    bid -= l * per_l;
    const int g = bid / (a.nrb * NW);
    bid -= g * a.nrb * NW;
    const int rb = bid / NW, wu = bid % NW;
    if constexpr (H == 256) {
        if (a.ly[l].Wu != nullptr) {
            bwd_body<H, MTW, true>(a, l, g, rb, wu, smem);
            return;
        }
    }
    bwd_body<H, MTW, false>(a, l, g, rb, wu, smem);
}

// ---- host side ----------------------------------------------------------------------
// Row blocks of 16 MTW rows: MTW = 2 (32 rows, 4 K-slices per tile) by
// default; MTW = 4 (64 rows, 2 K-slices) when the 32-row grid would not fit
// one workgroup per CU -- a 256-row bidirectional 512 encoder is 2 x 4 x 32 =
// 256 workgroups instead of 512. The caller picks nrb = ceil(B / (16 MTW)).
inline int mtw_of(int B, int nrb) {
    if (nrb == (B + 31) / 32) return 2;
    if (nrb == (B + 63) / 64) return 4;
    return 0;
}

// dynamic LDS: weights (K = 2H when a layer reads the layer below) + partial
// tiles + the transposition buffer
inline size_t fwd_lds(int H, int L, int mtw) {
    const int K = L > 1 ? 2 * H : H;
    return (size_t)64 * K * 2 + (size_t)(8 / mtw) * mtw * 4 * 64 * 16 + (size_t)mtw * 256 * 2;
}
inline size_t bwd_lds(int H, int L, int mtw) {
    return (size_t)(L > 1 ? 2 : 1) * 16 * 4 * H * 2 + (size_t)(8 / mtw) * mtw * 2 * 64 * 16 + (size_t)mtw * 1024 * 2;
}

template <typename A, typename KF>
int launch_persist(KF kern, const A& a, size_t lds, hipStream_t s) {
    const int NW = a.H / U;
    const int grid = a.L * a.nd * a.nrb * NW;
    static const void* attr_done[16];
    bool have = false;
    for (const void* p : attr_done) have |= (p == (const void*)kern);
    if (!have) {
        if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return -9;
        for (auto& p : attr_done)
            if (p == nullptr) { p = (const void*)kern; break; }
    }
    if (!grid_fits((const void*)kern, NTHR, lds, grid)) return -8;
    // Zero the flag words with a kernel, not hipMemsetAsync: on MI355X with
    // torch's HIP 7.0 runtime a memset node captured into a HIP graph is not
    // ordered before the next kernel node on replay -- replays 2.. of a
    // captured persistent launch saw the previous replay's epochs and read
    // hand-off buffers before they were written (tests/test_persist_gpu.py::
    // test_persistent_graph_replay_matches_eager, with poisoned buffers).
    const int nflags = a.L * a.nd * a.nrb * kFlagStride;
    hipLaunchKernelGGL(zero_flags, dim3((nflags + 255) / 256), dim3(256), 0, s, a.flags, nflags);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NTHR), lds, s, a);
    return SKR_CHECK_LAUNCH();
}

template <typename A>
int check_common(const A& a) {
    if (a.T <= 0 || a.B <= 0) return 1;
    if (a.L < 1 || a.L > 2 || a.nd < 1 || a.nd > 2 || (a.L == 2 && a.nd != 1)) return -2;
    if (a.H != 256 && (a.H != 512 || a.L > 1)) return -2;   // two stacked 512 layers exceed LDS
    if (mtw_of(a.B, a.nrb) == 0) return -4;
    if (a.flags == nullptr || a.err == nullptr) return -6;
    if (a.tlen != nullptr && a.L != 1) return -7;   // stacked layers run the full T
    // 32-bit buffer offsets
    if ((int64_t)(a.T + 1) * a.nd * a.B * 4 * a.H * 2 > 0x7fffffffLL) return -11;
    return 0;
}

}  // namespace

SKR_API int skr_lstm_persist_fwd(const PFwdArgs* a, hipStream_t s) {
    int rc = check_common(*a);
    if (rc) return rc > 0 ? 0 : rc;
    for (int l = 0; l < a->L; ++l)
        if (a->ly[l].kin != (l == 0 ? 0 : a->H)) return -3;
    const int m = mtw_of(a->B, a->nrb);
    switch (a->H * 8 + m) {
        case 256 * 8 + 2: return launch_persist(lstm_persist_fwd<256, 2>, *a, fwd_lds(256, a->L, 2), s);
        case 512 * 8 + 2: return launch_persist(lstm_persist_fwd<512, 2>, *a, fwd_lds(512, a->L, 2), s);
        case 256 * 8 + 4: return launch_persist(lstm_persist_fwd<256, 4>, *a, fwd_lds(256, a->L, 4), s);
        case 512 * 8 + 4: return launch_persist(lstm_persist_fwd<512, 4>, *a, fwd_lds(512, a->L, 4), s);
    }
    return -2;
}

SKR_API int skr_lstm_persist_bwd(const PBwdArgs* a, hipStream_t s) {
    int rc = check_common(*a);
    if (rc) return rc > 0 ? 0 : rc;
    for (int l = 0; l < a->L; ++l)
        if ((a->ly[l].Wu != nullptr) != (l < a->L - 1)) return -3;
    const int m = mtw_of(a->B, a->nrb);
    switch (a->H * 8 + m) {
        case 256 * 8 + 2: return launch_persist(lstm_persist_bwd<256, 2>, *a, bwd_lds(256, a->L, 2), s);
        case 512 * 8 + 2: return launch_persist(lstm_persist_bwd<512, 2>, *a, bwd_lds(512, a->L, 2), s);
        case 256 * 8 + 4: return launch_persist(lstm_persist_bwd<256, 4>, *a, bwd_lds(256, a->L, 4), s);
        case 512 * 8 + 4: return launch_persist(lstm_persist_bwd<512, 4>, *a, bwd_lds(512, a->L, 4), s);
    }
    return -2;
}

// Spin bound of the persistent kernels' waits (0: the default). Host-side,
// between launches (the value is read at each bound check).
SKR_API int skr_persist_set_spin_limit(unsigned polls) {
    const unsigned v = polls ? polls : kHandoffSpinLimit;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_persist_spin_limit), &v, sizeof v, 0, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}

SKR_API int skr_lstm_persist_fwd_args_size() { return (int)sizeof(PFwdArgs); }
SKR_API int skr_lstm_persist_bwd_args_size() { return (int)sizeof(PBwdArgs); }
