// Fused mixture-density head: output projection on MFMA + MDN loss + dL/dz
// in ONE forward kernel, and hand-written MFMA kernels for its backward.
//
// Forward (mdn_head_fwd): a workgroup owns 64 rows of the decoder output X
// [N, Hd] (fp32) and ALL NOUTP output columns (NOUT = 3 + 6M <= 160):
//   z = drop(X) @ W + b   v_mfma_f32_16x16x32_bf16, X converted to bf16 (and
//                         dropout-masked) while loading its fragments, W^T
//                         K-chunks staged through LDS (shared by 4 waves)
//   -> z tile in LDS (never written to HBM) -> per-row MDN loss exactly as
//   csrc/mdn.hip (log-space bivariate normal, logsumexp, reference clamp or
//   Magenta eps/mask) -> per-row loss terms folded into per-workgroup partial
//   sums, dL/dz (for an upstream gradient of 1/N per row) written ONCE, bf16,
//   [N, NOUTP] -- the only O(N) output. A 1-workgroup finish kernel sums the
//   partials in a fixed order (deterministic) into (total, shape, pen).
// Backward (the upstream gradients of (total, shape, pen) arrive as device
// scalars: pen columns scale by g_total + g_pen, mixture columns by
// g_total + g_shape; no host sync):
//   mdn_head_dx: dX = (dz * scale) @ W^T (* dropout mask), [64 x 128] tiles,
//                K = NOUTP, W tile in LDS, fp32 output through an LDS
//                transpose (16-byte stores)
//   mdn_head_dw: [dW ; db] = [drop(X) | 1]^T @ (dz * scale): the reduction
//                runs over the N rows, so X and dz chunks are transposed
//                through LDS into MFMA operands; row range split over S
//                slabs, the bias gradient is the extra "ones" input row Hd
//   mdn_head_dw_reduce: sums the S slabs (fixed order) into dW, db.
//
// Reference: model.py:98-99 (xw_plus_b), model.py:112-178 (mixture
// coefficients, bivariate normal, loss, pen cross-entropy).
#include "common.h"

namespace {

using namespace skr;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kMaxNoutP = 160;        // NOUTP = NOUT rounded up to 32 (M <= 24)
constexpr int kRows = 64;             // rows per forward workgroup (4 waves x 16)
constexpr int kKC = 64;               // K chunk staged per LDS buffer
constexpr int kLdk = kKC + 8;         // padded LDS row (144 B): conflict-free fragment reads
constexpr float kLog2Pi = 1.8378770664093453f;

__device__ __forceinline__ float hw_sum(float v) {
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 32);
    return v;
}
__device__ __forceinline__ float hw_max(float v) {
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 32));
    return v;
}
__device__ __forceinline__ float drop_mult(bool on, uint32_t key, int64_t idx, float keep) {
    if (!on) return 1.f;
    return hash_uniform(key, (uint32_t)idx) < keep ? 1.0f / keep : 0.f;
}
__device__ __forceinline__ uint32_t pack_bf16(float a, float b) {
    return (uint32_t)__builtin_bit_cast(unsigned short, to_bf16(a)) |
           ((uint32_t)__builtin_bit_cast(unsigned short, to_bf16(b)) << 16);
}

struct HeadFwd {
    const float* X; int64_t ldx; int64_t N; int Hd;
    const __hip_bfloat16* Wt;        // [NOUTP][Hd] bf16 (rows >= NOUT zero)
    const float* bias;               // [NOUT]
    const float* tgt; int64_t ldt;   // [N][5]
    int M, NOUT, NOUTP, mode, mask_pen;
    float F, log_floor, inv_n;
    float keep; const int64_t* seed; uint32_t stream;   // dropout on X (keep >= 1: off)
    __hip_bfloat16* dz;              // [N][ldz] bf16 (columns < NOUTP written), or null (no gradient)
    float* part;                     // [2][nblocks] per-workgroup sums of the shape / pen terms
    int x_bf16;                      // X is bf16 (the decoder's saved bf16 h rows, row stride ldx)
    int64_t ldz;                     // dz row stride (>= NOUTP, multiple of 8)
};

// ---------------------------------------------------------------------------------
// forward: projection + loss + dz
// ---------------------------------------------------------------------------------
// X fragments of one K chunk for lane (fr, fq): row arow, k = kc * kKC +
// ks * 32 + fq * 8 .. +7 for ks = 0, 1 -- raw, converted at use
template <bool XB> struct XChunk { f32x4 v[2][2]; };
template <> struct XChunk<true> { u32x4 v[2]; };

constexpr int kWPieces = kMaxNoutP * (kKC / 8) / 256;   // 16-byte W^T pieces per thread per chunk (5)
// K chunks of X and W^T in flight per thread: 2 on bf16 X (230 registers, 2
// waves per SIMD), 1 on fp32 X (a deeper fp32 ring drops to 1 wave per SIMD)
template <bool XB> constexpr int fwd_ring() { return XB ? 2 : 1; }

template <bool XB>
__global__ __launch_bounds__(256) void mdn_head_fwd(const HeadFwd a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __hip_bfloat16* Bs = (__hip_bfloat16*)smem;                 // [2][NOUTP][kLdk]
    float* zt = (float*)smem;                                     // [kRows][NOUTP] (after the K loop)
    float* red = (float*)(smem + 2 * kMaxNoutP * kLdk * 2);       // [8 half-waves][2]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const int NOUTP = a.NOUTP, NC = NOUTP / 16, Hd = a.Hd;
    const int64_t row0 = (int64_t)blockIdx.x * kRows;
    const int64_t arow = min(row0 + w * 16 + fr, a.N - 1);
    const bool keep_on = a.keep < 1.0f;
    const uint32_t key = keep_on ? hash_key(*a.seed, a.stream, 0u) : 0u;

    f32x4 acc[kMaxNoutP / 16];
#pragma unroll
    for (int c = 0; c < kMaxNoutP / 16; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};

    // K loop: the W^T chunk [NOUTP][kKC] and this lane's X fragments are
    // loaded R_ chunks ahead into registers (every wait is for loads
    // issued a ring ago, not one round trip per chunk); W^T goes through a
    // double-buffered padded LDS tile, X straight into MFMA operands.
    constexpr int R_ = fwd_ring<XB>();
    const int nchunks = Hd / kKC, npieces = NOUTP * (kKC / 8);
    u32x4 wr[R_][kWPieces];
    XChunk<XB> xr[R_];
    auto load_w = [&](u32x4 (&r)[kWPieces], int kc) {
#pragma unroll
        for (int j = 0; j < kWPieces; ++j) {
            const int p = tid + 256 * j;
            if (p < npieces) r[j] = *(const u32x4*)(a.Wt + (int64_t)(p >> 3) * Hd + kc * kKC + (p & 7) * 8);
        }
    };
    auto store_w = [&](const u32x4 (&r)[kWPieces], int buf) {
        __hip_bfloat16* dst = Bs + buf * kMaxNoutP * kLdk;
#pragma unroll
        for (int j = 0; j < kWPieces; ++j) {
            const int p = tid + 256 * j;
            if (p < npieces) *(u32x4*)(dst + (p >> 3) * kLdk + (p & 7) * 8) = r[j];
        }
    };
    auto load_x = [&](XChunk<XB>& r, int kc) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int64_t o = arow * a.ldx + kc * kKC + ks * 32 + fq * 8;
            if constexpr (XB) {
                r.v[ks] = *(const u32x4*)((const __hip_bfloat16*)(const void*)a.X + o);
            } else {
                r.v[ks][0] = *(const f32x4*)(a.X + o);
                r.v[ks][1] = *(const f32x4*)(a.X + o + 4);
            }
        }
    };
    auto frag = [&](const XChunk<XB>& r, int ks, int kc) -> bf16x8 {
        const int k = kc * kKC + ks * 32 + fq * 8;
        float xs[8];
        if constexpr (XB) {
            if (!keep_on) return __builtin_bit_cast(bf16x8, r.v[ks]);
            const bf16x8 v = __builtin_bit_cast(bf16x8, r.v[ks]);
#pragma unroll
            for (int j = 0; j < 8; ++j) xs[j] = (float)v[j];
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                xs[j] = r.v[ks][0][j];
                xs[4 + j] = r.v[ks][1][j];
            }
        }
        if (keep_on) {
#pragma unroll
            for (int j = 0; j < 8; ++j) xs[j] *= drop_mult(true, key, arow * Hd + k + j, a.keep);
        }
        const u32x4 pk = {pack_bf16(xs[0], xs[1]), pack_bf16(xs[2], xs[3]), pack_bf16(xs[4], xs[5]),
                          pack_bf16(xs[6], xs[7])};
        return __builtin_bit_cast(bf16x8, pk);
    };
    // prologue: W^T chunk 0 into LDS; W^T chunks 1..R and X chunks 0..R-1 in flight
    load_w(wr[0], 0);
    store_w(wr[0], 0);
#pragma unroll
    for (int r = 1; r <= R_; ++r)
        if (r < nchunks) load_w(wr[r % R_], r);
#pragma unroll
    for (int r = 0; r < R_; ++r)
        if (r < nchunks) load_x(xr[r], r);
    __syncthreads();
    for (int kc0 = 0; kc0 < nchunks; kc0 += R_) {
#pragma unroll
        for (int r = 0; r < R_; ++r) {
            const int kc = kc0 + r;                       // slot of chunk kc: r; of chunk kc + 1: (r + 1) % R
            if (kc >= nchunks) break;                     // uniform
            if (kc + 1 < nchunks) {
                store_w(wr[(r + 1) % R_], (kc + 1) & 1);
                if (kc + 1 + R_ < nchunks) load_w(wr[(r + 1) % R_], kc + 1 + R_);
            }
            const bf16x8 A0 = frag(xr[r], 0, kc), A1 = frag(xr[r], 1, kc);
            if (kc + R_ < nchunks) load_x(xr[r], kc + R_);
            const __hip_bfloat16* Bc = Bs + (kc & 1) * kMaxNoutP * kLdk;
#pragma unroll
            for (int ks = 0; ks < kKC / 32; ++ks) {
                const bf16x8 A = ks == 0 ? A0 : A1;
#pragma unroll
                for (int c = 0; c < kMaxNoutP / 16; ++c) {
                    if (c < NC) {
                        const bf16x8 Bf = *(const bf16x8*)(Bc + (c * 16 + fr) * kLdk + ks * 32 + fq * 8);
                        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, Bf, acc[c], 0, 0, 0);
                    }
                }
            }
            __syncthreads();
        }
    }
    // ---- z tile (+bias) into LDS (reuses the staging buffers)
#pragma unroll
    for (int c = 0; c < kMaxNoutP / 16; ++c) {
        if (c < NC) {
            const int col = c * 16 + fr;
            const float bv = col < a.NOUT ? a.bias[col] : 0.f;
#pragma unroll
            for (int e = 0; e < 4; ++e) zt[(w * 16 + 4 * fq + e) * NOUTP + col] = acc[c][e] + bv;
        }
    }
    __syncthreads();

    // ---- per-row MDN loss: one row per 32-lane half-wave, lane k = component k
    const int hl = tid & 31, hw = tid >> 5;            // half-wave index 0..7
    const int M = a.M;
    float s_shape = 0.f, s_pen = 0.f;
    for (int rr = hw; rr < kRows; rr += 8) {
        const int64_t row = row0 + rr;
        if (row >= a.N) break;                         // whole half-waves exit together
        float* zr = zt + rr * NOUTP;
        const float* tr = a.tgt + row * a.ldt;
        const bool on = hl < M;
        const float x1 = tr[0], x2 = tr[1];
        const float p0 = tr[2], p1 = tr[3], p2 = tr[4];
        const float zpi = on ? zr[3 + hl] : -INFINITY;
        const float mpi = hw_max(zpi);
        const float epi = on ? __expf(zpi - mpi) : 0.f;
        const float spi = hw_sum(epi);
        const float logpi = zpi - mpi - __logf(spi);
        const float pi = epi / spi;
        float lp = -INFINITY, n1 = 0.f, n2 = 0.f, rho = 0.f, om = 1.f, Z = 0.f, s1 = 1.f, s2 = 1.f;
        if (on) {
            const float mu1 = zr[3 + M + hl], mu2 = zr[3 + 2 * M + hl];
            const float ls1 = zr[3 + 3 * M + hl], ls2 = zr[3 + 4 * M + hl];
            rho = tanhf(zr[3 + 5 * M + hl]);
            s1 = expf(ls1);
            s2 = expf(ls2);
            n1 = (x1 - mu1) / s1;
            n2 = (x2 - mu2) / s2;
            om = 1.f - rho * rho;
            Z = n1 * n1 + n2 * n2 - 2.f * rho * n1 * n2;
            lp = logpi - Z / (2.f * om) - kLog2Pi - ls1 - ls2 - 0.5f * logf(om);
        }
        const float mlp = hw_max(lp);
        const float elp = on ? expf(lp - mlp) : 0.f;
        const float slp = hw_sum(elp);
        const float logS = mlp + logf(slp);
        const float gam = elp / slp;
        float shape, gS;
        const float fs = 1.f - p2;
        if (a.mode == 0) {
            if (logS < a.log_floor) { shape = -a.log_floor; gS = 0.f; }
            else { shape = -logS; gS = -1.f; }
        } else {
            const float mx = fmaxf(logS, a.log_floor), mn = fminf(logS, a.log_floor);
            const float lae = mx + log1pf(expf(mn - mx));
            shape = -lae * fs;
            gS = -expf(logS - lae) * fs;
        }
        const float l0 = zr[0], l1 = zr[1], l2 = zr[2];
        const float ml = fmaxf(l0, fmaxf(l1, l2));
        const float e0 = expf(l0 - ml), e1 = expf(l1 - ml), e2 = expf(l2 - ml);
        const float se = e0 + e1 + e2, lse = ml + logf(se);
        const float ce = -(p0 * (l0 - lse) + p1 * (l1 - lse) + p2 * (l2 - lse));
        const float wgt = a.mode == 0 ? p2 + sqrtf(a.F) * p0 + a.F * p1 : (a.mask_pen ? fs : 1.f);
        s_shape += shape;
        s_pen += wgt * ce;
        if (a.dz != nullptr) {
            // every lane has read its z values above: overwrite the row with dz
            // (fp32, in place), converted + stored coalesced after the loop
            const float inv_n = a.inv_n;
            float d0 = 0.f, dpi = 0.f, dm1 = 0.f, dm2 = 0.f, ds1 = 0.f, ds2 = 0.f, drh = 0.f;
            if (hl < 3) {
                const float ps = p0 + p1 + p2;
                const float q = (hl == 0 ? e0 : hl == 1 ? e1 : e2) / se;
                const float pl = hl == 0 ? p0 : hl == 1 ? p1 : p2;
                d0 = inv_n * wgt * (q * ps - pl);
            }
            if (on) {
                const float g = inv_n * gS * gam;
                const float inv_om = 1.f / om;
                dpi = inv_n * gS * (gam - pi);
                dm1 = g * inv_om * (n1 - rho * n2) / s1;
                dm2 = g * inv_om * (n2 - rho * n1) / s2;
                ds1 = g * ((n1 * n1 - rho * n1 * n2) * inv_om - 1.f);
                ds2 = g * ((n2 * n2 - rho * n1 * n2) * inv_om - 1.f);
                drh = g * (n1 * n2 - rho * Z * inv_om + rho);
            }
            __builtin_amdgcn_wave_barrier();
            if (hl < 3) zr[hl] = d0;
            if (on) {
                zr[3 + hl] = dpi;
                zr[3 + M + hl] = dm1;
                zr[3 + 2 * M + hl] = dm2;
                zr[3 + 3 * M + hl] = ds1;
                zr[3 + 4 * M + hl] = ds2;
                zr[3 + 5 * M + hl] = drh;
            }
            for (int c = a.NOUT + hl; c < NOUTP; c += 32) zr[c] = 0.f;
        }
    }
    // ---- deterministic per-workgroup partial sums of the loss terms
    if (hl == 0) {
        red[hw * 2] = s_shape;
        red[hw * 2 + 1] = s_pen;
    }
    __syncthreads();
    if (tid == 0) {
        float ss = 0.f, sp = 0.f;
        for (int k = 0; k < 8; ++k) {
            ss += red[k * 2];
            sp += red[k * 2 + 1];
        }
        a.part[blockIdx.x] = ss;
        a.part[gridDim.x + blockIdx.x] = sp;
    }
    if (a.dz == nullptr) return;
    // ---- dz tile -> bf16, coalesced 16-byte stores
    const int per_row = NOUTP / 8;
    for (int p = tid; p < kRows * per_row; p += 256) {
        const int rr = p / per_row, c8 = (p - rr * per_row) * 8;
        const int64_t row = row0 + rr;
        if (row >= a.N) continue;
        const float* zr = zt + rr * NOUTP + c8;
        const u32x4 v = {pack_bf16(zr[0], zr[1]), pack_bf16(zr[2], zr[3]), pack_bf16(zr[4], zr[5]),
                         pack_bf16(zr[6], zr[7])};
        *(u32x4*)(a.dz + row * a.ldz + c8) = v;
    }
}

// one workgroup: out[0..2] = (shape + pen, shape, pen) means, fixed summation order
__global__ __launch_bounds__(256) void mdn_head_finish(const float* part, int nb, float inv_n, float* out) {
    __shared__ float r2[2][4];
    float ss = 0.f, sp = 0.f;
    for (int i = threadIdx.x; i < nb; i += 256) {
        ss += part[i];
        sp += part[nb + i];
    }
    ss = wave_sum(ss);
    sp = wave_sum(sp);
    if ((threadIdx.x & 63) == 0) {
        r2[0][threadIdx.x >> 6] = ss;
        r2[1][threadIdx.x >> 6] = sp;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const float s = ((r2[0][0] + r2[0][1]) + (r2[0][2] + r2[0][3])) * inv_n;
        const float p = ((r2[1][0] + r2[1][1]) + (r2[1][2] + r2[1][3])) * inv_n;
        out[0] = s + p;
        out[1] = s;
        out[2] = p;
    }
}

// ---------------------------------------------------------------------------------
// backward 1: dX = (dz * scale) @ W^T, dropout-masked
// ---------------------------------------------------------------------------------
struct HeadDx {
    const __hip_bfloat16* dz; int64_t N; int NOUTP;
    const __hip_bfloat16* Wb;        // [Hd][NOUTP] bf16 (cols >= NOUT zero)
    int Hd;
    const float* scale;              // [2]: pen columns, mixture columns
    float keep; const int64_t* seed; uint32_t stream;
    float* dX; int64_t lddx;
    int64_t ldz;                     // dz row stride
};

constexpr int kDxCols = 128;

__global__ __launch_bounds__(256) void mdn_head_dx(const HeadDx a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int NOUTP = a.NOUTP, ldw = NOUTP + 8;                   // padded LDS row
    __hip_bfloat16* Ws = (__hip_bfloat16*)smem;                   // [128][NOUTP + 8]
    float* ot = (float*)(smem + (size_t)kDxCols * ldw * 2);       // [4 waves][16][128 + 4]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const int64_t row0 = (int64_t)blockIdx.x * kRows;
    const int col0 = blockIdx.y * kDxCols;
    for (int p = tid; p < kDxCols * (NOUTP / 8); p += 256) {
        const int n = p / (NOUTP / 8), c = p - n * (NOUTP / 8);
        *(u32x4*)(Ws + n * ldw + c * 8) = *(const u32x4*)(a.Wb + (int64_t)(col0 + n) * NOUTP + c * 8);
    }
    __syncthreads();
    const float sp = a.scale[0], sm = a.scale[1];
    const int64_t arow = min(row0 + w * 16 + fr, a.N - 1);
    f32x4 acc[kDxCols / 16];
#pragma unroll
    for (int c = 0; c < kDxCols / 16; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int ks = 0; ks < NOUTP / 32; ++ks) {
        const int k = ks * 32 + fq * 8;
        u32x4 raw = *(const u32x4*)(a.dz + arow * a.ldz + k);
        if (k < 8) {   // pen columns 0..2 carry the pen scale
            bf16x8 v = __builtin_bit_cast(bf16x8, raw);
            float f[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] = (float)v[j] * (k + j < 3 ? sp : sm);
            raw = u32x4{pack_bf16(f[0], f[1]), pack_bf16(f[2], f[3]), pack_bf16(f[4], f[5]), pack_bf16(f[6], f[7])};
        } else if (sm != 1.0f) {
            bf16x8 v = __builtin_bit_cast(bf16x8, raw);
            float f[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] = (float)v[j] * sm;
            raw = u32x4{pack_bf16(f[0], f[1]), pack_bf16(f[2], f[3]), pack_bf16(f[4], f[5]), pack_bf16(f[6], f[7])};
        }
        const bf16x8 A = __builtin_bit_cast(bf16x8, raw);
#pragma unroll
        for (int c = 0; c < kDxCols / 16; ++c) {
            const bf16x8 Bf = *(const bf16x8*)(Ws + (c * 16 + fr) * ldw + k);
            acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, Bf, acc[c], 0, 0, 0);
        }
    }
    // transpose through LDS -> 16-byte row stores (+ dropout mask)
    float* ow = ot + w * 16 * (kDxCols + 4);
#pragma unroll
    for (int c = 0; c < kDxCols / 16; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) ow[(4 * fq + e) * (kDxCols + 4) + c * 16 + fr] = acc[c][e];
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const bool keep_on = a.keep < 1.0f;
    const uint32_t key = keep_on ? hash_key(*a.seed, a.stream, 0u) : 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int p = lane + 64 * j;           // 512 pieces: row p >> 5, 4 cols (p & 31) * 4
        const int rr = p >> 5, c4 = (p & 31) * 4;
        const int64_t row = row0 + w * 16 + rr;
        if (row >= a.N) continue;
        f32x4 v = *(const f32x4*)(ow + rr * (kDxCols + 4) + c4);
        if (keep_on) {
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] *= drop_mult(true, key, row * a.Hd + col0 + c4 + q, a.keep);
        }
        *(f32x4*)(a.dX + row * a.lddx + col0 + c4) = v;
    }
}

// ---------------------------------------------------------------------------------
// backward 2: [dW ; db] slabs = [drop(X) | 1]^T @ (dz * scale) over a row range
// ---------------------------------------------------------------------------------
struct HeadDw {
    const float* X; int64_t ldx; int64_t N; int Hd;
    const __hip_bfloat16* dz; int NOUTP;
    const float* scale;
    float keep; const int64_t* seed; uint32_t stream;
    float* slab;                     // [S][Hd + 64][NOUTP]
    int64_t rows_per;                // rows per slab (multiple of 32)
    int64_t ldz;                     // dz row stride
    int x_bf16;                      // X is bf16 (row stride ldx)
};

constexpr int kDwRows = 64;          // input features (dW rows) per workgroup
constexpr int kRC = 32;              // rows per staged chunk (= MFMA K)

template <bool XB>
__global__ __launch_bounds__(256) void mdn_head_dw(const HeadDw a) {
    __shared__ __attribute__((aligned(16))) __hip_bfloat16 xt[kDwRows][kRC + 8];        // [feature][row]
    __shared__ __attribute__((aligned(16))) __hip_bfloat16 gt[kMaxNoutP][kRC + 8];      // [out col][row]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const int NOUTP = a.NOUTP, NC = NOUTP / 16, Hd = a.Hd;
    const int f0 = blockIdx.x * kDwRows;            // first feature (Hd = the ones row)
    const int s = blockIdx.y;
    const int64_t r_begin = (int64_t)s * a.rows_per, r_end = min(a.N, r_begin + a.rows_per);
    const float sp = a.scale[0], sm = a.scale[1];
    const bool keep_on = a.keep < 1.0f;
    const uint32_t key = keep_on ? hash_key(*a.seed, a.stream, 0u) : 0u;
    f32x4 acc[kMaxNoutP / 16];
#pragma unroll
    for (int c = 0; c < kMaxNoutP / 16; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int64_t r0 = r_begin; r0 < r_end; r0 += kRC) {
        // X chunk [32 rows][64 features] -> xt[feature][row] (bf16, dropout)
        for (int p = tid; p < kRC * (kDwRows / 4); p += 256) {
            const int rr = p / (kDwRows / 4), f4 = (p - rr * (kDwRows / 4)) * 4;
            const int64_t row = r0 + rr;
            float v[4] = {0.f, 0.f, 0.f, 0.f};
            if (row < r_end) {
                if (f0 + f4 + 3 < Hd) {
                    if constexpr (XB) {
                        const uint2 u = *(const uint2*)((const __hip_bfloat16*)(const void*)a.X + row * a.ldx + f0 + f4);
                        v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
                        v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
                    } else {
                        const f32x4 x = *(const f32x4*)(a.X + row * a.ldx + f0 + f4);
                        v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
                    }
                    if (keep_on) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) v[q] *= drop_mult(true, key, row * Hd + f0 + f4 + q, a.keep);
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int f = f0 + f4 + q;
                        const float xf = f >= Hd ? 0.f
                                         : XB ? __bfloat162float(((const __hip_bfloat16*)(const void*)a.X)[row * a.ldx + f])
                                                    : a.X[row * a.ldx + f];
                        v[q] = f < Hd ? xf * drop_mult(keep_on, key, row * Hd + f, a.keep) : (f == Hd ? 1.f : 0.f);
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) xt[f4 + q][rr] = to_bf16(v[q]);
        }
        // dz chunk [32 rows][NOUTP] -> gt[col][row] (scaled)
        for (int p = tid; p < kRC * (NOUTP / 8); p += 256) {
            const int rr = p / (NOUTP / 8), c8 = (p - rr * (NOUTP / 8)) * 8;
            const int64_t row = r0 + rr;
            bf16x8 v = {};
            if (row < r_end) v = __builtin_bit_cast(bf16x8, *(const u32x4*)(a.dz + row * a.ldz + c8));
#pragma unroll
            for (int j = 0; j < 8; ++j) gt[c8 + j][rr] = to_bf16((float)v[j] * (c8 + j < 3 ? sp : sm));
        }
        __syncthreads();
        // wave w: features 16w .. 16w+15 x all output columns, K = 32 rows
        const bf16x8 A = *(const bf16x8*)(&xt[w * 16 + fr][fq * 8]);
#pragma unroll
        for (int c = 0; c < kMaxNoutP / 16; ++c) {
            if (c < NC) {
                const bf16x8 Bf = *(const bf16x8*)(&gt[c * 16 + fr][fq * 8]);
                acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, Bf, acc[c], 0, 0, 0);
            }
        }
        __syncthreads();
    }
    float* out = a.slab + ((int64_t)s * (Hd + 64) + f0 + w * 16) * NOUTP;
#pragma unroll
    for (int c = 0; c < kMaxNoutP / 16; ++c) {
        if (c < NC) {
#pragma unroll
            for (int e = 0; e < 4; ++e) out[(4 * fq + e) * NOUTP + c * 16 + fr] = acc[c][e];
        }
    }
}

__global__ __launch_bounds__(256) void mdn_head_dw_reduce(const float* slab, int S, int Hd, int NOUTP, int NOUT,
                                                          float* dW, float* db) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t total = (int64_t)(Hd + 1) * NOUT;
    if (i >= total) return;
    const int f = (int)(i / NOUT), c = (int)(i - (int64_t)f * NOUT);
    float v = 0.f;
    for (int s = 0; s < S; ++s) v += slab[((int64_t)s * (Hd + 64) + f) * NOUTP + c];
    if (f < Hd) dW[(int64_t)f * NOUT + c] = v;
    else db[c] = v;
}

inline size_t fwd_lds() { return (size_t)2 * kMaxNoutP * kLdk * 2 + 64; }

}  // namespace

SKR_API int skr_mdn_head_fwd(const HeadFwd* a, float* out3, hipStream_t s) {
    if (a->M < 1 || a->M > 24 || a->NOUT != 3 + 6 * a->M || a->NOUTP % 32 || a->NOUTP < a->NOUT ||
        a->NOUTP > kMaxNoutP)
        return -2;
    if (a->Hd % kKC != 0 || a->ldx % (a->x_bf16 ? 8 : 4) != 0 || ((uintptr_t)a->X & 15)) return -3;
    if (a->dz != nullptr && (a->ldz < a->NOUTP || a->ldz % 8 || ((uintptr_t)a->dz & 15))) return -4;
    if (a->N <= 0) return 0;
    const int nb = (int)((a->N + kRows - 1) / kRows);
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute((const void*)mdn_head_fwd<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)fwd_lds()) != hipSuccess ||
            hipFuncSetAttribute((const void*)mdn_head_fwd<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)fwd_lds()) != hipSuccess)
            return -9;
        attr = true;
    }
    // the z tile reuses the staging buffers: kRows * NOUTP floats must fit
    static_assert((size_t)kRows * kMaxNoutP * 4 <= (size_t)2 * kMaxNoutP * kLdk * 2, "z tile fits");
    if (a->x_bf16) hipLaunchKernelGGL(mdn_head_fwd<true>, dim3(nb), dim3(256), fwd_lds(), s, *a);
    else hipLaunchKernelGGL(mdn_head_fwd<false>, dim3(nb), dim3(256), fwd_lds(), s, *a);
    hipLaunchKernelGGL(mdn_head_finish, dim3(1), dim3(256), 0, s, a->part, nb, a->inv_n, out3);
    return SKR_CHECK_LAUNCH();
}

SKR_API int skr_mdn_head_nblocks(int64_t N) { return (int)((N + kRows - 1) / kRows); }

SKR_API int skr_mdn_head_dx(const HeadDx* a, hipStream_t s) {
    if (a->Hd % kDxCols != 0 || a->NOUTP % 32 || a->NOUTP > kMaxNoutP || a->lddx % 4 || a->ldz < a->NOUTP ||
        a->ldz % 8)
        return -2;
    if (a->N <= 0) return 0;
    const size_t lds = (size_t)kDxCols * (a->NOUTP + 8) * 2 + (size_t)4 * 16 * (kDxCols + 4) * 4;
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute((const void*)mdn_head_dx, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)((size_t)kDxCols * (kMaxNoutP + 8) * 2 + (size_t)4 * 16 * (kDxCols + 4) * 4)) !=
            hipSuccess)
            return -9;
        attr = true;
    }
    hipLaunchKernelGGL(mdn_head_dx, dim3((unsigned)((a->N + kRows - 1) / kRows), a->Hd / kDxCols), dim3(256), lds, s,
                       *a);
    return SKR_CHECK_LAUNCH();
}

// slab: [S][Hd + 64][NOUTP] fp32 scratch; dW [Hd][NOUT], db [NOUT] outputs.
SKR_API int skr_mdn_head_dw(const HeadDw* a, int S, int NOUT, float* dW, float* db, hipStream_t s) {
    if (a->NOUTP % 32 || a->NOUTP > kMaxNoutP || a->rows_per % kRC || a->ldx % 4 || S < 1 || a->ldz < a->NOUTP ||
        a->ldz % 8)
        return -2;
    if (a->N <= 0) return 0;
    const int nf = (a->Hd + 1 + kDwRows - 1) / kDwRows;   // + the ones row (bias)
    if (a->x_bf16) hipLaunchKernelGGL(mdn_head_dw<true>, dim3(nf, S), dim3(256), 0, s, *a);
    else hipLaunchKernelGGL(mdn_head_dw<false>, dim3(nf, S), dim3(256), 0, s, *a);
    const int64_t total = (int64_t)(a->Hd + 1) * NOUT;
    hipLaunchKernelGGL(mdn_head_dw_reduce, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, a->slab, S, a->Hd,
                       a->NOUTP, NOUT, dW, db);
    return SKR_CHECK_LAUNCH();
}

SKR_API int skr_mdn_head_fwd_args_size() { return (int)sizeof(HeadFwd); }
SKR_API int skr_mdn_head_dx_args_size() { return (int)sizeof(HeadDx); }
SKR_API int skr_mdn_head_dw_args_size() { return (int)sizeof(HeadDw); }
