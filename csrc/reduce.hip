// Column reductions over the [T*B, C] per-step saves, for the parameter
// gradients that are sums over every (time, row) position: LayerNorm gamma /
// beta (sum dy*xhat, sum dy), biases (sum dg). One pass reads X (and Y) once
// -- instead of an elementwise product materialised at full size and a
// second reduction kernel -- and handles a two-level row index (i < R1 with
// stride s1, j < R2 with stride s2) so per-direction groups of the
// bidirectional encoder ([T, nd, B, C] views) reduce without a copy.
//
// Grid (ceil(C/256), RS): thread = one column, block row RS_idx owns a slice
// of the R1*R2 rows; per-slice partial sums go to part[RS][C] (fp32),
// summed by a deterministic second pass. RS is chosen by the caller
// (ops/reduce.py): about 1024 / ceil(C/256) slices, capped at R/16 rows per
// slice -- e.g. the [30000, 123] MDN-head bias gradient runs RS = 1024
// slices of ~30 rows.
#include "common.h"

namespace {

template <bool XBF16>
__device__ __forceinline__ float ldx(const void* x, int64_t i) {
    if constexpr (XBF16) return __bfloat162float(((const __hip_bfloat16*)x)[i]);
    else return ((const float*)x)[i];
}

// V consecutive columns from element offset i (V = 8: one 16-byte bf16 load;
// V = 4: one 8-byte bf16 or 16-byte fp32 vector load per row; V = 1: scalar)
template <bool BF, int V>
__device__ __forceinline__ void ldv(const void* x, int64_t i, float (&v)[V]) {
    if constexpr (V == 8) {
        static_assert(BF, "8-column loads: bf16 only");
        const uint4 u = *(const uint4*)((const __hip_bfloat16*)x + i);
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v[2 * k] = __uint_as_float(w[k] << 16);
            v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
        }
    } else if constexpr (V == 4) {
        if constexpr (BF) {
            const uint2 u = *(const uint2*)((const __hip_bfloat16*)x + i);
            v[0] = __uint_as_float(u.x << 16);
            v[1] = __uint_as_float(u.x & 0xffff0000u);
            v[2] = __uint_as_float(u.y << 16);
            v[3] = __uint_as_float(u.y & 0xffff0000u);
        } else {
            const float4 f = *(const float4*)((const float*)x + i);
            v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
        }
    } else {
        v[0] = ldx<BF>(x, i);
    }
}

template <bool XBF16, bool YBF16, int V>
__global__ __launch_bounds__(256) void colsum_kernel(const void* __restrict__ X, const void* __restrict__ Y,
                                                     int64_t R1, int64_t s1, int64_t R2, int64_t s2, int C,
                                                     float* __restrict__ part_xy, float* __restrict__ part_x) {
    const int c = (blockIdx.x * 256 + threadIdx.x) * V;
    if (c >= C) return;
    const int64_t R = R1 * R2;
    const int64_t per = (R + gridDim.y - 1) / gridDim.y;
    const int64_t r0 = blockIdx.y * per, r1 = min(R, r0 + per);
    float sxy[V], sx[V];
#pragma unroll
    for (int k = 0; k < V; ++k) sxy[k] = sx[k] = 0.f;
    // walk (i, j) incrementally: no 64-bit division per element
    int64_t i = r0 / R2, j = r0 % R2;
    int64_t r = r0;
    constexpr int U = V == 4 ? 2 : 4;     // rows in flight per thread
    for (; r + U <= r1; r += U) {
        float xv[U][V], yv[U][V];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int64_t off = i * s1 + j * s2 + c;
            ldv<XBF16, V>(X, off, xv[k]);
            if (Y) ldv<YBF16, V>(Y, off, yv[k]);
            else
#pragma unroll
                for (int e = 0; e < V; ++e) yv[k][e] = 0.f;
            if (++j == R2) {
                j = 0;
                ++i;
            }
        }
#pragma unroll
        for (int k = 0; k < U; ++k)
#pragma unroll
            for (int e = 0; e < V; ++e) {
                sx[e] += xv[k][e];
                sxy[e] += xv[k][e] * yv[k][e];
            }
    }
    for (; r < r1; ++r) {
        const int64_t off = i * s1 + j * s2 + c;
        float xv[V], yv[V];
        ldv<XBF16, V>(X, off, xv);
        if (Y) ldv<YBF16, V>(Y, off, yv);
#pragma unroll
        for (int e = 0; e < V; ++e) {
            sx[e] += xv[e];
            if (Y) sxy[e] += xv[e] * yv[e];
        }
        if (++j == R2) {
            j = 0;
            ++i;
        }
    }
#pragma unroll
    for (int e = 0; e < V; ++e) {
        part_x[(int64_t)blockIdx.y * C + c + e] = sx[e];
        if (Y) part_xy[(int64_t)blockIdx.y * C + c + e] = sxy[e];
    }
}

// Second pass: out[c] = sum over the RS row-slice partials (out_xy null when
// there is no Y). Workgroup = 64 columns x 4 waves; wave w sums slices
// w, w + 4, ... eight loads in flight at a time, then the four wave sums are
// added in wave order -- deterministic.
__global__ __launch_bounds__(256) void colsum_finish(const float* __restrict__ part_xy, const float* __restrict__ part_x,
                                                     int RS, int C, float* __restrict__ out_xy,
                                                     float* __restrict__ out_x) {
    __shared__ float red[2][4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + lane, cc = min(c, C - 1);
    float sx = 0.f, sxy = 0.f;
    for (int r0 = w; r0 < RS; r0 += 32) {
        float tx[8], txy[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int r = min(r0 + 4 * k, RS - 1);
            tx[k] = part_x[(int64_t)r * C + cc];
            txy[k] = out_xy ? part_xy[(int64_t)r * C + cc] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const bool on = r0 + 4 * k < RS;
            sx += on ? tx[k] : 0.f;
            sxy += on ? txy[k] : 0.f;
        }
    }
    red[0][w][lane] = sx;
    red[1][w][lane] = sxy;
    __syncthreads();
    if (w != 0 || c >= C) return;
    out_x[c] = ((red[0][0][lane] + red[0][1][lane]) + red[0][2][lane]) + red[0][3][lane];
    if (out_xy) out_xy[c] = ((red[1][0][lane] + red[1][1][lane]) + red[1][2][lane]) + red[1][3][lane];
}

}  // namespace

// Both passes: partials into part_* ([RS][C] each), then the column totals
// into out_xy / out_x (out_xy ignored without Y).
SKR_API int skr_colsum2(const void* X, int x_kind, const void* Y, int y_kind, int64_t R1, int64_t s1, int64_t R2,
                        int64_t s2, int C, int RS, float* part_xy, float* part_x, float* out_xy, float* out_x,
                        hipStream_t s);

// x_kind / y_kind: 1 bf16, 2 fp32. Y (same strides) may be null (then part_xy unused).
// Four columns per thread when C, the strides and the bases allow 8-byte
// (bf16) / 16-byte (fp32) vector loads.
SKR_API int skr_colsum(const void* X, int x_kind, const void* Y, int y_kind, int64_t R1, int64_t s1, int64_t R2,
                       int64_t s2, int C, int RS, float* part_xy, float* part_x, hipStream_t s) {
    if (C <= 0 || RS <= 0 || R1 * R2 <= 0) return -2;
    const bool xb = x_kind == 1, yb = y_kind == 1;
    const uintptr_t al = (uintptr_t)X | (uintptr_t)(Y ? Y : X);
    const bool v4 = C % 4 == 0 && s1 % 4 == 0 && s2 % 4 == 0 && (al & 15) == 0;
    const int V = v4 ? 4 : 1;
    const dim3 grid((C / V + 255) / 256, RS);
#define SKR_CS(XB, YB, VV) hipLaunchKernelGGL((colsum_kernel<XB, YB, VV>), grid, dim3(256), 0, s, X, Y, R1, s1, R2, s2, C, part_xy, part_x)
    if (v4) {
        if (xb && yb) SKR_CS(true, true, 4);
        else if (xb) SKR_CS(true, false, 4);
        else if (yb) SKR_CS(false, true, 4);
        else SKR_CS(false, false, 4);
    } else {
        if (xb && yb) SKR_CS(true, true, 1);
        else if (xb) SKR_CS(true, false, 1);
        else if (yb) SKR_CS(false, true, 1);
        else SKR_CS(false, false, 1);
    }
#undef SKR_CS
    return SKR_CHECK_LAUNCH();
}

SKR_API int skr_colsum2(const void* X, int x_kind, const void* Y, int y_kind, int64_t R1, int64_t s1, int64_t R2,
                        int64_t s2, int C, int RS, float* part_xy, float* part_x, float* out_xy, float* out_x,
                        hipStream_t s) {
    const int rc = skr_colsum(X, x_kind, Y, y_kind, R1, s1, R2, s2, C, RS, part_xy, part_x, s);
    if (rc != 0) return rc;
    hipLaunchKernelGGL(colsum_finish, dim3((C + 63) / 64), dim3(256), 0, s, part_xy, part_x, RS, C,
                       Y ? out_xy : nullptr, out_x);
    return SKR_CHECK_LAUNCH();
}

// Several column reductions in ONE launch per pass (the LayerNorm gamma /
// beta gradients of a HyperLSTM step are four: [T*B, 8192 | 2048 | 1024 |
// 256]). The narrow ones are latency-bound and would each pay a kernel
// boundary and a tail on their own; here their workgroups fill the chip
// beside the wide one's. Vector path only (NC columns per thread: C, the
// strides and the bases multiples of NC elements; NC = 8 -- one 16-byte load
// per row and operand -- when every operand is bf16, else 4).
struct CsJob {
    const void* X; const void* Y;          // Y may be null
    int64_t R1, s1, R2, s2;
    int C, RS, xbf, ybf;                    // xbf / ybf: 1 bf16, 0 fp32
    float* part_xy; float* part_x;          // [RS][C] each
    float* out_xy; float* out_x;            // [C] (out_xy unused without Y)
};
constexpr int kCsMax = 4;
struct CsJobs {
    CsJob j[kCsMax];
    int n;
    int start[kCsMax + 1];                  // first-pass workgroups: prefix sums of RS * ceil(C / (256 NC))
    int fstart[kCsMax + 1];                 // finish workgroups: prefix sums of ceil(C / 64)
};

namespace {

// KIND 0: operand dtypes read per job at run time; KIND 1: every X and Y
// bf16 (the LayerNorm saves of bf16 training), fixed at compile time
template <int KIND, int NC>
__device__ __forceinline__ void ldn(const void* x, int64_t i, bool bf, float (&v)[NC]) {
    if constexpr (NC == 8) ldv<true, 8>(x, i, v);
    else if (KIND == 1 || bf) ldv<true, 4>(x, i, v);
    else ldv<false, 4>(x, i, v);
}

// Thread mapping per job: cq = min(C / NC, 256) column groups x rg = 256 / cq
// row groups per workgroup (narrow reductions: C = 256, NC = 4 -> 64 x 4), the
// workgroup's rows split over the row groups and the groups summed in LDS
// in a fixed order, one partial row per workgroup: narrow reductions keep
// 256 threads busy per workgroup and few rows in flight per thread.
constexpr int kCsRowsInFlight = 8;

template <int KIND, int NC>
__global__ __launch_bounds__(256) void colsum_multi_kernel(const CsJobs jobs) {
    static_assert(NC == 4 || (NC == 8 && KIND == 1), "8 columns per thread: bf16 operands");
    __shared__ float red[2][256][NC];
    int q = 0;
    while (q + 1 < jobs.n && (int)blockIdx.x >= jobs.start[q + 1]) ++q;
    const CsJob& J = jobs.j[q];
    const int local = blockIdx.x - jobs.start[q];
    const int cq = min(J.C / NC, 256), rg = 256 / cq;
    const int cb = (J.C / NC + cq - 1) / cq;
    const int rs = local / cb, cbi = local - rs * cb;
    const int tq = threadIdx.x % cq, grp = threadIdx.x / cq;
    const int c = (cbi * cq + tq) * NC;
    const bool on = c < J.C && grp < rg;
    const int64_t R = J.R1 * J.R2;
    const int64_t per = (R + J.RS - 1) / J.RS;
    const int64_t w0 = rs * per, w1 = min(R, w0 + per);
    const int64_t gper = (w1 - w0 + rg - 1) / rg;
    const int64_t r0 = w0 + grp * gper, r1 = min(w1, r0 + gper);
    float sxy[NC], sx[NC];
#pragma unroll
    for (int e = 0; e < NC; ++e) sxy[e] = sx[e] = 0.f;
    if (on && r0 < r1) {
        int64_t i = r0 / J.R2, j = r0 % J.R2;
        int64_t r = r0;
        // kRowsInFlight rows loaded before any is summed (rows still summed in
        // order: the result does not depend on the unroll)
        constexpr int U = kCsRowsInFlight;
        for (; r + U <= r1; r += U) {
            float xv[U][NC], yv[U][NC];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int64_t off = i * J.s1 + j * J.s2 + c;
                ldn<KIND, NC>(J.X, off, J.xbf, xv[k]);
                if (J.Y) ldn<KIND, NC>(J.Y, off, J.ybf, yv[k]);
                else
#pragma unroll
                    for (int e = 0; e < NC; ++e) yv[k][e] = 0.f;
                if (++j == J.R2) {
                    j = 0;
                    ++i;
                }
            }
#pragma unroll
            for (int k = 0; k < U; ++k)
#pragma unroll
                for (int e = 0; e < NC; ++e) {
                    sx[e] += xv[k][e];
                    sxy[e] += xv[k][e] * yv[k][e];
                }
        }
        for (; r < r1; ++r) {
            const int64_t off = i * J.s1 + j * J.s2 + c;
            float xv[NC], yv[NC];
            ldn<KIND, NC>(J.X, off, J.xbf, xv);
            if (J.Y) ldn<KIND, NC>(J.Y, off, J.ybf, yv);
            else
#pragma unroll
                for (int e = 0; e < NC; ++e) yv[e] = 0.f;
#pragma unroll
            for (int e = 0; e < NC; ++e) {
                sx[e] += xv[e];
                sxy[e] += xv[e] * yv[e];
            }
            if (++j == J.R2) {
                j = 0;
                ++i;
            }
        }
    }
    const int64_t o = (int64_t)rs * J.C + c;
    if (rg == 1) {
        if (on) {
#pragma unroll
            for (int e = 0; e < NC; e += 4) {
                *(float4*)(J.part_x + o + e) = float4{sx[e], sx[e + 1], sx[e + 2], sx[e + 3]};
                if (J.Y) *(float4*)(J.part_xy + o + e) = float4{sxy[e], sxy[e + 1], sxy[e + 2], sxy[e + 3]};
            }
        }
        return;
    }
#pragma unroll
    for (int e = 0; e < NC; ++e) {
        red[0][threadIdx.x][e] = sx[e];
        red[1][threadIdx.x][e] = sxy[e];
    }
    __syncthreads();
    if (grp != 0 || !on) return;
    float tx[NC], txy[NC];
#pragma unroll
    for (int e = 0; e < NC; ++e) {
        tx[e] = red[0][tq][e];
        txy[e] = red[1][tq][e];
    }
    for (int g2 = 1; g2 < rg; ++g2)   // fixed order: deterministic
#pragma unroll
        for (int e = 0; e < NC; ++e) {
            tx[e] += red[0][g2 * cq + tq][e];
            txy[e] += red[1][g2 * cq + tq][e];
        }
#pragma unroll
    for (int e = 0; e < NC; e += 4) {
        *(float4*)(J.part_x + o + e) = float4{tx[e], tx[e + 1], tx[e + 2], tx[e + 3]};
        if (J.Y) *(float4*)(J.part_xy + o + e) = float4{txy[e], txy[e + 1], txy[e + 2], txy[e + 3]};
    }
}

// colsum_finish of every job, one launch (the same fixed summation order)
__global__ __launch_bounds__(256) void colsum_multi_finish(const CsJobs jobs) {
    int q = 0;
    while (q + 1 < jobs.n && (int)blockIdx.x >= jobs.fstart[q + 1]) ++q;
    const CsJob& J = jobs.j[q];
    __shared__ float red[2][4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = (blockIdx.x - jobs.fstart[q]) * 64 + lane, cc = min(c, J.C - 1);
    const bool hy = J.Y != nullptr;
    float sx = 0.f, sxy = 0.f;
    for (int r0 = w; r0 < J.RS; r0 += 32) {
        float tx[8], txy[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int rr = min(r0 + 4 * k, J.RS - 1);
            tx[k] = J.part_x[(int64_t)rr * J.C + cc];
            txy[k] = hy ? J.part_xy[(int64_t)rr * J.C + cc] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const bool on = r0 + 4 * k < J.RS;
            sx += on ? tx[k] : 0.f;
            sxy += on ? txy[k] : 0.f;
        }
    }
    red[0][w][lane] = sx;
    red[1][w][lane] = sxy;
    __syncthreads();
    if (w != 0 || c >= J.C) return;
    J.out_x[c] = ((red[0][0][lane] + red[0][1][lane]) + red[0][2][lane]) + red[0][3][lane];
    if (hy) J.out_xy[c] = ((red[1][0][lane] + red[1][1][lane]) + red[1][2][lane]) + red[1][3][lane];
}

}  // namespace

// n <= 4 column reductions (CsJob each), both passes, two launches in all;
// nc: columns per thread (8: every operand bf16, C / strides multiples of 8,
// 16-byte aligned bases; else 4) -- the caller sizes RS for it
// (ops/reduce.py colsum_many). Returns -2 / -4 for a job the vector path
// does not take (callers then use skr_colsum2 per job).
SKR_API int skr_colsum_multi(const CsJob* jobs, int n, int nc, hipStream_t s) {
    if (n < 1 || n > kCsMax || (nc != 4 && nc != 8)) return -2;
    CsJobs g{};
    g.n = n;
    bool all_bf = true;
    for (int q = 0; q < n; ++q) all_bf = all_bf && jobs[q].xbf && (jobs[q].Y == nullptr || jobs[q].ybf);
    if (nc == 8 && !all_bf) return -2;
    for (int q = 0; q < n; ++q) {
        const CsJob& J = jobs[q];
        if (J.C <= 0 || J.C % nc || J.RS <= 0 || J.R1 * J.R2 <= 0 || J.s1 % nc || J.s2 % nc) return -2;
        if ((((uintptr_t)J.X | (uintptr_t)(J.Y ? J.Y : J.X)) & 15) ||
            (((uintptr_t)J.part_x | (uintptr_t)(J.Y ? J.part_xy : J.part_x)) & 15))
            return -4;
        g.j[q] = J;
        const int cq = J.C / nc < 256 ? J.C / nc : 256;
        if (256 % cq != 0 && cq != 256) return -2;   // narrow C: C / nc must divide 256
        g.start[q + 1] = g.start[q] + J.RS * ((J.C / nc + cq - 1) / cq);
        g.fstart[q + 1] = g.fstart[q] + (J.C + 63) / 64;
    }
    for (int q = n + 1; q <= kCsMax; ++q) g.start[q] = g.start[n], g.fstart[q] = g.fstart[n];
    if (nc == 8) hipLaunchKernelGGL((colsum_multi_kernel<1, 8>), dim3(g.start[n]), dim3(256), 0, s, g);
    else if (all_bf) hipLaunchKernelGGL((colsum_multi_kernel<1, 4>), dim3(g.start[n]), dim3(256), 0, s, g);
    else hipLaunchKernelGGL((colsum_multi_kernel<0, 4>), dim3(g.start[n]), dim3(256), 0, s, g);
    hipLaunchKernelGGL(colsum_multi_finish, dim3(g.fstart[n]), dim3(256), 0, s, g);
    return SKR_CHECK_LAUNCH();
}

SKR_API int skr_colsum_job_size() { return (int)sizeof(CsJob); }

// out[r][c] = sum_s a[s*a_slab + r*a_ld + c] + sum_s b[s*b_slab + r*b_ld + c]
// (b may be null): the gradient into a recurrence's initial state from the
// split-K dh slabs of its first step (HyperLSTM: the d[h | hh] and dR_main
// slabs), in slab order. One launch instead of a reduction per source + add.
namespace {
__global__ __launch_bounds__(256) void slab_sum2_kernel(const float* __restrict__ a, int na, int64_t a_slab, int64_t a_ld,
                                                        const float* __restrict__ b, int nb, int64_t b_slab, int64_t b_ld,
                                                        int rows, int cols, float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)rows * cols) return;
    const int r = (int)(i / cols), c = (int)(i - (int64_t)r * cols);
    float v = 0.f;
    for (int s = 0; s < na; ++s) v += a[s * a_slab + r * a_ld + c];
    for (int s = 0; s < nb; ++s) v += b[s * b_slab + r * b_ld + c];
    out[i] = v;
}
}  // namespace

SKR_API int skr_slab_sum2(const float* a, int na, int64_t a_slab, int64_t a_ld, const float* b, int nb, int64_t b_slab,
                          int64_t b_ld, int rows, int cols, float* out, hipStream_t s) {
    if (rows <= 0 || cols <= 0) return 0;
    if (a == nullptr || na < 1 || (b == nullptr && nb > 0)) return -2;
    const int64_t n = (int64_t)rows * cols;
    hipLaunchKernelGGL(slab_sum2_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a, na, a_slab, a_ld,
                       b, b ? nb : 0, b_slab, b_ld, rows, cols, out);
    return SKR_CHECK_LAUNCH();
}
