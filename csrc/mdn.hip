// Fused mixture-density-network loss: forward value AND gradient in one pass.
//
// z [N, 3 + 6M] = [pen(3) | pi(M) | mu1(M) | mu2(M) | s1(M) | s2(M) | rho(M)]
// (reference model.py:142-163). One row per 32-lane half-wave (M <= 32): lane
// k owns mixture component k, so the softmax over pi and the log-sum-exp over
// components are 5-step xor-shuffle reductions inside the half-wave and every
// load of a parameter block is contiguous across lanes.
//
// The density is evaluated in log space:
//   log N_k = -Z/(2(1-rho^2)) - log(2 pi) - s1 - s2 - 0.5 log(1-rho^2)
//   log S   = logsumexp_k(log pi_k + log N_k)
// mode 0 (reference, model.py:124-139):
//   shape = log S < log(clamp) ? -log(clamp) [zero grad] : -log S
//   pen   = (cont + sqrt(F) eos + F eoc) * CE(pen_logits, target)
// mode 1 (sketch-rnn VAE):
//   shape = -logaddexp(log S, log eps) * (1 - p3);  pen = CE * ((1 - p3) if mask_pen)
// Because the loss is the last op of the graph, the kernel writes dL/dz
// (for an upstream gradient of 1/N per row) together with the per-row loss
// terms; the autograd backward only rescales the two column groups.
#include "common.h"

namespace {

constexpr float kLog2Pi = 1.8378770664093453f;

__device__ __forceinline__ float hw_sum(float v) {  // half-wave (32 lanes) sum
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 32);
    return v;
}
__device__ __forceinline__ float hw_max(float v) {
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 32));
    return v;
}

__global__ __launch_bounds__(256) void mdn_loss_kernel(
    const float* __restrict__ z, int64_t ldz, const float* __restrict__ tgt, int64_t ldt, int64_t N, int M,
    int mode, float F, int mask_pen, float log_floor, float inv_n,
    float* __restrict__ row_shape, float* __restrict__ row_pen, float* __restrict__ dz) {
    const int lane = threadIdx.x & 31;
    const int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 5;
    if (row >= N) return;  // whole half-waves exit together
    const float* zr = z + row * ldz;
    const float* tr = tgt + row * ldt;
    const bool on = lane < M;
    const float x1 = tr[0], x2 = tr[1];
    const float p0 = tr[2], p1 = tr[3], p2 = tr[4];
    // ---- mixture weights: log-softmax over pi ----
    const float zpi = on ? zr[3 + lane] : -INFINITY;
    const float mpi = hw_max(zpi);
    const float epi = on ? expf(zpi - mpi) : 0.f;
    const float spi = hw_sum(epi);
    const float logpi = zpi - mpi - logf(spi);
    const float pi = epi / spi;
    // ---- bivariate normal ----
    float lp = -INFINITY, n1 = 0.f, n2 = 0.f, rho = 0.f, om = 1.f, Z = 0.f, s1 = 1.f, s2 = 1.f;
    if (on) {
        const float mu1 = zr[3 + M + lane], mu2 = zr[3 + 2 * M + lane];
        const float ls1 = zr[3 + 3 * M + lane], ls2 = zr[3 + 4 * M + lane];
        rho = tanhf(zr[3 + 5 * M + lane]);
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
    const float gam = elp / slp;  // responsibility of component k
    // ---- shape term ----
    float shape, gS;  // gS = d shape / d logS
    const float fs = 1.f - p2;
    if (mode == 0) {
        if (logS < log_floor) {
            shape = -log_floor;
            gS = 0.f;
        } else {
            shape = -logS;
            gS = -1.f;
        }
    } else {
        // -log(S + eps) = -logaddexp(logS, log eps)
        const float mx = fmaxf(logS, log_floor), mn = fminf(logS, log_floor);
        const float lae = mx + log1pf(expf(mn - mx));
        shape = -lae * fs;
        gS = -expf(logS - lae) * fs;  // -S/(S+eps)
    }
    // ---- pen term ----
    const float l0 = zr[0], l1 = zr[1], l2 = zr[2];
    const float ml = fmaxf(l0, fmaxf(l1, l2));
    const float e0 = expf(l0 - ml), e1 = expf(l1 - ml), e2 = expf(l2 - ml);
    const float se = e0 + e1 + e2, lse = ml + logf(se);
    const float ce = -(p0 * (l0 - lse) + p1 * (l1 - lse) + p2 * (l2 - lse));
    float w;
    if (mode == 0) w = p2 + sqrtf(F) * p0 + F * p1;  // ref layout: [eos, eoc, cont]
    else w = mask_pen ? fs : 1.f;
    if (lane == 0) {
        row_shape[row] = shape;
        row_pen[row] = w * ce;
    }
    if (dz == nullptr) return;
    float* dr = dz + row * ldz;
    if (lane < 3) {
        const float ps = p0 + p1 + p2;
        const float q = (lane == 0 ? e0 : lane == 1 ? e1 : e2) / se;
        const float pl = lane == 0 ? p0 : lane == 1 ? p1 : p2;
        dr[lane] = inv_n * w * (q * ps - pl);
    }
    if (on) {
        const float g = inv_n * gS * gam;
        const float inv_om = 1.f / om;
        dr[3 + lane] = inv_n * gS * (gam - pi);
        dr[3 + M + lane] = g * inv_om * (n1 - rho * n2) / s1;
        dr[3 + 2 * M + lane] = g * inv_om * (n2 - rho * n1) / s2;
        dr[3 + 3 * M + lane] = g * ((n1 * n1 - rho * n1 * n2) * inv_om - 1.f);
        dr[3 + 4 * M + lane] = g * ((n2 * n2 - rho * n1 * n2) * inv_om - 1.f);
        dr[3 + 5 * M + lane] = g * (n1 * n2 - rho * Z * inv_om + rho);
    }
}

}  // namespace

SKR_API int skr_mdn_loss(const float* z, int64_t ldz, const float* tgt, int64_t ldt, int64_t N, int M, int mode,
                         float F, int mask_pen, float log_floor, float* row_shape, float* row_pen, float* dz,
                         hipStream_t s) {
    if (M < 1 || M > 32) return -2;
    if (N == 0) return 0;
    const int rows_per_block = 256 / 32;
    const int64_t grid = (N + rows_per_block - 1) / rows_per_block;
    hipLaunchKernelGGL(mdn_loss_kernel, dim3((unsigned)grid), dim3(256), 0, s, z, ldz, tgt, ldt, N, M, mode, F,
                       mask_pen, log_floor, 1.0f / (float)N, row_shape, row_pen, dz);
    return SKR_CHECK_LAUNCH();
}
