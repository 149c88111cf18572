// HyperLSTM hyper-norm projections folded (reference: magenta sketch_rnn
// rnn.py HyperLSTMCell, hyper_norm; ours: sketch_rnn_amd/models/cells.py
// HyperLSTMParams, ops/recurrent.py _HyperSeq):
//
//   vec_j = (hh @ W_z_j + b_z_j) @ W_a_j = hh @ P_j + q_j      j < 12 (x / h / shift per gate)
//   P_j   = W_z_j W_a_j  [Hh, H],   q_j = b_z_j W_a_j  [H]
//
// Forward (once per step of training, per weight update at inference):
// hyper_fold writes P in BOTH bf16 GEMM layouts (P [Hh, 12H] for the
// backward dvec @ P^T, P^T [12H, Hh] for the forward hh @ P), q (fp32) and
// qb = q + the main bias on the shift block -- one launch instead of a
// batched library GEMM, a permute copy, a cast-transpose and the bias add.
// Backward, from dP = hh^T dvec [Hh, 12H] and sV = colsum(dvec) [12H]
// (ops/hyper.py _hyper_proj_grads, batched strided products on
// csrc/small_gemm.hip):
//   dW_a[j][e][u] = sum_k W_z[k][jE+e] dP[k][jH+u] + b_z[jE+e] sV[jH+u]
//   dW_z[k][jE+e] = sum_u dP[k][jH+u] W_a[j][e][u]
//   db_z[jE+e]    = sum_u sV[jH+u] W_a[j][e][u]
// All fp32 accumulation; E <= 32.
#include "common.h"

namespace {

constexpr int NTH = 256, KT = 16, MAXE = 32;

// grid (12H / 256, Hh / KT); H % 256 == 0: a block's columns share one j
__global__ __launch_bounds__(NTH) void hyper_fold(const float* __restrict__ Wz, const float* __restrict__ bz,
                                                  const float* __restrict__ Wa, const float* __restrict__ bias,
                                                  int Hh, int H, int E, __hip_bfloat16* __restrict__ P,
                                                  __hip_bfloat16* __restrict__ PT, float* __restrict__ q,
                                                  float* __restrict__ qb) {
    __shared__ float wz[KT][MAXE];
    const int tid = threadIdx.x, c = blockIdx.x * NTH + tid, NC = 12 * H;
    const int j = (blockIdx.x * NTH) / H, u = c - j * H, k0 = blockIdx.y * KT;
    for (int i = tid; i < KT * MAXE; i += NTH) {   // entries e >= E are zero (they meet wa[e] = 0)
        const int k = i / MAXE, e = i - k * MAXE;
        wz[k][e] = e < E ? Wz[(int64_t)(k0 + k) * 12 * E + j * E + e] : 0.f;
    }
    float wa[MAXE];
#pragma unroll
    for (int e = 0; e < MAXE; ++e) wa[e] = e < E ? Wa[((int64_t)j * E + e) * H + u] : 0.f;
    __syncthreads();
    float acc[KT];
#pragma unroll
    for (int k = 0; k < KT; ++k) {
        float s = 0.f;
#pragma unroll
        for (int e = 0; e < MAXE; ++e) s += wz[k][e] * wa[e];
        acc[k] = s;
        P[(int64_t)(k0 + k) * NC + c] = skr::to_bf16(s);
    }
    // P^T row c, columns k0 .. k0+15: 32 contiguous bytes
    uint32_t pk[KT / 2];
#pragma unroll
    for (int k = 0; k < KT / 2; ++k)
        pk[k] = (uint32_t)__bfloat16_as_ushort(skr::to_bf16(acc[2 * k])) |
                ((uint32_t)__bfloat16_as_ushort(skr::to_bf16(acc[2 * k + 1])) << 16);
    uint4* dst = (uint4*)(PT + (int64_t)c * Hh + k0);
    dst[0] = uint4{pk[0], pk[1], pk[2], pk[3]};
    dst[1] = uint4{pk[4], pk[5], pk[6], pk[7]};
    if (blockIdx.y == 0) {
        float s = 0.f;
        for (int e = 0; e < E; ++e) s += bz[j * E + e] * wa[e];
        q[c] = s;
        if (qb) qb[c] = s + ((j >= 8 && bias) ? bias[(j - 8) * H + u] : 0.f);
    }
}

}  // namespace

// W_z [Hh, 12E], b_z [12E], W_a [12, E, H] fp32; bias [4H] or null (qb shift term);
// out P [Hh, 12H] bf16, PT [12H, Hh] bf16, q [12H] fp32, qb [12H] fp32 or null
SKR_API int skr_hyper_fold(const float* Wz, const float* bz, const float* Wa, const float* bias, int Hh, int H,
                           int E, void* P, void* PT, float* q, float* qb, hipStream_t s) {
    if (H % NTH || Hh % KT || E < 1 || E > MAXE) return -2;
    if (((uintptr_t)PT & 15) || (Hh % 8)) return -4;
    hipLaunchKernelGGL(hyper_fold, dim3(12 * H / NTH, Hh / KT), dim3(NTH), 0, s, Wz, bz, Wa, bias, Hh, H, E,
                       (__hip_bfloat16*)P, (__hip_bfloat16*)PT, q, qb);
    return SKR_CHECK_LAUNCH();
}
