// HyperLSTM hyper-norm modulation vectors, unfolded, one launch per step:
//
//   zs   = hh @ W_z                       [B, 12E]   (E = 32: 12 embeddings)
//   vec  = zs_k @ W_a[k]  for k = 0..11   [B, 12, H] (bf16 out)
//
// (the embedding bias b_z enters as vec_bias = b_z @ W_a, added by the cell
// kernel, exactly as with the folded form vec = hh @ P, P = [W_z_k W_a_k]_k.)
// The folded product streams P (Hh x 12H = 12.6 MB bf16 at the vae_large
// shape) every step; unfolded, the per-step weights are W_z (196 KB) and
// W_a (1.5 MB). Workgroup (k, column tile of 64 units) recomputes its own
// zs_k = hh @ W_z[:, 32k : 32k+32] (a [B x 32] tile, K = Hh -- 2% of the
// step's MFMAs, read from L2), passes it through LDS into A-fragment layout
// and multiplies by W_a[k][:, tile] (K = 32: one MFMA per 16x16 output tile).
// v_mfma_f32_16x16x32_bf16 throughout; fp32 accumulation.
#include "common.h"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
constexpr int E = 32, NT = 64;   // embedding width, units per workgroup

// grid (12, H / 64), 512 threads: wave w owns row tile w (B <= 128). The
// W_z / W_a slices are staged once into LDS; each wave issues its A loads
// first, so their latency overlaps the staging; the [16 x 64] bf16 output
// tile goes out through LDS as 16-byte row stores.
template <int HH>
__global__ __launch_bounds__(512) void hyper_vec_fwd(const __hip_bfloat16* __restrict__ hh, int64_t ld_hh,
                                                     const __hip_bfloat16* __restrict__ WzT,   // [12E][HH]
                                                     const __hip_bfloat16* __restrict__ WaT,   // [12][H][E]
                                                     __hip_bfloat16* __restrict__ vec, int64_t vec_gs,
                                                     int64_t vec_ld, int B, int H) {
    constexpr int CZ = HH / 8;                                   // 16-byte chunks per W_z row
    constexpr int SWZ = (CZ < 16 ? CZ : 16) - 1;                 // chunk XOR mask (stays inside the row)
    __shared__ __attribute__((aligned(16))) __hip_bfloat16 wz[E * HH];    // [32][HH], chunks XOR-swizzled
    __shared__ __attribute__((aligned(16))) __hip_bfloat16 wa[NT * E];    // [64][32]
    __shared__ __attribute__((aligned(16))) __hip_bfloat16 tl[8][16 * NT]; // per-wave tile (zs, then vec)
    const int k = blockIdx.x, u0 = blockIdx.y * NT;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const bool on = w * 16 < B;
    // ---- this wave's A fragments (hh rows), issued before the staging
    bf16x8 af[HH / 32];
    const int row = min(w * 16 + fr, B - 1);
    if (on) {
        const __hip_bfloat16* ap = hh + (int64_t)row * ld_hh + fq * 8;
#pragma unroll
        for (int ks = 0; ks < HH / 32; ++ks) af[ks] = *(const bf16x8*)(ap + ks * 32);
    }
    // ---- stage W_z[:, 32k .. 32k+32]^T and W_a[k][:, u0 .. u0+64]^T
    const __hip_bfloat16* wzg = WzT + (int64_t)(k * E) * HH;
    for (int i = tid; i < E * CZ; i += 512) {
        const int r = i / CZ, c = i - r * CZ;
        *(bf16x8*)(wz + r * HH + ((c ^ (r & SWZ)) * 8)) = *(const bf16x8*)(wzg + (int64_t)r * HH + c * 8);
    }
    if (tid < NT * E / 8) {
        const int r = tid / (E / 8), c = tid % (E / 8);
        *(bf16x8*)(wa + r * E + c * 8) = *(const bf16x8*)(WaT + ((int64_t)k * H + u0 + r) * E + c * 8);
    }
    __syncthreads();
    if (!on) return;
    // ---- zs tile [16 x 32] = hh @ W_z-slice
    f32x4 az[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int ks = 0; ks < HH / 32; ++ks)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int r = j * 16 + fr, c = ks * 4 + fq;
            const bf16x8 b = *(const bf16x8*)(wz + r * HH + ((c ^ (r & SWZ)) * 8));
            az[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks], b, az[j], 0, 0, 0);
        }
    __hip_bfloat16* t = tl[w];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) t[(4 * fq + i) * E + j * 16 + fr] = skr::to_bf16(az[j][i]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const bf16x8 za = *(const bf16x8*)(t + fr * E + fq * 8);
    // ---- vec tile [16 x 64] = zs @ W_a[k][:, tile]
    f32x4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
        v[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(za, *(const bf16x8*)(wa + (j * 16 + fr) * E + fq * 8),
                                                        f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // zs fragment read before the tile is overwritten
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) t[(4 * fq + i) * NT + j * 16 + fr] = skr::to_bf16(v[j][i]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const int s = lane + 64 * p, r = s >> 3, c = s & 7;   // 16 rows x 8 16-byte pieces
        const int gr = w * 16 + r;
        if (gr < B)
            *(bf16x8*)(vec + (int64_t)k * vec_gs + (int64_t)gr * vec_ld + u0 + c * 8) = *(const bf16x8*)(t + r * NT + c * 8);
    }
}

}  // namespace

// hh: [B, Hh] bf16 rows (stride ld_hh); WzT [12*32, Hh]; WaT [12, H, 32]; vec bf16
// element (k, b, u) at k*vec_gs + b*vec_ld + u.
SKR_API int skr_hyper_vec_fwd(const void* hh, int64_t ld_hh, const void* WzT, const void* WaT, void* vec,
                              int64_t vec_gs, int64_t vec_ld, int B, int H, int Hh, hipStream_t s) {
    if (B <= 0) return 0;
    if (B > 128) return -2;
    if (H % NT || (vec_ld % 8) || (vec_gs % 8) || (ld_hh % 8) || (((uintptr_t)hh | (uintptr_t)WzT | (uintptr_t)WaT | (uintptr_t)vec) & 15)) return -3;
    const dim3 grid(12, H / NT);
    const auto* a = (const __hip_bfloat16*)hh;
    const auto* z = (const __hip_bfloat16*)WzT;
    const auto* w = (const __hip_bfloat16*)WaT;
    auto* v = (__hip_bfloat16*)vec;
    switch (Hh) {
        case 64: hipLaunchKernelGGL(hyper_vec_fwd<64>, grid, dim3(512), 0, s, a, ld_hh, z, w, v, vec_gs, vec_ld, B, H); break;
        case 128: hipLaunchKernelGGL(hyper_vec_fwd<128>, grid, dim3(512), 0, s, a, ld_hh, z, w, v, vec_gs, vec_ld, B, H); break;
        case 256: hipLaunchKernelGGL(hyper_vec_fwd<256>, grid, dim3(512), 0, s, a, ld_hh, z, w, v, vec_gs, vec_ld, B, H); break;
        case 512: hipLaunchKernelGGL(hyper_vec_fwd<512>, grid, dim3(512), 0, s, a, ld_hh, z, w, v, vec_gs, vec_ld, B, H); break;
        default: return -2;
    }
    return SKR_CHECK_LAUNCH();
}
