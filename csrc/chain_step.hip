// Chained HyperLSTM backward step: the dR_hyp W_y^T product of step t + 1
// and the main LayerNorm cell backward rows of step t in ONE launch
// (ops/hyper.py).
//
//   [d[h | hh] = dR_hyp W_y^T of step t + 1   (producers: 144 tiles, 8 waves)]
//   [main cell rows of step t                 (512 threads: every operand but
//                                              the d[h] slabs -- ~90 % of the
//                                              row's ~300 KB -- is loaded
//                                              BEFORE the wait)]
//
// The main-cell backward (one 512-thread workgroup per row, csrc/row_cell.h)
// is bound by one CU's streaming rate; its dh input is the only operand the
// small W_y^T product produces. So the rows stream their saves, modulation
// vectors and LayerNorm parameters while the product computes, wait on the
// launch's arrival counter, then read the four d[h] slabs: one launch and one
// kernel boundary fewer per backward step, the row's load phase overlapped
// (profiles/r5: 21.6 -> 15.7 us per step). Reference recurrence:
// /root/reference model.py:66-95.
//
// (Measured and not adopted, round 5: the same chaining for the hyper cell
// -- forward beside R_main after R_hyp, backward beside dR_main W_h^T after
// dvec P^T. Their producers are big enough that sharing the chip with the
// independent product delayed them, and the cell, more than the saved
// boundary: forward 17.57 vs 17.59 us, backward 28.0 vs 20.1 us per step.)
//
// Synchronisation (csrc/handoff.h, chain_*): producer tiles store their
// split-K slabs write-through (sc1), drain and add 1 to the launch's
// arrival counter; a row polls the counter from one lane (bounded; a
// timeout sets *err, which the trainers raise on), joins a barrier and reads
// the slabs with sc1 loads. Producers have the lowest workgroup ids and
// never wait, and workgroups are dispatched in id order, so every producer
// is resident or finished when a row that waits on it is dispatched.
// Counters rotate (chain_rotate): no reset launch per call.
#include "row_cell.h"
#include "skinny_tile.h"

namespace {

constexpr int kNs = 3;    // LDS ring depth of the tiles (the grouped launches' setting)
constexpr int kBn = 64;   // N-tile width

template <int NW>
__device__ __forceinline__ void producer_tile(const GemmGroup& g, const ChainSync& cs, __hip_bfloat16* smem) {
    if (blockIdx.x == 0) chain_rotate(cs.counters, cs.n, cs.k);
    group_tile<kBn, kNs, NW, true>(g, blockIdx.x, smem);
    chain_arrive(cs.counters + cs.k);
}

// backward, main cell: [producers (dR_hyp W_y^T of step t + 1), 8 waves][main cell rows of step t]
// POLL: the rows' poll period (s_sleep units), skr_chain_set_poll.
// CL = 2: each row on two workgroups (1024 units each: waves 0-3 of the
// 512-thread workgroup; waves 4-7 end at once -- a barrier waits only on the
// waves still running), the two LayerNorm-backward row sums exchanged
// in-launch (row_bwd_body CL): half of the row's ~300 KB of loads per CU.
template <int POLL, int CL>
__global__ __launch_bounds__(512) void chain_bwd_main_kernel(const GemmGroup g, const int nprod, const skr::BwdArgs cell,
                                                             const ChainSync cs) {
    extern __shared__ __attribute__((aligned(16))) __hip_bfloat16 smem[];
    const int id = blockIdx.x;
    if (id < nprod) {
        producer_tile<8>(g, cs, smem);
        return;
    }
    if constexpr (CL == 1) {
        row_bwd_body<512, 4, true, 1, true, false, POLL>(cell, id - nprod, cs.counters + cs.k, (uint32_t)nprod, cs.err);
    } else {
        if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 512 / CL) return;   // (wave-uniform)
        const int r = id - nprod;
        row_bwd_body<512 / CL, 4, true, 1, true, false, POLL, CL>(cell, r / CL, cs.counters + cs.k, (uint32_t)nprod,
                                                                   cs.err, r % CL);
    }
}

static int g_row_poll = 1;

// ---- LayerNorm-LSTM chained steps (ops/recurrent.py) ----------------------------------
// forward: [h_{t-1} W_h tiles -> R slabs][cell rows of step t]; backward:
// [dG_{t+1} W_h^T tiles -> dh slabs][cell backward rows of step t]. One row
// per workgroup: NTR = H / 4 threads (waves past NTR / 64 end at once), every
// load but the slabs issued before the in-launch wait (row_fwd_body /
// row_bwd_body CHAIN); the arithmetic of the row kernels (csrc/row_cell.hip).
// probe (skr_chain_ln_set_probe; outputs WRONG while set): 1 the rows end at
// once (producers only), 2 the producers only arrive (rows only, no GEMM).
template <int NTR, int DS>
__global__ __launch_bounds__(512) void chain_ln_fwd_kernel(const GemmGroup g, const int nprod, const skr::FwdArgs cell,
                                                           const ChainSync cs, const int probe) {
    extern __shared__ __attribute__((aligned(16))) __hip_bfloat16 smem[];
    const int id = blockIdx.x;
    if (id < nprod) {
        if (probe == 2) {
            if (blockIdx.x == 0) chain_rotate(cs.counters, cs.n, cs.k);
            chain_arrive(cs.counters + cs.k);
            return;
        }
        producer_tile<8>(g, cs, smem);
        return;
    }
    if (probe == 1 || __builtin_amdgcn_readfirstlane(threadIdx.x) >= NTR) return;   // (wave-uniform)
    row_fwd_body<NTR, 4, 0, DS, true>(cell, id - nprod, cs.counters + cs.k, (uint32_t)nprod, cs.err);
}

template <int NTR>
__global__ __launch_bounds__(512) void chain_ln_bwd_kernel(const GemmGroup g, const int nprod, const skr::BwdArgs cell,
                                                           const ChainSync cs, const int probe) {
    extern __shared__ __attribute__((aligned(16))) __hip_bfloat16 smem[];
    const int id = blockIdx.x;
    if (id < nprod) {
        if (probe == 2) {
            if (blockIdx.x == 0) chain_rotate(cs.counters, cs.n, cs.k);
            chain_arrive(cs.counters + cs.k);
            return;
        }
        producer_tile<8>(g, cs, smem);
        return;
    }
    if (probe == 1 || __builtin_amdgcn_readfirstlane(threadIdx.x) >= NTR) return;
    row_bwd_body<NTR, 4, false, 1, true>(cell, id - nprod, cs.counters + cs.k, (uint32_t)nprod, cs.err);
}

// ---- three-stage launch: + the dvec P^T product of step t ------------------------------
// [producers: dR_hyp W_y^T of step t + 1] -> [main-cell rows of step t] ->
// [dvec P^T tiles of step t]. The first nprod2 producer workgroups switch
// role once their producer tile has arrived: they DMA their whole P^T weight
// slice (BN x kslice bf16, <= 96 KB) into the LDS the producer ring used --
// while the rows compute -- then wait on the rows' counter and run the tile
// from LDS with the A operand (the dvec rows) read through sc1 loads. Same
// fragments, k order and MFMA as glds_mma: the slabs are bit-identical to the
// separate launch (skinny_gemm_glds_kernel). Residency: producers never wait
// before their arrival; rows wait only on producers; tiles wait only on rows,
// and a row that cannot be placed gets the CU of a row that finished.
template <int BN, int NW>
__device__ __forceinline__ void resident_issue(const GemmProblem& p, const TileIdx& t, __hip_bfloat16* smem) {
    constexpr int B_CH = BN / 8;                    // 1-KiB chunks (8 rows x 64 k) per stage
    static_assert(B_CH % NW == 0, "resident tile: wave layout");
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int kslice = p.K / p.splits, nst = kslice / skr::BK;
    const int64_t k0 = (int64_t)t.split * kslice;
    const int r8 = lane >> 3, slot = lane & 7;
    const __hip_bfloat16* Bt = (const __hip_bfloat16*)p.Bt;
    for (int st = 0; st < nst; ++st) {
#pragma unroll
        for (int i = 0; i < B_CH / NW; ++i) {
            const int row = (w + NW * i) * 8 + r8;
            const int kc = slot ^ ((row >> 1) & 7);
            __builtin_amdgcn_global_load_lds((const void*)(Bt + (int64_t)(t.nt * BN + row) * p.ldb + k0 + st * skr::BK + kc * 8),
                                             (__attribute__((address_space(3))) void*)(smem + st * BN * skr::BK + (w + NW * i) * 512),
                                             16, 0, 0);
        }
    }
}

template <int BN, int NW>
__device__ __forceinline__ void resident_finish(const GemmProblem& p, const TileIdx& t, const __hip_bfloat16* smem) {
    constexpr int NJ = skr::glds_nj<BN, NW>();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wr = w % 4, wc = w / 4;
    const int fr = lane & 15, fq = lane >> 4;
    const int kslice = p.K / p.splits, nk = kslice / 32;
    const int64_t k0 = (int64_t)t.split * kslice;
    const int M = t.rows;
    const __hip_bfloat16* A = (const __hip_bfloat16*)p.A + (int64_t)t.rb * skr::BM * p.lda;
    const __amdgpu_buffer_rsrc_t ra = rsrc(A, (int64_t)M * p.lda * 2);
    bool live[2];
    uint32_t aoff[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int row = 32 * wr + 16 * i + fr;
        live[i] = 32 * wr + 16 * i < M;                      // uniform per wave
        aoff[i] = (uint32_t)(((int64_t)min(row, M - 1) * p.lda + k0 + 8 * fq) * 2);
    }
    tile_f32x4 acc[2][NJ];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = tile_f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int G = 4;                                     // k32 steps of A in flight per batch
    // two register sets with compile-time indices only (a runtime-indexed
    // double buffer is placed in scratch memory)
    skr::bf16x8 cur[G][2], nxt[G][2];
    auto load = [&](skr::bf16x8 (&dst)[G][2], int kk0) {
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int i = 0; i < 2; ++i)
                if (live[i] && kk0 + g < nk) dst[g][i] = ld_sc1(ra, aoff[i] + (uint32_t)(kk0 + g) * 64);
    };
    load(cur, 0);
    for (int kb = 0; kb < nk; kb += G) {
        if (kb + G < nk) load(nxt, kb + G);
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int kk = kb + g;
            if (kk >= nk) break;
            const __hip_bfloat16* Bs = smem + (kk >> 1) * BN * skr::BK;
            const int kc = (kk & 1) * 4 + fq;
            skr::bf16x8_t bfr[NJ];
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int row = 16 * (wc * NJ + j) + fr;
                bfr[j] = *(const skr::bf16x8_t*)(&Bs[row * skr::BK + ((kc ^ ((row >> 1) & 7)) * 8)]);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                if (!live[i]) continue;
                const skr::bf16x8_t a = __builtin_bit_cast(skr::bf16x8_t, cur[g][i]);
#pragma unroll
                for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bfr[j], acc[i][j], 0, 0, 0);
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int i = 0; i < 2; ++i) cur[g][i] = nxt[g][i];
    }
    float* C = p.C + split_off(p, t);
    const int c0 = t.nt * BN + wc * NJ * 16;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = 32 * wr + 16 * i + fq * 4 + e;
                if (row < M) C[row * p.ldc + c0 + 16 * j + fr] = acc[i][j][e];
            }
}

struct Chain3 {
    GemmProblem tail;      // dvec P^T: A = dvec rows (written by this launch's rows), Bt = P^T weights
    int ntail;             // its tile count (<= producer count)
    ChainSync rows;        // the rows' arrival counters
    int probe;             // timing probes (skr_chain3_set_probe; results invalid)
};

static int g_chain3_probe = 0;

__global__ __launch_bounds__(512) void chain_bwd_main3_kernel(const GemmGroup g, const int nprod, const skr::BwdArgs cell,
                                                              const ChainSync cs, const Chain3 c3) {
    extern __shared__ __attribute__((aligned(16))) __hip_bfloat16 smem[];
    const int id = blockIdx.x;
    if (id < nprod) {
        if (id == 0) chain_rotate(c3.rows.counters, c3.rows.n, c3.rows.k);
        producer_tile<8>(g, cs, smem);      // ends with the arrival (vmcnt(0) + barrier): the ring is free
        if (id >= c3.ntail || c3.probe == 1) return;
        // tiles of one split (the same dvec K slice, read with sc1 loads) on one
        // XCD: workgroup id -> (xcd = id % 8, j = id / 8), N tile j % NTL, split
        // (j / NTL) * 8 + xcd -- the later readers of a slice hit that XCD's L2
        const int ntl = c3.tail.N / kBn, x = id & 7, j = id >> 3;
        const int local = (((j / ntl) * 8 + x) * ntl) + j % ntl;
        if (local >= c3.ntail) return;
        const TileIdx t = tile_idx(local, c3.tail.M, c3.tail.N, c3.tail.splits, kBn);
        if (c3.probe != 3) resident_issue<kBn, 8>(c3.tail, t, smem);
        chain_wait<16>(c3.rows.counters + c3.rows.k, (uint32_t)cell.B, cs.err);   // (a ~10 us wait: poll sparsely)
        if (c3.probe == 3) return;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's weight DMAs landed ...
        __syncthreads();                                   // ... and every other wave's
        if (c3.probe == 2) return;
        resident_finish<kBn, 8>(c3.tail, t, smem);
        return;
    }
    row_bwd_body<512, 4, true, 1, true, true>(cell, id - nprod, cs.counters + cs.k, (uint32_t)nprod, cs.err);
    chain_arrive(c3.rows.counters + c3.rows.k);
}

template <typename K>
void lds_attr(K k, size_t lds) {
    static bool done = false;   // per instantiation, once (never during a graph capture's second call)
    if (!done) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        done = true;
    }
}

constexpr size_t kLds = (size_t)kNs * (skr::BM + kBn) * skr::BK * 2;

// Group of n problems, the first nprod of which are producers; returns the
// producer tile count (> 0) or a negative code.
int build_group(const GemmProblem* probs, int n, int nprod, GemmGroup& g) {
    if (n < 1 || n > kMaxGroup || nprod < 1 || nprod > n) return -2;
    g = GemmGroup{};
    g.n = n;
    g.start[0] = 0;
    for (int i = 0; i < n; ++i) {
        const int rc = check_problem64(probs[i]);
        if (rc) return rc;
        g.p[i] = probs[i];
        g.start[i + 1] = g.start[i] + (probs[i].N / kBn) * probs[i].splits * row_blocks_of(probs[i].M);
    }
    for (int i = n + 1; i <= kMaxGroup; ++i) g.start[i] = g.start[n];
    return g.start[nprod];
}

int check_sync(const ChainSync* cs) {
    if (cs == nullptr || cs->counters == nullptr || cs->err == nullptr || cs->n < 2 || cs->k < 0 || cs->k >= cs->n)
        return -6;
    return 0;
}

}  // namespace

// Backward main-cell chain: probs[0 .. n) (all producers) produce the row's
// dh_rec slabs (<= 8); everything else as skr_row_bwd_step mod 2 with
// H = 2048 (512 threads x 4 units) and a single dh_out slab; cell->cluster
// == 2 splits every row over two workgroups (exchange buffer cell->part).
SKR_API int skr_chain_bwd_main(const GemmProblem* probs, int n, const skr::BwdArgs* cell, const ChainSync* cs,
                               hipStream_t s) {
    if (cell == nullptr || check_sync(cs)) return -6;
    const skr::BwdArgs& a = *cell;
    if (a.H != 2048 || a.dh_rec == nullptr || a.dhr_nslab < 1 || a.dhr_nslab > 8) return -2;
    if (a.dh_out && a.dho_nslab != 1) return -2;
    const int rc = row_bwd_check(a, 2);
    if (rc) return rc;
    GemmGroup g;
    const int np = build_group(probs, n, n, g);
    if (np < 0) return np;
    // cell.cluster == 2: two workgroups per row (a.part / a.err: the exchange buffer, [2][B][2][16])
    const int cl = a.cluster == 2 ? 2 : 1;
    if (cl == 2 && (a.part == nullptr || a.err == nullptr)) return -6;
#define SKR_CBM(P_, CL_)                                                                              \
    do {                                                                                              \
        lds_attr(chain_bwd_main_kernel<P_, CL_>, kLds);                                               \
        hipLaunchKernelGGL((chain_bwd_main_kernel<P_, CL_>), dim3(np + a.B * CL_), dim3(512), kLds, s, g, np, a, *cs); \
    } while (0)
    if (cl == 2) SKR_CBM(1, 2);
    else if (g_row_poll >= 16) SKR_CBM(16, 1);
    else if (g_row_poll >= 4) SKR_CBM(4, 1);
    else SKR_CBM(1, 1);
#undef SKR_CBM
    return SKR_CHECK_LAUNCH();
}

// Three-stage backward launch: as skr_chain_bwd_main, plus the dvec P^T
// product `tail` (A = cell.dvec rows, M = cell.B; Bt = P^T) run by the first
// tail-tile-count producer workgroups after their producer tile, on the rows'
// counters `rows`. Returns -2 (shape not taken: callers keep the separate
// launch) when the tail has more tiles than there are producers, a K slice
// that is not a whole number of 64-wide steps, or a weight slice over 96 KB.
SKR_API int skr_chain_bwd_main3(const GemmProblem* probs, int n, const GemmProblem* tail, const skr::BwdArgs* cell,
                                const ChainSync* cs, const ChainSync* rows, hipStream_t s) {
    if (cell == nullptr || tail == nullptr || check_sync(cs) || check_sync(rows)) return -6;
    const skr::BwdArgs& a = *cell;
    if (a.H != 2048 || a.dh_rec == nullptr || a.dhr_nslab < 1 || a.dhr_nslab > 8) return -2;
    if (a.dh_out && a.dho_nslab != 1) return -2;
    int rc = row_bwd_check(a, 2);
    if (rc) return rc;
    rc = check_problem64(*tail);
    if (rc) return rc;
    if (tail->M != a.B || tail->M > skr::BM || tail->A != a.dvec) return -2;
    const int kslice = tail->K / tail->splits;
    const size_t slice_lds = (size_t)kBn * kslice * 2;
    if (slice_lds > 96 * 1024) return -2;
    GemmGroup g;
    const int np = build_group(probs, n, n, g);
    if (np < 0) return np;
    Chain3 c3;
    c3.tail = *tail;
    c3.ntail = (tail->N / kBn) * tail->splits;
    c3.rows = *rows;
    c3.probe = g_chain3_probe;
    if (c3.ntail > np || c3.ntail % (8 * (tail->N / kBn))) return -2;   // (the XCD-grouped tile map is a bijection)
    const size_t lds = slice_lds > kLds ? slice_lds : kLds;
    lds_attr(chain_bwd_main3_kernel, 96 * 1024);
    hipLaunchKernelGGL(chain_bwd_main3_kernel, dim3(np + a.B), dim3(512), lds, s, g, np, a, *cs, c3);
    return SKR_CHECK_LAUNCH();
}

// Timing probes of the three-stage launch (scripts/micro/chain3_probe.py; the
// gradients are WRONG while a probe is set): 0 off, 1 producers exit after
// their tile (no dvec P^T), 2 the tail stages its weights and waits on the
// rows but computes nothing, 3 the tail only waits (no weight staging).
SKR_API int skr_chain3_set_probe(int p) {
    const int prev = g_chain3_probe;
    g_chain3_probe = p;
    return prev;
}

// A/B hook: poll period of the chained main-cell rows (1, 4 or 16 s_sleep
// units); returns the previous one.
SKR_API int skr_chain_set_poll(int p) {
    const int prev = g_row_poll;
    if (p > 0) g_row_poll = p;
    return prev;
}

SKR_API int skr_chain_sync_size() { return (int)sizeof(ChainSync); }

static int g_chain_ln_probe = 0;

// ---- skewed LayerNorm-LSTM forward step ---------------------------------------------------
// Launch t: [cell rows of step t][h_t W_h tiles of step t + 1]. The rows'
// R slabs were written by the previous launch, so they load everything at
// once (no wait); they store their bf16 h_t row write-through and arrive.
// The tiles of step t + 1 stage their whole 64-column weight slice in LDS
// (the latency that does not depend on h_t) while the rows compute, wait
// for all B rows, then load their h_t fragments with sc1 loads and run the
// K-steps from LDS (v_mfma_f32_16x16x32_bf16, ascending k, as the grouped
// tiles). Rows have the lowest ids and never wait. Tile: 128 rows (8 waves x
// one 16-row tile) x 64 columns x kslice = 32 KS; LDS row r of the slice
// keeps its 16-byte chunk c at c ^ (r & 15) (conflict-free fragment reads).
template <int KS>
__device__ __forceinline__ void skew_tile(const __hip_bfloat16* __restrict__ WT, int H, const __hip_bfloat16* __restrict__ A,
                                          int64_t lda, int B, float* __restrict__ Rn, int64_t r_slab, int64_t ld_r, int p,
                                          const uint32_t* cnt, uint32_t target, int* err, __hip_bfloat16* lds) {
    constexpr int KSL = 32 * KS, CPR = KSL / 8;          // slice width, 16-byte chunks per LDS row
    const int G = 4 * H, ntile = G / kBn;
    const int n0 = (p % ntile) * kBn, k0 = (p / ntile) * KSL, sl = p / ntile;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, fq = lane >> 4;
    for (int i = tid; i < kBn * CPR; i += 512) {          // the weight slice: independent of h_t
        const int r = i / CPR, c = i - r * CPR;
        const bf16x8 v = *(const bf16x8*)(WT + (int64_t)(n0 + r) * H + k0 + 8 * c);
        *(bf16x8*)(lds + r * KSL + ((c ^ (r & 15)) * 8)) = v;
    }
    chain_wait(cnt, target, err);                          // (its barrier also publishes the LDS slice)
    const int row = 16 * w + fr;
    const __amdgpu_buffer_rsrc_t ar = rsrc(A, (int64_t)B * lda * 2);
    bf16x8 af[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) af[ks] = ld_sc1(ar, (uint32_t)(((int64_t)min(row, B - 1) * lda + k0 + 32 * ks + 8 * fq) * 2));
    f32x4 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r = 16 * j + fr;
            const bf16x8 b = *(const bf16x8*)(lds + r * KSL + (((4 * ks + fq) ^ (r & 15)) * 8));
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks], b, acc[j], 0, 0, 0);
        }
    if (16 * w >= B) return;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int rr = 16 * w + 4 * fq + i;
            if (rr < B) Rn[(int64_t)sl * r_slab + (int64_t)rr * ld_r + n0 + 16 * j + fr] = acc[j][i];
        }
}

template <int NTR, int DS, int KS>
__global__ __launch_bounds__(512) void skew_ln_fwd_kernel(const skr::FwdArgs cell, const __hip_bfloat16* __restrict__ WT,
                                                          float* __restrict__ Rn, const ChainSync cs) {
    extern __shared__ __attribute__((aligned(16))) __hip_bfloat16 smem[];
    const int id = blockIdx.x, B = cell.B;
    if (id == 0) chain_rotate(cs.counters, cs.n, cs.k);
    if (id < B) {
        if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= NTR) return;   // (wave-uniform)
        row_fwd_body<NTR, 4, 0, DS, false, true>(cell, id);
        chain_arrive(cs.counters + cs.k);
        return;
    }
    skew_tile<KS>(WT, cell.H, (const __hip_bfloat16*)cell.h_lp, cell.ld_lp, B, Rn, cell.R_slab, cell.ld_R, id - B,
                  cs.counters + cs.k, (uint32_t)B, cs.err, smem);
}

// Skewed LayerNorm-LSTM forward step t: the cell rows of step t (cell: R =
// the slabs of step t, written by an earlier launch; lp_kind 1) and, when
// Rn != null, the tiles of step t + 1 writing its S = R_nslab slabs into Rn
// (same slab stride and row stride as cell.R) from WT [4H][H] bf16 and the
// rows' h_t. H in {256, 512, 1024}, B <= 128, H / S in {128, 256, 512}.
// Returns -2 / -3 / -4 when not taken.
SKR_API int skr_skew_ln_fwd(const skr::FwdArgs* cell, const void* WT, float* Rn, const ChainSync* cs, hipStream_t s) {
    if (cell == nullptr || check_sync(cs)) return -6;
    const skr::FwdArgs& a = *cell;
    if (a.B <= 0) return 0;
    const int H = a.H, S = a.R_nslab;
    if ((H != 256 && H != 512 && H != 1024) || a.B > 128 || a.lp_kind != 1 || a.grp_rows > 0 || S < 1 || S > 4 ||
        H % S != 0)
        return -2;
    const int rc = row_fwd_check(a, 0);
    if (rc) return rc;
    const int kslice = H / S;
    if (kslice != 128 && kslice != 256 && kslice != 512) return -2;
    if ((((uintptr_t)WT | (uintptr_t)Rn | (uintptr_t)a.h_lp) & 15) || a.ld_lp % 8) return -4;
    const int ntr = H / 4, ds = S <= 1 ? 1 : S <= 2 ? 2 : 4, ks = kslice / 32;
    const int nprod = Rn ? (4 * H / kBn) * S : 0;
    const size_t lds = (size_t)kBn * kslice * 2;
    const void* k = nullptr;
#define SKR_SK(NTR_, DS_, KS_) if (ntr == NTR_ && ds == DS_ && ks == KS_) k = (const void*)skew_ln_fwd_kernel<NTR_, DS_, KS_>;
#define SKR_SK_KS(NTR_, DS_) SKR_SK(NTR_, DS_, 4) SKR_SK(NTR_, DS_, 8) SKR_SK(NTR_, DS_, 16)
#define SKR_SK_DS(NTR_) SKR_SK_KS(NTR_, 1) SKR_SK_KS(NTR_, 2) SKR_SK_KS(NTR_, 4)
    SKR_SK_DS(64) SKR_SK_DS(128) SKR_SK_DS(256)
#undef SKR_SK_DS
#undef SKR_SK_KS
#undef SKR_SK
    if (k == nullptr) return -2;
    if (lds > 48 * 1024) (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    const __hip_bfloat16* wt = (const __hip_bfloat16*)WT;
    float* rn = Rn;
    void* args[] = {(void*)&a, (void*)&wt, (void*)&rn, (void*)cs};
    if (hipLaunchKernel(k, dim3(a.B + nprod), dim3(512), args, lds, s) != hipSuccess) return -1;
    return SKR_CHECK_LAUNCH();
}

// Timing probes of the chained LayerNorm-LSTM steps (scripts/micro/ln_probe.py;
// outputs WRONG while set): 1 producers only, 2 rows only. Returns the previous.
SKR_API int skr_chain_ln_set_probe(int p) {
    const int prev = g_chain_ln_probe;
    if (p >= 0) g_chain_ln_probe = p;
    return prev;
}

// LayerNorm-LSTM forward step chained: probs (all producers) write the R
// slabs (cell->R, <= 8) the rows of this step sum; rows as skr_row_fwd_step
// mod 0 with H in {256, 512, 1024, 2048}. Returns -2 / -3 / -4 when not taken.
SKR_API int skr_chain_ln_fwd(const GemmProblem* probs, int n, const skr::FwdArgs* cell, const ChainSync* cs,
                             hipStream_t s) {
    if (cell == nullptr || check_sync(cs)) return -6;
    const skr::FwdArgs& a = *cell;
    if (a.B <= 0) return 0;
    if (a.H % 256 != 0 || a.H > 2048 || a.R_nslab < 1 || a.R_nslab > 8 || a.grp_rows > 0) return -2;
    const int rc = row_fwd_check(a, 0);
    if (rc) return rc;
    GemmGroup g;
    const int np = build_group(probs, n, n, g);
    if (np < 0) return np;
    const int ntr = a.H / 4, ds = a.R_nslab <= 1 ? 1 : a.R_nslab <= 2 ? 2 : a.R_nslab <= 4 ? 4 : 8;
    const void* k = nullptr;
#define SKR_CLF(NTR_, DS_) if (ntr == NTR_ && ds == DS_) k = (const void*)chain_ln_fwd_kernel<NTR_, DS_>;
#define SKR_CLF_DS(NTR_) SKR_CLF(NTR_, 1) SKR_CLF(NTR_, 2) SKR_CLF(NTR_, 4) SKR_CLF(NTR_, 8)
    SKR_CLF_DS(64) SKR_CLF_DS(128) SKR_CLF_DS(256) SKR_CLF_DS(512)
#undef SKR_CLF_DS
#undef SKR_CLF
    if (k == nullptr) return -2;
    static const void* attr_done[16];
    static int n_attr = 0;
    bool done = false;
    for (int i = 0; i < n_attr; ++i) done |= attr_done[i] == k;
    if (!done && n_attr < 16) {
        (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLds);
        attr_done[n_attr++] = k;
    }
    int npv = np, prb = g_chain_ln_probe;
    void* args[] = {(void*)&g, (void*)&npv, (void*)&a, (void*)cs, (void*)&prb};
    if (hipLaunchKernel(k, dim3(np + a.B), dim3(512), args, kLds, s) != hipSuccess) return -1;
    return SKR_CHECK_LAUNCH();
}

// LayerNorm-LSTM backward step chained: probs (all producers) write the dh_rec
// slabs (cell->dh_rec, <= 8) of this step's rows; rows as skr_row_bwd_step
// mod 0 with a single dh_out slab (or none).
SKR_API int skr_chain_ln_bwd(const GemmProblem* probs, int n, const skr::BwdArgs* cell, const ChainSync* cs,
                             hipStream_t s) {
    if (cell == nullptr || check_sync(cs)) return -6;
    const skr::BwdArgs& a = *cell;
    if (a.B <= 0) return 0;
    if (a.H % 256 != 0 || a.H > 2048 || a.dh_rec == nullptr || a.dhr_nslab < 1 || a.dhr_nslab > 8 ||
        a.dh_rec2 != nullptr || a.grp_rows > 0)
        return -2;
    if (a.dh_out && a.dho_nslab != 1) return -2;
    const int rc = row_bwd_check(a, 0);
    if (rc) return rc;
    GemmGroup g;
    const int np = build_group(probs, n, n, g);
    if (np < 0) return np;
    const int ntr = a.H / 4;
    const void* k = ntr == 64 ? (const void*)chain_ln_bwd_kernel<64> : ntr == 128 ? (const void*)chain_ln_bwd_kernel<128>
                  : ntr == 256 ? (const void*)chain_ln_bwd_kernel<256> : (const void*)chain_ln_bwd_kernel<512>;
    static const void* attr_done[4];
    static int n_attr = 0;
    bool done = false;
    for (int i = 0; i < n_attr; ++i) done |= attr_done[i] == k;
    if (!done && n_attr < 4) {
        (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLds);
        attr_done[n_attr++] = k;
    }
    int npv = np, prb = g_chain_ln_probe;
    void* args[] = {(void*)&g, (void*)&npv, (void*)&a, (void*)cs, (void*)&prb};
    if (hipLaunchKernel(k, dim3(np + a.B), dim3(512), args, kLds, s) != hipSuccess) return -1;
    return SKR_CHECK_LAUNCH();
}
