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
__global__ __launch_bounds__(512) void chain_bwd_main_kernel(const GemmGroup g, const int nprod, const skr::BwdArgs cell,
                                                             const ChainSync cs) {
    extern __shared__ __attribute__((aligned(16))) __hip_bfloat16 smem[];
    const int id = blockIdx.x;
    if (id < nprod) {
        producer_tile<8>(g, cs, smem);
        return;
    }
    row_bwd_body<512, 4, true, 1, true>(cell, id - nprod, cs.counters + cs.k, (uint32_t)nprod, cs.err);
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
// H = 2048 (512 threads x 4 units) and a single dh_out slab.
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
    lds_attr(chain_bwd_main_kernel, kLds);
    hipLaunchKernelGGL(chain_bwd_main_kernel, dim3(np + a.B), dim3(512), kLds, s, g, np, a, *cs);
    return SKR_CHECK_LAUNCH();
}

SKR_API int skr_chain_sync_size() { return (int)sizeof(ChainSync); }
