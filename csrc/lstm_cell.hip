// Fused LSTM-family cell step (forward + backward) for gfx950.
//
// Everything between one step's recurrent GEMM and the next step's GEMM is
// one launch:
//
//   g      = xp + R                              (plain / LN-LSTM)
//          = xh*ax + R*ah + bh + bias            (HyperLSTM main cell, MOD;
//                                                 a/b = vec + vec_bias per gate)
//   y      = LN_all(g)*gamma + beta              (LN: per gate block over H)
//   c'     = c*sig(y_f + fb) + sig(y_i)*tanh(y_j)*mask
//   h'     = tanh(LN(c')*gc + bc)*sig(y_o)  |  tanh(c')*sig(y_o)
//   carry  = reset[b] ? init : (h', c')          (reference eoc reset)
//
// plus the saves the backward needs (LN layers: xhat / rstd / chat only; the
// backward recomputes sig/tanh of the gates from xhat instead of re-reading a
// stored [B, 4H] activation tensor; none at inference) and a bf16 copy of the
// carried h written
// straight into the next GEMM's A operand (a column slice of a concatenated
// [h | h_hyper] buffer, hence the explicit row stride). R is the sum of the
// split-K partial slabs of csrc/skinny_gemm.hip, reduced here while loading.
// The recurrent dropout mask is regenerated from a stateless hash of
// (seed, stream, step, b*H + u) in both passes -- never stored. Rows can be
// split into parameter groups (grp_rows): the two directions of the
// bidirectional encoder run as 2B rows of one launch.
//
// Geometry: grid (C, B), NT threads (256, or 1024 for a whole wide row in one
// workgroup); workgroup c of row b owns the UPT*NT contiguous hidden units
// [c*UPT*NT, (c+1)*UPT*NT), every thread UPT units (stride NT) x 4 gates.
// The step is latency-bound (B ~ 100 rows, a few hundred KB per row), so the
// kernel is written for memory-level
// parallelism: every global load of a thread is issued up front, from
// clamped (never predicated) addresses, with the split-K slab count a
// template parameter -- no branch or runtime loop sits between a load and
// its first use, so one s_waitcnt covers them all. (A per-gate load -> use
// chain costs one full memory round trip per dependency.)
//
// C > 1 (a row split over C workgroups) only matters with LayerNorm: the C
// workgroups exchange partial (sum, sum of squares) statistics inside the
// launch as data-tagged granules -- each value travels in one 8-byte word {value,
// tag = step + 1}, written with a write-through (sc1, agent-scope) 64-bit
// store; one wave per workgroup polls the row's C*nv words with sc1 loads
// (s_sleep backoff, bounded: a timeout sets *err for the host) until every
// tag is current, then sums them. No separate flag, no
// vmcnt drain and no counter atomics: one store-to-visible hop per exchange
// (CDNA4 guide: handoff-1to1 vs handoff-flag). Every slot owns its
// workgroup's 128-byte line; the buffer is zeroed once per sequence and the
// tags make slots of the previous step stale. All B*C workgroups must be
// co-resident; the host only picks C > 1 when that holds.
//
// Reference semantics: model.py:19-23 (BasicLSTMCell), model.py:82-92 (eoc
// reset); LayerNorm-/Hyper-LSTM semantics: sketch_rnn_amd/models/cells.py.
#include <type_traits>

#include "cell_bwd_body.h"

namespace {

using namespace skr;

template <int NT, int UPT, int NS, bool LN, int MOD>
__global__ __launch_bounds__(NT) void cell_fwd(const FwdArgs a) {
    cell_fwd_body<NT, UPT, NS, LN, MOD>(a, blockIdx.x, blockIdx.y, gridDim.x);
}

template <int NT, int UPT, int NS, bool LN, int MOD, int DHS = 0>
__global__ __launch_bounds__(NT) void cell_bwd(const BwdArgs a) {
    cell_bwd_body<NT, UPT, NS, LN, MOD, DHS>(a, blockIdx.x, blockIdx.y, gridDim.x);
}

// ---- dispatch: (NT, UPT, NS, LN, MOD) ---------------------------------------------------
template <typename A>
using KernelT = void (*)(const A);

// MOD without LN: the HyperLSTM with a plain main cell (use_layer_norm=False;
// the hyper cell itself is always a LayerNorm cell)
template <int NT, int UPT, int NS>
KernelT<FwdArgs> pick(bool ln, int mod, const FwdArgs*) {
    if (mod == 3) return ln ? cell_fwd<NT, UPT, 1, true, 3> : cell_fwd<NT, UPT, 1, false, 3>;
    if (mod == 2) return ln ? cell_fwd<NT, UPT, NS, true, 2> : cell_fwd<NT, UPT, NS, false, 2>;
    if (mod) return ln ? cell_fwd<NT, UPT, NS, true, 1> : cell_fwd<NT, UPT, NS, false, 1>;
    if (ln) return cell_fwd<NT, UPT, NS, true, 0>;
    return cell_fwd<NT, UPT, NS, false, 0>;
}
// dh_out slab ceiling of a backward step for the unrolled loads: 1, 8, 32, 64,
// or 0 (runtime loops) when a source does not fit the ceilings
inline int dh_ceiling(const BwdArgs& a) {
    if ((a.dh_rec && (a.dhr_nslab < 1 || a.dhr_nslab > kRecSlabs)) ||
        (a.dh_rec2 && (a.dhr2_nslab < 1 || a.dhr2_nslab > kRecSlabs)))
        return 0;
    const int n = a.dh_out ? a.dho_nslab : 1;
    return n == 1 ? 1 : (n >= 2 && n <= 8) ? 8 : (n > 8 && n <= 32) ? 32 : (n > 32 && n <= 64) ? 64 : 0;
}

template <int NT, int UPT, int NS, int MOD>
KernelT<BwdArgs> pick_dh(int d) {
    switch (d) {
        case 1: return cell_bwd<NT, UPT, NS, true, MOD, 1>;
        case 8: return cell_bwd<NT, UPT, NS, true, MOD, 8>;
        case 32: return cell_bwd<NT, UPT, NS, true, MOD, 32>;
        case 64: return cell_bwd<NT, UPT, NS, true, MOD, 64>;
        default: return cell_bwd<NT, UPT, NS, true, MOD, 0>;
    }
}

template <int NT, int UPT, int NS>
KernelT<BwdArgs> pick(bool ln, int mod, const BwdArgs* a) {
    // hot LayerNorm shapes (HyperLSTM main / hyper cells, LN-LSTM layers):
    // dh slab loads unrolled to compile-time ceilings
    if constexpr (NT == 256 && UPT == 1 && (NS == 1 || NS == 2)) {
        if (ln && mod == 2) return pick_dh<NT, UPT, NS, 2>(dh_ceiling(*a));
        if (ln && mod == 0) return pick_dh<NT, UPT, NS, 0>(dh_ceiling(*a));
    }
    if (mod == 2) return ln ? cell_bwd<NT, UPT, NS, true, 2> : cell_bwd<NT, UPT, NS, false, 2>;
    if (mod) return ln ? cell_bwd<NT, UPT, NS, true, 1> : cell_bwd<NT, UPT, NS, false, 1>;
    if (ln) return cell_bwd<NT, UPT, NS, true, 0>;
    return cell_bwd<NT, UPT, NS, false, 0>;
}

template <int NT, int UPT, typename A>
KernelT<A> pick_ns(const A& a, bool ln, int mod) {
    // the backward reads R only with MOD
    const int ns = (std::is_same<A, FwdArgs>::value || mod) ? a.R_nslab : 1;
    switch (ns) {
        case 1: return pick<NT, UPT, 1>(ln, mod, &a);
        case 2: return pick<NT, UPT, 2>(ln, mod, &a);
        case 4: return pick<NT, UPT, 4>(ln, mod, &a);
        case 8: return pick<NT, UPT, 8>(ln, mod, &a);
        default: return pick<NT, UPT, 0>(ln, mod, &a);
    }
}

// Workgroups of kernel k (nt threads) that can be resident on the whole
// device at once: occupancy API x CU count, at most 4 per CU. Cached per
// kernel (queried on the first, eager, launch -- before any graph capture).
inline int64_t coresident_capacity(const void* k, int nt) {
    static const void* keys[64];
    static int64_t vals[64];
    static int n = 0;
    for (int i = 0; i < n; ++i)
        if (keys[i] == k) return vals[i];
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, nt, 0) != hipSuccess)
        return 0;
    const int64_t cap = (int64_t)cus * (per < 4 ? per : 4);
    if (n < 64) {
        keys[n] = k;
        vals[n] = cap;
        ++n;
    }
    return cap;
}

static int g_cell_oversub = 0;

// Geometry: C = args->cluster workgroups per row. C == 1 rows wider than 256
// units run on 1024-thread workgroups (one row per CU, no exchange);
// otherwise 256 threads with UPT units each.
template <typename A>
int launch(const A& a, bool ln, int mod, hipStream_t s) {
    if constexpr (std::is_same<A, FwdArgs>::value) {
        if (mod == 3 && (a.gpre == nullptr || a.gstats == nullptr || a.gstat_tiles < 1 || a.r_lp != nullptr)) return -3;
    }
    if constexpr (std::is_same<A, BwdArgs>::value) {
        if (mod == 3) return -3;
    }
    if constexpr (std::is_same<A, FwdArgs>::value) {
        if (a.h_q8 != nullptr && (a.H % 128 != 0 || a.h_qs == nullptr)) return -3;
    }
    if (a.B <= 0) return 0;
    const int H = a.H;
    const int C = a.cluster > 1 ? a.cluster : 1;
    if (C > kMaxCluster) return -5;
    if (C > 1 && ln && (a.part == nullptr || a.err == nullptr)) return -6;
    const int per = (H + C - 1) / C;  // units per workgroup
    const int nt = (C == 1 && per > 256) ? 1024 : 256;
    int upt = (per + nt - 1) / nt;
    upt = upt <= 1 ? 1 : upt <= 2 ? 2 : upt <= 4 ? 4 : upt <= 8 ? 8 : 0;
    if (upt == 0 || (nt == 1024 && upt > 2)) return -2;
    if ((C - 1) * upt * nt >= H) return -7;  // an empty workgroup would never arrive
    KernelT<A> k = nullptr;
    if (nt == 1024) {
        k = upt == 1 ? pick_ns<1024, 1>(a, ln, mod) : pick_ns<1024, 2>(a, ln, mod);
    } else {
        switch (upt) {
            case 1: k = pick_ns<256, 1>(a, ln, mod); break;
            case 2: k = pick_ns<256, 2>(a, ln, mod); break;
            case 4: k = pick_ns<256, 4>(a, ln, mod); break;
            default: k = pick_ns<256, 8>(a, ln, mod); break;
        }
    }
    // Rows split over C > 1 workgroups spin-wait on each other: every one of
    // the B*C workgroups must be resident at once. Checked against the
    // occupancy API (capped at 4 per CU, below the API's answer near the
    // SGPR edges where it reads one block high) -- a grid that could strand
    // a workgroup is refused instead of spinning into the timeout.
    // (g_cell_oversub: the caller accepts rows past the resident capacity --
    // a row's C workgroups are consecutive ids, so on every XCD they share one
    // in-order dispatch position: a waiting row's partners are dispatched no
    // later than the rows ahead of them finish)
    if (C > 1 && ln && !g_cell_oversub && (int64_t)a.B * C > coresident_capacity((const void*)k, nt)) return -8;
    hipLaunchKernelGGL(k, dim3(C, a.B), dim3(nt), 0, s, a);
    return SKR_CHECK_LAUNCH();
}

}  // namespace

// Host entry points: argument structs are passed by pointer from Python (ctypes
// mirrors of FwdArgs / BwdArgs in sketch_rnn_amd/ops/_hipapi.py).
// args->cluster = C workgroups per row (<= 1: one).
SKR_API int skr_lstm_fwd_step(const FwdArgs* args, int ln, int mod, hipStream_t s) {
    return launch(*args, ln != 0, mod, s);   // mod: 0 none, 1 fp32 vec, 2 bf16 vec, 3 precomputed g + stats
}

SKR_API int skr_lstm_bwd_step(const BwdArgs* args, int ln, int mod, hipStream_t s) {
    return launch(*args, ln != 0, mod, s);   // mod: 0 none, 1 fp32 vec, 2 bf16 vec
}

SKR_API int skr_lstm_fwd_args_size() { return (int)sizeof(FwdArgs); }
SKR_API int skr_lstm_bwd_args_size() { return (int)sizeof(BwdArgs); }

// Clustered rows beyond the co-resident capacity (see launch): 1 allows them
// for the next launches, 0 restores the check. Returns the previous setting.
SKR_API int skr_cell_set_oversub(int on) {
    const int prev = g_cell_oversub;
    if (on >= 0) g_cell_oversub = on != 0;
    return prev;
}
