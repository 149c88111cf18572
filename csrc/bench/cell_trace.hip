// Diagnostic: in-kernel timeline of the HyperLSTM main-cell forward step
// (csrc/cell_fwd_body.h with SKR_TRACE_CELL stamps) at the vae_large shape.
// Build: hipcc -O3 --offload-arch=gfx950 -I csrc csrc/bench/cell_trace.hip -o build/cell_trace
// Prints, over the workgroups of the last of N graph-replayed launches, the
// spread of: dispatch (entry - first entry), loads landed, exchange 1,
// exchange 2 (+ cell), stores drained -- in microseconds (100 MHz stamps).
#define SKR_TRACE_CELL 1
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../lstm_cell.hip"

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

static float* dalloc(size_t n, float v = 0.01f) {
    float* p;
    CK(hipMalloc(&p, n * sizeof(float)));
    std::vector<float> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = v * (float)((i * 2654435761u) % 1000) / 1000.f;
    CK(hipMemcpy(p, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
    return p;
}

static void pct(const char* name, std::vector<double> v) {
    std::sort(v.begin(), v.end());
    auto q = [&](double f) { return v[std::min(v.size() - 1, (size_t)(f * v.size()))]; };
    printf("  %-26s min %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f us\n", name, v.front(), q(0.5), q(0.9), v.back());
}

int main(int argc, char** argv) {
    const int C = argc > 1 ? atoi(argv[1]) : 8;
    const int mod = argc > 2 ? atoi(argv[2]) : 2;
    const int B = 100, H = 2048, G = 4 * H, NS = 2;
    skr::FwdArgs a{};
    a.B = B; a.H = H; a.grp_rows = 0;
    a.xp = dalloc((size_t)B * G); a.ld_xp = G;
    a.R = dalloc((size_t)NS * B * G); a.ld_R = G; a.R_nslab = NS; a.R_slab = (int64_t)B * G;
    a.vec = dalloc((size_t)B * 12 * H); a.vec_gs = H; a.vec_ld = 12 * H;
    a.vec_bias = dalloc(12 * H); a.bias = dalloc(G);
    a.c_prev = dalloc((size_t)B * H);
    a.ln_g = dalloc(G, 1.f); a.ln_b = dalloc(G); a.lnc_g = dalloc(H, 1.f); a.lnc_b = dalloc(H);
    a.forget_bias = 1.f; a.keep = 0.9f;
    int64_t* seed; CK(hipMalloc(&seed, 8)); CK(hipMemset(seed, 0, 8)); a.seed = seed; a.stream = 3;
    a.h_out = dalloc((size_t)B * H);
    a.xhat = dalloc((size_t)B * G); a.rstd = dalloc((size_t)B * 5); a.chat = dalloc((size_t)B * H);
    a.c_carry = dalloc((size_t)B * H);
    a.h_lp = dalloc((size_t)B * H); a.ld_lp = H; a.lp_kind = 1;
    a.r_lp = (__hip_bfloat16*)dalloc((size_t)B * G / 2);
    a.cluster = C;
    uint64_t* part; CK(hipMalloc(&part, (size_t)2 * B * C * 16 * 8)); CK(hipMemset(part, 0, (size_t)2 * B * C * 128));
    int* err; CK(hipMalloc(&err, 4)); CK(hipMemset(err, 0, 4));
    a.part = part; a.err = err;
    uint64_t* tr; CK(hipMalloc(&tr, (size_t)B * C * 8 * 8)); CK(hipMemset(tr, 0, (size_t)B * C * 64));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_cell_trace), &tr, sizeof(tr)));
    const int steps = 50;
    for (int t = 0; t < steps; ++t) {
        a.step = t;
        if (skr_lstm_fwd_step(&a, 1, mod, 0)) { fprintf(stderr, "launch failed\n"); return 1; }
    }
    CK(hipDeviceSynchronize());
    int herr; CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    if (herr) fprintf(stderr, "cluster wait timeout!\n");
    std::vector<uint64_t> h((size_t)B * C * 8);
    CK(hipMemcpy(h.data(), tr, h.size() * 8, hipMemcpyDeviceToHost));
    uint64_t t0 = ~0ull, tend = 0;
    for (int i = 0; i < B * C; ++i) { t0 = std::min(t0, h[i * 8]); tend = std::max(tend, h[i * 8 + 4]); }
    std::vector<double> disp, load, ex1, ex2, st, tot;
    for (int i = 0; i < B * C; ++i) {
        const uint64_t* s = &h[i * 8];
        disp.push_back((s[0] - t0) / 100.0);
        load.push_back((s[1] - s[0]) / 100.0);
        ex1.push_back((s[2] - s[1]) / 100.0);
        ex2.push_back((s[3] - s[2]) / 100.0);
        st.push_back((s[4] - s[3]) / 100.0);
        tot.push_back((s[4] - t0) / 100.0);
    }
    printf("main cell fwd B=%d H=%d C=%d mod=%d: last launch span %.2f us\n", B, H, C, mod, (tend - t0) / 100.0);
    pct("dispatch offset", disp);
    pct("loads landed", load);
    pct("LN exchange 1", ex1);
    pct("cell + LN exchange 2", ex2);
    pct("stores drained", st);
    pct("end offset", tot);
    // back-to-back time per launch (stamps off the hot path: same kernel)
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    for (int t = 0; t < 200; ++t) { a.step = steps + t; skr_lstm_fwd_step(&a, 1, mod, 0); }
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("  eager back-to-back: %.2f us/launch\n", ms * 1000 / 200);
    return 0;
}
