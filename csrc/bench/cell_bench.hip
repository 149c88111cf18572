// Microbenchmark of the fused cell kernels at the flagship shapes (not part
// of the library). Build: hipcc -O3 --offload-arch=gfx950 -I csrc
// csrc/bench/cell_bench.hip -o build/cell_bench ; run on the GPU box.
// Times back-to-back launches (steps) of one configuration with hipEvents and
// prints microseconds per launch, so variants (LN / MOD / cluster width /
// slab count / batch) can be compared in isolation.
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
    std::vector<float> h(n, v);
    for (size_t i = 0; i < n; ++i) h[i] = v * (float)((i * 2654435761u) % 1000) / 1000.f;
    CK(hipMemcpy(p, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
    return p;
}

struct Cfg {
    const char* name;
    int B, H, C, NS;
    bool ln, mod;   // mod: bf16 modulation vectors (the HyperLSTM main cell)
    int dhr = 2, dhr2 = 0, dho = 1;   // backward dh split-K slab counts (dh_rec, dh_rec2, dh_out)
};

static double run_fwd(const Cfg& c, int steps) {
    const int B = c.B, H = c.H, G = 4 * H;
    skr::FwdArgs a{};
    a.B = B; a.H = H; a.grp_rows = 0;
    a.xp = dalloc((size_t)B * G); a.ld_xp = G;
    a.R = dalloc((size_t)c.NS * B * G); a.ld_R = G; a.R_nslab = c.NS; a.R_slab = (int64_t)B * G;
    a.vec = dalloc((size_t)B * 12 * H); a.vec_gs = H; a.vec_ld = 12 * H;
    a.vec_bias = dalloc(12 * H); a.bias = dalloc(G);
    a.c_prev = dalloc((size_t)B * H);
    a.ln_g = dalloc(G, 1.f); a.ln_b = dalloc(G); a.lnc_g = dalloc(H, 1.f); a.lnc_b = dalloc(H);
    a.forget_bias = 1.f; a.keep = 0.9f;
    int64_t* seed; CK(hipMalloc(&seed, 8)); CK(hipMemset(seed, 0, 8)); a.seed = seed; a.stream = 3;
    a.h_out = dalloc((size_t)B * H); a.c_out = dalloc((size_t)B * H); a.act = dalloc((size_t)B * G);
    a.xhat = dalloc((size_t)B * G); a.rstd = dalloc((size_t)B * 5); a.chat = dalloc((size_t)B * H);
    a.h_carry = dalloc((size_t)B * H); a.c_carry = dalloc((size_t)B * H);
    a.h_lp = dalloc((size_t)B * H); a.ld_lp = H; a.lp_kind = 1;
    a.cluster = c.C;
    uint64_t* part; CK(hipMalloc(&part, (size_t)2 * B * c.C * 16 * 8)); CK(hipMemset(part, 0, (size_t)2 * B * c.C * 128));
    int* err; CK(hipMalloc(&err, 4)); CK(hipMemset(err, 0, 4));
    a.part = part; a.err = err;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int t = 0; t < 5; ++t) { a.step = t; if (skr_lstm_fwd_step(&a, c.ln, c.mod ? 2 : 0, 0)) { fprintf(stderr, "launch failed\n"); exit(1); } }
    CK(hipDeviceSynchronize());
    // capture the launches in a graph: times kernels + graph boundaries, not host launch cost
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipMemset(part, 0, (size_t)2 * B * c.C * 128));
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int t = 0; t < steps; ++t) { a.step = 5 + t; skr_lstm_fwd_step(&a, c.ln, c.mod ? 2 : 0, st); }
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    CK(hipMemset(part, 0, (size_t)2 * B * c.C * 128));
    CK(hipEventRecord(e0, st));
    CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    int herr; CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    if (herr) fprintf(stderr, "cluster wait timeout!\n");
    return 1000.0 * ms / steps;
}

static double run_bwd(const Cfg& c, int steps) {
    const int B = c.B, H = c.H, G = 4 * H;
    skr::BwdArgs a{};
    a.B = B; a.H = H; a.grp_rows = 0;
    a.dh_out = dalloc((size_t)c.dho * B * H); a.dho_nslab = c.dho; a.dho_slab = (int64_t)B * H;
    a.dh_rec = dalloc((size_t)c.dhr * B * H); a.ld_dh_rec = H; a.dhr_nslab = c.dhr; a.dhr_slab = (int64_t)B * H;
    if (c.dhr2 > 0) {
        a.dh_rec2 = dalloc((size_t)c.dhr2 * B * H); a.ld_dh_rec2 = H; a.dhr2_nslab = c.dhr2;
        a.dhr2_slab = (int64_t)B * H;
    }
    a.dc_rec = dalloc((size_t)B * H);
    a.act = dalloc((size_t)B * G); a.c_new = dalloc((size_t)B * H); a.c_prev = dalloc((size_t)B * H);
    a.xhat = dalloc((size_t)B * G); a.rstd = dalloc((size_t)B * 5, 1.f); a.chat = dalloc((size_t)B * H);
    a.ln_g = dalloc(G, 1.f); a.ln_b = dalloc(G); a.lnc_g = dalloc(H, 1.f); a.lnc_b = dalloc(H);
    a.forget_bias = 1.f;
    a.xp = dalloc((size_t)B * G); a.ld_xp = G;
    a.R = dalloc((size_t)c.NS * B * G); a.ld_R = G; a.R_nslab = c.NS; a.R_slab = (int64_t)B * G;
    a.vec = dalloc((size_t)B * 12 * H); a.vec_gs = H; a.vec_ld = 12 * H; a.vec_bias = dalloc(12 * H);
    a.keep = 0.9f;
    int64_t* seed; CK(hipMalloc(&seed, 8)); CK(hipMemset(seed, 0, 8)); a.seed = seed; a.stream = 3;
    a.dG = nullptr; a.ld_dG = G;
    a.dG_lp = dalloc((size_t)B * G); a.ld_dG_lp = G; a.dG_lp_kind = 1;
    a.dxp = dalloc((size_t)B * G); a.ld_dxp = G; a.dxp_kind = 1;
    a.dvec = dalloc((size_t)B * 12 * H); a.dvec_kind = 1;
    a.dlny = dalloc((size_t)B * G); a.dlncy = dalloc((size_t)B * H);
    a.cluster = c.C;
    uint64_t* part; CK(hipMalloc(&part, (size_t)2 * B * c.C * 16 * 8)); CK(hipMemset(part, 0, (size_t)2 * B * c.C * 128));
    int* err; CK(hipMalloc(&err, 4)); CK(hipMemset(err, 0, 4));
    a.part = part; a.err = err;
    const int mod = c.mod ? 2 : 0;
    for (int t = 0; t < 5; ++t) { a.step = t; if (skr_lstm_bwd_step(&a, c.ln, mod, 0)) { fprintf(stderr, "launch failed\n"); exit(1); } }
    CK(hipDeviceSynchronize());
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipMemset(part, 0, (size_t)2 * B * c.C * 128));
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int t = 0; t < steps; ++t) { a.step = 5 + t; skr_lstm_bwd_step(&a, c.ln, mod, st); }
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    CK(hipMemset(part, 0, (size_t)2 * B * c.C * 128));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, st));
    CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    int herr; CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    if (herr) fprintf(stderr, "cluster wait timeout!\n");
    return 1000.0 * ms / steps;
}

int main(int argc, char** argv) {
    const int steps = argc > 1 ? atoi(argv[1]) : 200;
    const Cfg cfgs[] = {
        {"main hyper  H2048 C8 NS2 LN MOD", 100, 2048, 8, 2, true, true},
        {"main hyper  H2048 C4 NS2 LN MOD", 100, 2048, 4, 2, true, true},
        {"main hyper  H2048 C2 NS2 LN MOD", 100, 2048, 2, 2, true, true},
        {"main hyper  H2048 C1 NS2 LN MOD", 100, 2048, 1, 2, true, true},
        {"main LN     H2048 C8 NS2 LN    ", 100, 2048, 8, 2, true, false},
        {"main LN     H2048 C1 NS2 LN    ", 100, 2048, 1, 2, true, false},
        {"main LN     H2048 C2 NS2 LN    ", 100, 2048, 2, 2, true, false},
        {"main plain  H2048 C8 NS2       ", 100, 2048, 8, 2, false, false},
        {"main plain  H2048 C8 NS1       ", 100, 2048, 8, 1, false, false},
        {"hyper cell  H256  C1 NS2 LN    ", 100, 256, 1, 2, true, false},
        {"LN          H1024 C1 NS2 LN    ", 100, 1024, 1, 2, true, false},
        {"LN          H1024 C4 NS2 LN    ", 100, 1024, 4, 2, true, false},
        {"hyper plain H256  C1 NS1       ", 100, 256, 1, 1, false, false},
        {"encoder     H512  C2 NS4 (2B)  ", 200, 512, 2, 4, false, false},
        {"tiny        H64   C1 NS1 B8    ", 8, 64, 1, 1, false, false},
        // vae_large backward slab counts: main cell dh 8 + 8 slabs, hyper cell dh_out 32 + dh_rec 8
        {"main hyper  H2048 C8 dh 8+8      ", 100, 2048, 8, 2, true, true, 8, 8, 1},
        {"hyper cell  H256  C1 dh 8, out 32", 100, 256, 1, 1, true, false, 8, 0, 32},
    };
    for (const Cfg& c : cfgs) printf("fwd %-36s %8.2f us/launch\n", c.name, run_fwd(c, steps));
    for (const Cfg& c : cfgs)
        if (c.ln) printf("bwd %-36s %8.2f us/launch\n", c.name, run_bwd(c, steps));
    return 0;
}
