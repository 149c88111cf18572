// Sanitizer driver for the host packer (host-side ASan /
// UBSan on the native runtime). Built with -fsanitize=address,undefined by
// tests/test_native.py and run as its own process: random corpora (sketch
// lengths 2..40, epochs wrapping mid-batch), every output row checked for a
// one-hot pen state and the epoch flag / pointer contract.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

extern "C" int64_t skr_pack_reference(const float* flat, const int64_t* offsets, int64_t n_sketch,
                                      const int64_t* perm, int64_t n_perm, int64_t pointer,
                                      int32_t* epoch_finished, int64_t batch, int64_t n,
                                      const double* scales, float* out);

int main() {
    std::mt19937_64 rng(1234);
    int failures = 0;
    for (int trial = 0; trial < 200; ++trial) {
        const int64_t n_sketch = 1 + rng() % 30;
        std::vector<int64_t> offsets(n_sketch + 1, 0);
        for (int64_t k = 0; k < n_sketch; ++k) offsets[k + 1] = offsets[k] + 2 + (int64_t)(rng() % 39);
        // exact-size heap buffers: any read past a sketch's end at the corpus end is an ASan report
        std::vector<float> flat(offsets[n_sketch] * 4);
        std::uniform_real_distribution<float> u(-1.f, 1.f);
        for (int64_t i = 0; i < offsets[n_sketch]; ++i) {
            flat[i * 4 + 0] = u(rng);
            flat[i * 4 + 1] = u(rng);
            flat[i * 4 + 2] = (rng() % 5 == 0) ? 1.f : 0.f;
            flat[i * 4 + 3] = 0.f;
        }
        std::vector<int64_t> perm(n_sketch);
        for (int64_t k = 0; k < n_sketch; ++k) perm[k] = k;
        std::shuffle(perm.begin(), perm.end(), rng);
        const int64_t batch = 1 + rng() % 8, n = 1 + rng() % 64;
        std::vector<double> scales(2 * batch);
        for (auto& s : scales) s = 0.7 + 0.6 * std::generate_canonical<double, 53>(rng);
        std::vector<float> out(batch * n * 5);
        int64_t pointer = (int64_t)(rng() % n_sketch);
        for (int rep = 0; rep < 5; ++rep) {
            int32_t finished = 0;
            const int64_t p = skr_pack_reference(flat.data(), offsets.data(), n_sketch, perm.data(), n_sketch,
                                                 pointer, &finished, batch, n, scales.data(), out.data());
            if (p < 0 || p >= n_sketch) {
                std::printf("trial %d: bad pointer %lld\n", trial, (long long)p);
                ++failures;
                break;
            }
            for (int64_t r = 0; r < batch * n; ++r) {
                const float* row = &out[r * 5];
                const float s = row[2] + row[3] + row[4];
                if (std::fabs(s - 1.f) > 0 || !std::isfinite(row[0]) || !std::isfinite(row[1])) {
                    std::printf("trial %d: row %lld pen state not one-hot\n", trial, (long long)r);
                    ++failures;
                    break;
                }
            }
            pointer = p;
        }
    }
    std::printf("packer_sanitize: %d failures\n", failures);
    return failures == 0 ? 0 : 1;
}
