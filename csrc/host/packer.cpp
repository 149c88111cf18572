// Host-side batch packer for reference-mode training (capability R6).
//
// Packs B rows of n stroke-5 points [dx, dy, eos, eoc, cont] from a flat
// [total, 4] float32 point buffer (one sketch per offsets[k]..offsets[k+1])
// walking an epoch permutation. Semantics follow the reference packer
// (utils.py:231-264): a row starts at the current sketch's first point, the
// point at idx == len-2 is relabelled eoc and the cursor advances, one extra
// cursor tick per row, per-row (sx, sy) scaling. The scale product is taken
// in double and rounded once, which is what NumPy does for a float32 array
// times a float64 scalar, so the output is bitwise-identical to the Python
// oracle (sketch_rnn_amd/data/loader.py:pack_rows_reference).
#include <cstdint>
#include <cstring>

extern "C" {

int64_t skr_pack_reference(const float* flat, const int64_t* offsets, int64_t n_sketch,
                           const int64_t* perm, int64_t n_perm, int64_t pointer,
                           int32_t* epoch_finished, int64_t batch, int64_t n,
                           const double* scales, float* out) {
    if (n_perm <= 0 || n_sketch <= 0) return -1;
    auto tick = [&]() {
        ++pointer;
        if (pointer >= n_perm) {
            pointer = 0;
            *epoch_finished = 1;
        }
    };
    for (int64_t b = 0; b < batch; ++b) {
        float* row = out + b * n * 5;
        int64_t k = perm[pointer];
        if (k < 0 || k >= n_sketch) return -2;
        const float* data = flat + offsets[k] * 4;
        int64_t len = offsets[k + 1] - offsets[k];
        int64_t idx = 0;
        for (int64_t i = 0; i < n; ++i) {
            float* r = row + i * 5;
            std::memcpy(r, data + idx * 4, 4 * sizeof(float));
            r[4] = (r[2] > 0.f || r[3] > 0.f) ? 0.f : 1.f;
            ++idx;
            if (idx >= len - 1) {
                r[4] = 0.f;
                r[3] = 1.f;
                r[2] = 0.f;
                idx = 0;
                tick();
                k = perm[pointer];
                if (k < 0 || k >= n_sketch) return -2;
                data = flat + offsets[k] * 4;
                len = offsets[k + 1] - offsets[k];
            }
        }
        tick();
        const double sx = scales[2 * b], sy = scales[2 * b + 1];
        for (int64_t i = 0; i < n; ++i) {
            row[i * 5 + 0] = (float)((double)row[i * 5 + 0] * sx);
            row[i * 5 + 1] = (float)((double)row[i * 5 + 1] * sy);
        }
    }
    return pointer;
}

}  // extern "C"
