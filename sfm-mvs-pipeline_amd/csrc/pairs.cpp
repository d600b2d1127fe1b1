// SPDX-License-Identifier: MIT
// sfmx pair enumeration (§8a a1) — the three reference strategies' pair loops,
// host-side (negligible cost: O(pairs) integer work).
//   Unordered: src/photogrammetrie/sfm/UnorderedFeatureMatchingStrategy.cpp:32-37
//   Video:     src/photogrammetrie/sfm/VideoFeatureMatchingStrategy.cpp:43-48 (seq >= 2, :32-35)
//   Grid:      src/photogrammetrie/sfm/GridFeatureMatchingStrategy.cpp:48-85 (seq >= 2, rowLength >= 1, :32-44)
#include <cstdint>
#include "../../include/sfmx.h"

namespace {
struct Emit {
    int32_t* out; int64_t cap; int64_t n = 0;
    void operator()(int32_t l, int32_t r) {
        if (out && n < cap) { out[2 * n] = l; out[2 * n + 1] = r; }
        ++n;
    }
};
}  // namespace

extern "C" {

int64_t sfmx_pairs_unordered(int32_t n_images, int32_t* out, int64_t cap) {
    if (n_images < 0) return SFMX_EINVAL;
    Emit e{out, cap};
    for (int32_t i = 0; i < n_images; ++i)
        for (int32_t j = i + 1; j < n_images; ++j) e(i, j);
    return e.n;
}

int64_t sfmx_pairs_video(int32_t n_images, int32_t seq, int32_t* out, int64_t cap) {
    if (n_images < 0 || seq < 2) return SFMX_EINVAL;
    Emit e{out, cap};
    for (int32_t i = 0; i < n_images; ++i)
        for (int32_t j = i + 1; j < n_images && (j - (i + 1)) < (seq - 1); ++j) e(i, j);
    return e.n;
}

int64_t sfmx_pairs_grid(int32_t n_images, int32_t seq, int32_t row_len, int32_t grid_mode, int32_t* out, int64_t cap) {
    if (n_images < 0 || seq < 2 || row_len < 1 || (grid_mode != 0 && grid_mode != 1)) return SFMX_EINVAL;
    // mode 0: rowCount = n / rowLength as the reference computes it (:48, integer
    // division inside ceil); mode 1: ceil, with empty trailing cells skipped.
    const int32_t rows = grid_mode == 0 ? n_images / row_len : (n_images + row_len - 1) / row_len;
    auto cell = [&](int32_t r, int32_t c) -> int32_t {
        const int64_t i = (int64_t)r * row_len + c;
        return i < n_images ? (int32_t)i : -1;
    };
    Emit e{out, cap};
    for (int32_t r = 0; r < rows; ++r)
        for (int32_t c = 0; c < row_len; ++c) {
            if (cell(r, c) < 0) continue;
            for (int32_t dr = 0; dr < seq; ++dr)          // loop order row -> col -> dr -> dc (:62-85)
                for (int32_t dc = 0; dc < seq; ++dc) {
                    const int32_t rr = r + dr, cc = c + dc;
                    const bool same = dr == 0 && dc == 0;
                    const bool tri = dr + dc < seq;
                    const bool in = rr < rows && cc < row_len;
                    if (same || !tri || !in || cell(rr, cc) < 0) continue;
                    e(cell(r, c), cell(rr, cc));
                }
        }
    return e.n;
}

}  // extern "C"
