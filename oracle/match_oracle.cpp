// SPDX-License-Identifier: MIT
//
// sfmx ORACLE — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference's feature-matching hot path, used as the
// parity checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
// leg.  Nothing in the product path (sfm-mvs-pipeline_amd/, include/) links or
// calls this file.
//
// Parity status: UNPINNED against the reference itself.  The reference
// (brunothg/sfm-mvs-pipeline) cannot be built here (OpenCV 4.5.1, Ceres 1.x,
// openMVS, PCL, CGAL are absent, no network) and ships no tests or fixtures
// (SURVEY.md §4, §8c).  The semantics restated below follow the reference call
// sites cited per function plus OpenCV 4.5.1's published BFMatcher /
// batchDistance behaviour [ext], and are cross-checked in tests/ against an
// independent numpy restatement and hand-built known-answer vectors.
//
// What is restated:
//   * cv::BFMatcher(NORM_L2 | NORM_HAMMING)::knnMatch(q, t, m, 2)   [ext]
//       called at src/photogrammetrie/sfm/UnorderedFeatureMatchingStrategy.cpp:50-52
//       (identically VideoFeatureMatchingStrategy.cpp:61-63, GridFeatureMatchingStrategy.cpp:104-106)
//       - L2: d = sqrtf(sum (a-b)^2) (float), ranked on the float's bit pattern
//       - Hamming: d = popcount(a ^ b) (int), DMatch.distance = (float)d
//       - top-2 kept with strict '<' insertion: equal distances keep the lower
//         train index first (OpenCV batchDistance K-NN update loop [ext])
//   * Lowe ratio test + <2-neighbour rule: UnorderedFeatureMatchingStrategy.cpp:54-64
//   * pair generators: Unordered :32-37, Video VideoFeatureMatchingStrategy.cpp:43-48,
//     Grid GridFeatureMatchingStrategy.cpp:48-85
//   * match-graph filters: SfM.cpp:547-570 (distinct-trainIdx filter, min-count)
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#include <algorithm>
#include <omp.h>

namespace {

struct DMatch { int32_t queryIdx, trainIdx, imgIdx; float distance; };  // == cv::DMatch layout

inline uint32_t fbits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

// Squared L2 of two float rows.  8 partial sums in k order, then a left fold.
// For integer-valued descriptors (OpenCV SIFT [ext]) every partial and the
// total are exact integers < 2^24, so this equals OpenCV's SIMD normL2Sqr
// bit-for-bit; for non-integer rows it defines the oracle's own order (the
// GPU fp32 fallback uses the same order).
inline float l2sqr(const float* a, const float* b, int dim) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int k = 0;
    for (; k + 8 <= dim; k += 8)
        for (int l = 0; l < 8; ++l) { float d = a[k + l] - b[k + l]; acc[l] += d * d; }
    for (; k < dim; ++k) { float d = a[k] - b[k]; acc[k & 7] += d * d; }
    float s = acc[0];
    for (int l = 1; l < 8; ++l) s += acc[l];
    return s;
}

inline int hamming(const uint8_t* a, const uint8_t* b, int nbytes) {
    int d = 0, k = 0;
    for (; k + 8 <= nbytes; k += 8) {
        uint64_t x, y; std::memcpy(&x, a + k, 8); std::memcpy(&y, b + k, 8);
        d += __builtin_popcountll(x ^ y);
    }
    for (; k < nbytes; ++k) d += __builtin_popcount((unsigned)(a[k] ^ b[k]));
    return d;
}

// OpenCV batchDistance K=2 insertion on int keys (float bits for L2, ints for
// Hamming): insert iff key < dist[1]; shift only entries strictly greater.
inline void insert2(int32_t key, int32_t j, int32_t* dist, int32_t* idx) {
    if (key < dist[1]) {
        if (dist[0] > key) { dist[1] = dist[0]; idx[1] = idx[0]; dist[0] = key; idx[0] = j; }
        else { dist[1] = key; idx[1] = j; }
    }
}

constexpr int32_t FLT_MAX_BITS = 0x7f7fffff;

}  // namespace

extern "C" {

// knn k=2 over one (query, train) pair.  Writes idx[2*nq], dist[2*nq] and
// returns the number of neighbours per query (= min(2, nt)); idx = -1 marks
// an absent neighbour.
int orc_knn2_l2(const float* q, int nq, const float* t, int nt, int dim, int32_t* idx, float* dist) {
    #pragma omp parallel for schedule(static)
    for (int i = 0; i < nq; ++i) {
        int32_t dk[2] = {FLT_MAX_BITS, FLT_MAX_BITS}, ik[2] = {-1, -1};
        const float* a = q + (size_t)i * dim;
        for (int j = 0; j < nt; ++j) {
            float d = std::sqrt(l2sqr(a, t + (size_t)j * dim, dim));
            insert2((int32_t)fbits(d), j, dk, ik);
        }
        for (int k = 0; k < 2; ++k) {
            idx[2 * i + k] = ik[k];
            float f; uint32_t u = (uint32_t)dk[k]; std::memcpy(&f, &u, 4);
            dist[2 * i + k] = f;
        }
    }
    return nt < 2 ? nt : 2;
}

int orc_knn2_hamming(const uint8_t* q, int nq, const uint8_t* t, int nt, int nbytes, int32_t* idx, float* dist) {
    #pragma omp parallel for schedule(static)
    for (int i = 0; i < nq; ++i) {
        int32_t dk[2] = {INT32_MAX, INT32_MAX}, ik[2] = {-1, -1};
        const uint8_t* a = q + (size_t)i * nbytes;
        for (int j = 0; j < nt; ++j) insert2(hamming(a, t + (size_t)j * nbytes, nbytes), j, dk, ik);
        for (int k = 0; k < 2; ++k) { idx[2 * i + k] = ik[k]; dist[2 * i + k] = (float)dk[k]; }
    }
    return nt < 2 ? nt : 2;
}

// Lowe ratio test over knn results (UnorderedFeatureMatchingStrategy.cpp:54-64):
//   size>=2: accept m[0] iff (double)m[0].distance < (double)m[1].distance * ratio
//   size==1: accept m[0] unconditionally
//   size==0: OpenCV returns no neighbours for an empty train set [ext]; the
//            reference would read m[0] of an empty vector (UB) — we emit nothing.
// Output DMatch{queryIdx, trainIdx, imgIdx=0, distance} in query order.
int64_t orc_ratio_filter(const int32_t* idx, const float* dist, int nq, int nn, double ratio, void* out_v) {
    DMatch* out = (DMatch*)out_v;
    int64_t n = 0;
    for (int i = 0; i < nq; ++i) {
        if (nn == 0) continue;
        bool accept = (nn >= 2) ? ((double)dist[2 * i] < (double)dist[2 * i + 1] * ratio) : true;
        if (accept) out[n++] = DMatch{i, idx[2 * i], 0, dist[2 * i]};
    }
    return n;
}

// One image pair end to end (knnMatch + ratio).  type 0 = f32 rows of `dim`
// floats (NORM_L2), type 1 = u8 rows of `dim` bytes (NORM_HAMMING).
int64_t orc_match_pair(int type, const void* q, int nq, const void* t, int nt, int dim, double ratio, void* out) {
    std::vector<int32_t> idx((size_t)nq * 2);
    std::vector<float> dist((size_t)nq * 2);
    int nn = type == 0 ? orc_knn2_l2((const float*)q, nq, (const float*)t, nt, dim, idx.data(), dist.data())
                       : orc_knn2_hamming((const uint8_t*)q, nq, (const uint8_t*)t, nt, dim, idx.data(), dist.data());
    return orc_ratio_filter(idx.data(), dist.data(), nq, nn, ratio, out);
}

// Pair-parallel batch over a pair list — the reference's OpenMP pair loop
// (UnorderedFeatureMatchingStrategy.cpp:40) with per-pair exact BF matching.
// Results are written per pair at out + out_base[p] (capacity = rows of the
// left image), counts[p] = accepted matches.  This is also the CPU baseline
// leg of bench.py (threads = nthreads, 0 = all cores).
int orc_match_pairs(int type, const void* const* imgs, const int32_t* rows, int dim,
                    const int32_t* pairs, int npairs, double ratio,
                    void* out_v, const int64_t* out_base, int64_t* counts, int nthreads) {
    DMatch* out = (DMatch*)out_v;
    int nt = nthreads > 0 ? nthreads : omp_get_max_threads();
    #pragma omp parallel for schedule(dynamic, 1) num_threads(nt)
    for (int p = 0; p < npairs; ++p) {
        int L = pairs[2 * p], R = pairs[2 * p + 1];
        int nq = rows[L], ntr = rows[R];
        const size_t esz = type == 0 ? sizeof(float) : 1;
        const uint8_t* qb = (const uint8_t*)imgs[L];
        const uint8_t* tb = (const uint8_t*)imgs[R];
        int32_t dk[2], ik[2];
        int64_t n = 0;
        DMatch* o = out + out_base[p];
        for (int i = 0; i < nq; ++i) {
            dk[0] = dk[1] = type == 0 ? FLT_MAX_BITS : INT32_MAX; ik[0] = ik[1] = -1;
            if (type == 0) {
                const float* a = (const float*)(qb + (size_t)i * dim * esz);
                for (int j = 0; j < ntr; ++j) {
                    float d = std::sqrt(l2sqr(a, (const float*)(tb + (size_t)j * dim * esz), dim));
                    insert2((int32_t)fbits(d), j, dk, ik);
                }
            } else {
                const uint8_t* a = qb + (size_t)i * dim;
                for (int j = 0; j < ntr; ++j) insert2(hamming(a, tb + (size_t)j * dim, dim), j, dk, ik);
            }
            int nn = ntr < 2 ? ntr : 2;
            if (nn == 0) continue;
            float d0, d1;
            if (type == 0) { uint32_t u0 = dk[0], u1 = dk[1]; std::memcpy(&d0, &u0, 4); std::memcpy(&d1, &u1, 4); }
            else { d0 = (float)dk[0]; d1 = (float)dk[1]; }
            bool accept = nn >= 2 ? ((double)d0 < (double)d1 * ratio) : true;
            if (accept) o[n++] = DMatch{i, ik[0], 0, d0};
        }
        counts[p] = n;
    }
    return 0;
}

// ---- pair generators (§8a a1) -------------------------------------------
// Each writes (left,right) int32 pairs and returns the pair count; when
// out == nullptr only the count is returned.

int64_t orc_pairs_unordered(int n, int32_t* out) {          // UnorderedFeatureMatchingStrategy.cpp:32-37
    int64_t k = 0;
    for (int i = 0; i < n; ++i)
        for (int j = i + 1; j < n; ++j) { if (out) { out[2 * k] = i; out[2 * k + 1] = j; } ++k; }
    return k;
}

int64_t orc_pairs_video(int n, int seq, int32_t* out) {     // VideoFeatureMatchingStrategy.cpp:43-48
    if (seq < 2) return -1;                                  // setSequenceLength throws (:32-35)
    int64_t k = 0;
    for (int i = 0; i < n; ++i)
        for (int j = i + 1; j < n && (j - (i + 1)) < (seq - 1); ++j) {
            if (out) { out[2 * k] = i; out[2 * k + 1] = j; } ++k;
        }
    return k;
}

// GridFeatureMatchingStrategy.cpp:48-85.  mode 0 ("reference"): rowCount =
// n / rowLength (integer division, :48) — the reference's observable pair
// set; trailing n % rowLength images land outside its VLA (UB) and are never
// enumerated.  mode 1 ("intended"): rowCount = ceil(n / rowLength), empty
// cells skipped.  Both agree when n % rowLength == 0.
int64_t orc_pairs_grid(int n, int seq, int row_len, int mode, int32_t* out) {
    if (seq < 2 || row_len < 1) return -1;                   // setters throw (:32-44)
    int rows = mode == 0 ? n / row_len : (n + row_len - 1) / row_len;
    auto cell = [&](int r, int c) -> int { int i = r * row_len + c; return i < n ? i : -1; };
    int64_t k = 0;
    for (int r = 0; r < rows; ++r)
        for (int c = 0; c < row_len; ++c) {
            if (cell(r, c) < 0) continue;
            for (int dr = 0; dr < seq; ++dr)
                for (int dc = 0; dc < seq; ++dc) {
                    int rr = r + dr, cc = c + dc;
                    bool same = dr == 0 && dc == 0, tri = dr + dc < seq, in = rr < rows && cc < row_len;
                    if (same || !tri || !in || cell(rr, cc) < 0) continue;
                    if (out) { out[2 * k] = cell(r, c); out[2 * k + 1] = cell(rr, cc); }
                    ++k;
                }
        }
    return k;
}

// ---- match-graph filters (§8a a5, SfM.cpp:547-570) ------------------------
// In: per-pair lists at m + base[p], counts[p].  distinct: drop every match
// whose trainIdx appears in another match of the same pair with a different
// queryIdx (:547-564).  Then keep[p] = (count >= min_count) (:566-570, strict
// '<' drops).  Filtering is in place; counts are updated.
int orc_filter_matches(void* m_v, const int64_t* base, int64_t* counts, int npairs,
                       int distinct, int min_count, int32_t* keep) {
    DMatch* m = (DMatch*)m_v;
    for (int p = 0; p < npairs; ++p) {
        DMatch* l = m + base[p];
        int64_t n = counts[p];
        if (distinct) {
            std::vector<DMatch> orig(l, l + n);   // the reference lambda captures the original list by value
            int64_t w = 0;
            for (int64_t a = 0; a < n; ++a) {
                bool dup = false;
                for (int64_t b = 0; b < n && !dup; ++b)
                    dup = orig[a].trainIdx == orig[b].trainIdx && orig[a].queryIdx != orig[b].queryIdx;
                if (!dup) l[w++] = orig[a];
            }
            counts[p] = n = w;
        }
        keep[p] = n < min_count ? 0 : 1;
    }
    return 0;
}

// sqrtf of every integer in [0, n) as float bits — used by tests to locate the
// first float-sqrt collision.
int64_t orc_first_sqrt_collision(int64_t n) {
    float prev = -1.f;
    for (int64_t s = 0; s < n; ++s) {
        float d = std::sqrt((float)s);
        if (d == prev) return s;
        prev = d;
    }
    return -1;
}

}  // extern "C"
