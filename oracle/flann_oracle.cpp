// SPDX-License-Identifier: MIT
//
// sfmx ORACLE — TEST INFRASTRUCTURE ONLY (CPU baseline + recall reference).
//
// A restatement of the reference's *approximate* matcher path, so that
// bench.py can time the faster of the two CPU baselines SURVEY.md §8d asks
// for (exact BF vs FLANN) and tests/ can report exact-vs-FLANN recall
// (FLANN is RNG-driven and rebuilt per pair, so no parity
// oracle is possible for it; the GPU path is exact BF).
//
// Reference call sites:
//   matcher factory  src/photogrammetrie/cli/PhotogrammetrieCli.cpp:371-384
//     SIFT: cv::FlannBasedMatcher(KDTreeIndexParams(5), SearchParams(100))
//     ORB:  cv::FlannBasedMatcher(LshIndexParams(6, 12, 1), SearchParams(100))
//   per-pair use     src/photogrammetrie/sfm/UnorderedFeatureMatchingStrategy.cpp:40-79
//     matcher->knnMatch(left, right, m, 2) — the 2-argument knnMatch clones the
//     matcher with empty train data, adds `right` and trains a NEW index for
//     every pair (OpenCV 4.5.1 DescriptorMatcher::knnMatch [ext]), then the
//     ratio test of :54-64 runs on the returned distances.
//
// Third-party algorithm restated (absent from /root/reference): FLANN 1.6.10
// as bundled in OpenCV 4.5.1 (modules/flann) [ext]:
//   * KDTreeIndex: `trees` randomized kd-trees over the train rows.  Each tree
//     shuffles the row order, then splits recursively at the mean of the
//     highest-variance dimension, chosen at random among the top RAND_DIM=5
//     variances measured on the first SAMPLE_MEAN+1=101 rows of the node; the
//     split index follows FLANN's planeSplit/meanSplit rules (lim1/lim2,
//     balanced fallback).  Leaves hold one row.
//     Search (getNeighbors): one descent per tree, pushing the far branch with
//     its incremental lower bound onto a min-heap; then pop branches while
//     (checks < maxChecks || result not full).  A leaf is checked once per
//     query (bitset).  maxChecks = SearchParams(100).checks.  eps = 0.
//   * LshIndex(table_number=6, key_size=12, multi_probe_level=1): per table a
//     random 12-bit subset of the 256 descriptor bits forms the bucket key; a
//     query probes its own bucket and every bucket at Hamming distance 1 of
//     the key (13 buckets per table), computing the full 256-bit Hamming
//     distance of every row found.  `checks` does not bound LSH (FLANN).
//   * Result set: KNNUniqueResultSet(k=2) — a row seen in several trees or
//     tables is counted once; ordered by (distance, index).
//   * L2 distances are squared inside FLANN; DMatch.distance = sqrt (float).
// Deviation (unavoidable, documented): FLANN draws from the C rand() stream /
// cv::RNG state of the calling thread, so the reference's forests are not
// reproducible even run to run under OpenMP.  Here every pair draws from a
// std::mt19937 seeded with (seed, pair index), so this baseline is
// deterministic.  Its cost per query (index build + ~100 leaf checks, or the
// LSH bucket scans) is the reference's; its matches are *a* FLANN outcome, not
// *the* reference's.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <limits>
#include <queue>
#include <random>
#include <vector>
#include <omp.h>

namespace {

struct DMatch { int32_t queryIdx, trainIdx, imgIdx; float distance; };   // == cv::DMatch layout

constexpr int RAND_DIM = 5;       // FLANN kdtree_index.h
constexpr int SAMPLE_MEAN = 100;  // FLANN kdtree_index.h

// Squared L2, same 8-partial order as match_oracle.cpp::l2sqr.
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

// KNNUniqueResultSet, k = 2: a std::set of (dist, index); once full, only a
// strictly smaller distance enters (`if (dist >= worst_distance_) return;`).
template <typename D>
struct Top2 {
    D d[2];
    int32_t i[2];
    int n = 0;
    void clear() { n = 0; }
    bool full() const { return n == 2; }
    D worst() const { return n == 2 ? d[1] : std::numeric_limits<D>::max(); }
    void add(D dist, int32_t idx) {
        if (n == 2 && !(dist < d[1])) return;
        for (int k = 0; k < n; ++k) if (i[k] == idx) return;
        // insert keeping (dist, idx) order
        int pos = n < 2 ? n : 1;
        if (n < 2) ++n;
        d[pos] = dist; i[pos] = idx;
        if (pos == 1 && (d[1] < d[0] || (d[1] == d[0] && i[1] < i[0]))) { std::swap(d[0], d[1]); std::swap(i[0], i[1]); }
    }
};

// ---------------------------------------------------------------- kd-forest
struct KDNode { int32_t child1, child2; int32_t divfeat; float divval; };   // leaf: child1 < 0, divfeat = row

struct KDForest {
    const float* data; int n, dim;
    std::vector<KDNode> nodes;
    std::vector<int32_t> roots;
    std::vector<float> mean, var;
    std::mt19937& rng;

    KDForest(const float* d, int n_, int dim_, int trees, std::mt19937& r) : data(d), n(n_), dim(dim_), rng(r) {
        mean.resize(dim); var.resize(dim);
        nodes.reserve((size_t)trees * 2 * (size_t)std::max(n, 1));
        std::vector<int32_t> ind(n);
        for (int t = 0; t < trees; ++t) {
            for (int i = 0; i < n; ++i) ind[i] = i;
            std::shuffle(ind.begin(), ind.end(), rng);          // FLANN: random_shuffle per tree
            roots.push_back(n ? divide(ind.data(), n) : -1);
        }
    }
    const float* row(int i) const { return data + (size_t)i * dim; }

    int32_t divide(int32_t* ind, int count) {
        const int32_t id = (int32_t)nodes.size();
        nodes.push_back(KDNode{-1, -1, 0, 0.f});
        if (count == 1) { nodes[id].divfeat = ind[0]; return id; }
        int idx, cutfeat; float cutval;
        mean_split(ind, count, idx, cutfeat, cutval);
        const int32_t c1 = divide(ind, idx);
        const int32_t c2 = divide(ind + idx, count - idx);
        nodes[id] = KDNode{c1, c2, cutfeat, cutval};
        return id;
    }

    void mean_split(int32_t* ind, int count, int& index, int& cutfeat, float& cutval) {
        std::fill(mean.begin(), mean.end(), 0.f);
        std::fill(var.begin(), var.end(), 0.f);
        const int cnt = std::min(SAMPLE_MEAN + 1, count);
        for (int j = 0; j < cnt; ++j) { const float* v = row(ind[j]); for (int k = 0; k < dim; ++k) mean[k] += v[k]; }
        for (int k = 0; k < dim; ++k) mean[k] /= cnt;
        for (int j = 0; j < cnt; ++j) {
            const float* v = row(ind[j]);
            for (int k = 0; k < dim; ++k) { const float t = v[k] - mean[k]; var[k] += t * t; }
        }
        cutfeat = select_division();
        cutval = mean[cutfeat];
        int lim1, lim2;
        plane_split(ind, count, cutfeat, cutval, lim1, lim2);
        if (lim1 > count / 2) index = lim1;
        else if (lim2 < count / 2) index = lim2;
        else index = count / 2;
        if (lim1 == count || lim2 == 0) index = count / 2;   // all rows identical along the cut
    }

    int select_division() {
        int num = 0, top[RAND_DIM];
        for (int i = 0; i < dim; ++i) {
            if (num < RAND_DIM || var[i] > var[top[num - 1]]) {
                if (num < RAND_DIM) top[num++] = i; else top[num - 1] = i;
                for (int j = num - 1; j > 0 && var[top[j]] > var[top[j - 1]]; --j) std::swap(top[j], top[j - 1]);
            }
        }
        return top[std::uniform_int_distribution<int>(0, num - 1)(rng)];
    }

    void plane_split(int32_t* ind, int count, int f, float cv, int& lim1, int& lim2) {
        int left = 0, right = count - 1;
        for (;;) {
            while (left <= right && row(ind[left])[f] < cv) ++left;
            while (left <= right && row(ind[right])[f] >= cv) --right;
            if (left > right) break;
            std::swap(ind[left], ind[right]); ++left; --right;
        }
        lim1 = left;
        right = count - 1;
        for (;;) {
            while (left <= right && row(ind[left])[f] <= cv) ++left;
            while (left <= right && row(ind[right])[f] > cv) --right;
            if (left > right) break;
            std::swap(ind[left], ind[right]); ++left; --right;
        }
        lim2 = left;
    }

    struct Branch { float mindist; int32_t node; bool operator>(const Branch& o) const { return mindist > o.mindist; } };
    using Heap = std::priority_queue<Branch, std::vector<Branch>, std::greater<Branch>>;

    void search_level(Top2<float>& res, const float* q, int32_t node, float mindist, int& checks, int max_checks,
                      Heap& heap, std::vector<uint8_t>& checked) const {
        for (;;) {
            if (res.worst() < mindist) return;
            const KDNode& nd = nodes[node];
            if (nd.child1 < 0) {
                const int idx = nd.divfeat;
                if (checked[idx] || (checks >= max_checks && res.full())) return;
                checked[idx] = 1;
                ++checks;
                res.add(l2sqr(q, row(idx), dim), idx);
                return;
            }
            const float val = q[nd.divfeat], diff = val - nd.divval;
            const int32_t best = diff < 0 ? nd.child1 : nd.child2, other = diff < 0 ? nd.child2 : nd.child1;
            const float nd2 = mindist + diff * diff;            // L2::accum_dist
            if (nd2 < res.worst() || !res.full()) heap.push(Branch{nd2, other});
            node = best;                                         // tail recursion on the near child
        }
    }

    void knn2(const float* q, int max_checks, Top2<float>& res, Heap& heap, std::vector<uint8_t>& checked) const {
        res.clear();
        while (!heap.empty()) heap.pop();
        std::fill(checked.begin(), checked.end(), 0);
        int checks = 0;
        for (int32_t r : roots) if (r >= 0) search_level(res, q, r, 0.f, checks, max_checks, heap, checked);
        while (!heap.empty() && (checks < max_checks || !res.full())) {
            const Branch b = heap.top(); heap.pop();
            search_level(res, q, b.node, b.mindist, checks, max_checks, heap, checked);
        }
    }
};

// ---------------------------------------------------------------- LSH
struct LshTables {
    const uint8_t* data; int n, nbytes, key_size;
    std::vector<std::vector<int>> key_bits;                 // per table: bit positions
    std::vector<std::vector<int32_t>> start, items;         // per table: bucket CSR (2^key_size buckets)

    uint32_t key(int t, const uint8_t* v) const {
        uint32_t k = 0;
        for (int b = 0; b < key_size; ++b) {
            const int bit = key_bits[t][b];
            k |= (uint32_t)((v[bit >> 3] >> (bit & 7)) & 1u) << b;
        }
        return k;
    }
    LshTables(const uint8_t* d, int n_, int nbytes_, int tables, int ks, std::mt19937& rng)
        : data(d), n(n_), nbytes(nbytes_), key_size(ks) {
        const int nb = 1 << ks;
        std::vector<int> bits(nbytes * 8);
        for (int t = 0; t < tables; ++t) {
            for (int i = 0; i < nbytes * 8; ++i) bits[i] = i;
            std::shuffle(bits.begin(), bits.end(), rng);         // FLANN LshTable: random subset of bits
            key_bits.emplace_back(bits.begin(), bits.begin() + ks);
            std::vector<int32_t> cnt(nb + 1, 0), it(n);
            std::vector<uint32_t> keys(n);
            for (int i = 0; i < n; ++i) { keys[i] = key(t, d + (size_t)i * nbytes); ++cnt[keys[i] + 1]; }
            for (int b = 0; b < nb; ++b) cnt[b + 1] += cnt[b];
            std::vector<int32_t> fill(cnt.begin(), cnt.end() - 1);
            for (int i = 0; i < n; ++i) it[fill[keys[i]]++] = i;
            start.push_back(std::move(cnt));
            items.push_back(std::move(it));
        }
    }
    void knn2(const uint8_t* q, Top2<int>& res) const {
        res.clear();
        for (size_t t = 0; t < key_bits.size(); ++t) {
            const uint32_t k0 = key((int)t, q);
            for (int m = -1; m < key_size; ++m) {                // multi_probe_level 1: own bucket + 1-bit flips
                const uint32_t k = m < 0 ? k0 : (k0 ^ (1u << m));
                for (int32_t e = start[t][k]; e < start[t][k + 1]; ++e) {
                    const int idx = items[t][e];
                    res.add(hamming(q, data + (size_t)idx * nbytes, nbytes), idx);
                }
            }
        }
    }
};

}  // namespace

extern "C" {

// Pair-parallel FLANN-style matching — the reference's OpenMP pair loop
// (UnorderedFeatureMatchingStrategy.cpp:40) with a per-pair index build.
// Same packing as orc_match_pairs (match_oracle.cpp).  type 0 = f32 rows
// (KDTreeIndexParams(trees), SearchParams(checks)), type 1 = u8 rows
// (LshIndexParams(tables, key_size, 1)).
int orc_flann_match_pairs(int type, const void* const* imgs, const int32_t* rows, int dim,
                          const int32_t* pairs, int npairs, double ratio, void* out_v, const int64_t* out_base,
                          int64_t* counts, int nthreads, int trees, int checks, int tables, int key_size,
                          uint64_t seed) {
    DMatch* out = (DMatch*)out_v;
    const int nt = nthreads > 0 ? nthreads : omp_get_max_threads();
    #pragma omp parallel for schedule(dynamic, 1) num_threads(nt)
    for (int p = 0; p < npairs; ++p) {
        const int L = pairs[2 * p], R = pairs[2 * p + 1];
        const int nq = rows[L], ntr = rows[R];
        std::mt19937 rng((uint32_t)((seed * 0x9E3779B97F4A7C15ull + (uint64_t)p * 0xBF58476D1CE4E5B9ull) >> 17));
        DMatch* o = out + out_base[p];
        int64_t n = 0;
        auto emit = [&](int i, int nn, int32_t i0, float d0, float d1) {
            if (nn == 0) return;                                 // reference: m[0] of empty vector (UB)
            const bool accept = nn >= 2 ? ((double)d0 < (double)d1 * ratio) : true;   // :54-64
            if (accept) o[n++] = DMatch{i, i0, 0, d0};
        };
        if (type == 0) {
            const float* qb = (const float*)imgs[L];
            const float* tb = (const float*)imgs[R];
            KDForest forest(tb, ntr, dim, trees, rng);
            KDForest::Heap heap;
            std::vector<uint8_t> checked(std::max(ntr, 1));
            Top2<float> res;
            for (int i = 0; i < nq; ++i) {
                forest.knn2(qb + (size_t)i * dim, checks, res, heap, checked);
                emit(i, res.n, res.n ? res.i[0] : -1, res.n ? std::sqrt(res.d[0]) : 0.f,
                     res.n > 1 ? std::sqrt(res.d[1]) : 0.f);
            }
        } else {
            const uint8_t* qb = (const uint8_t*)imgs[L];
            const uint8_t* tb = (const uint8_t*)imgs[R];
            LshTables lsh(tb, ntr, dim, tables, key_size, rng);
            Top2<int> res;
            for (int i = 0; i < nq; ++i) {
                lsh.knn2(qb + (size_t)i * dim, res);
                emit(i, res.n, res.n ? res.i[0] : -1, res.n ? (float)res.d[0] : 0.f, res.n > 1 ? (float)res.d[1] : 0.f);
            }
        }
        counts[p] = n;
    }
    return 0;
}

}  // extern "C"
