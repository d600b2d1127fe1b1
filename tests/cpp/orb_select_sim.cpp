// Test helper (CPU): the parallel formulation of KeyPointsFilter::retainBest for a device selection
// (the r03 orb_retain_kernel, tools/archive/r03_unvalidated_orb_device_retain.patch), restated sequentially and compared
// with libstdc++'s own std::nth_element / std::partition / std::__introselect / std::__heap_select
// on random arrays with many ties.  Exit status 0 = every permutation identical.
//
// The formulation ("retainBest on the device"):
//  * __unguarded_partition(first + 1, last, pivot = first) with comp = response greater: the left
//    scan stops at positions with response <= P (Ls, ascending), the right scan at response >= P
//    (Rs, descending).  While Ls[k] < Rs[k] the two are swapped; K = the number of such k (a prefix,
//    Ls rises and Rs falls).  Swapped positions lie behind both scans, so every stop is at an
//    original position, and the returned cut is min(Ls[K + 1], Rs[K]).
//  * std::partition(first, last, pred) (bidirectional form): the same pairing with Ls = !pred
//    positions and Rs = pred positions; the result is first + count(pred).
#include <algorithm>
#include <climits>
#include <cstdio>
#include <random>
#include <vector>

struct Resp {
    float response;
    int idx;
};
static bool greater_r(const Resp& a, const Resp& b) { return a.response > b.response; }

static int hoare_step(std::vector<Resp>& a, int f, int l, float P) {
    std::vector<int> Ls, Rs;   // both ascending
    for (int p = f; p < l; ++p) {
        if (a[p].response <= P) Ls.push_back(p);
        if (a[p].response >= P) Rs.push_back(p);
    }
    const int nL = (int)Ls.size(), nR = (int)Rs.size();
    int K = 0;
    while (K < std::min(nL, nR) && Ls[K] < Rs[nR - 1 - K]) ++K;
    for (int k = 0; k < K; ++k) std::swap(a[Ls[k]], a[Rs[nR - 1 - k]]);
    int cut = INT_MAX;
    if (K < nL) cut = Ls[K];
    if (K >= 1) cut = std::min(cut, Rs[nR - K]);
    return cut;
}

static int partition_step(std::vector<Resp>& a, int f, int l, float amb) {
    std::vector<int> Ln, Rp;
    for (int p = f; p < l; ++p) (a[p].response >= amb ? Rp : Ln).push_back(p);
    const int nL = (int)Ln.size(), nR = (int)Rp.size();
    int K = 0;
    while (K < std::min(nL, nR) && Ln[K] < Rp[nR - 1 - K]) ++K;
    for (int k = 0; k < K; ++k) std::swap(a[Ln[k]], a[Rp[nR - 1 - k]]);
    return f + nR;
}

static void move_median_to_first(std::vector<Resp>& v, int result, int a, int b, int c) {
    auto cmp = [&](int x, int y) { return greater_r(v[x], v[y]); };
    if (cmp(a, b)) {
        if (cmp(b, c)) std::swap(v[result], v[b]);
        else if (cmp(a, c)) std::swap(v[result], v[c]);
        else std::swap(v[result], v[a]);
    } else if (cmp(a, c)) std::swap(v[result], v[a]);
    else if (cmp(b, c)) std::swap(v[result], v[c]);
    else std::swap(v[result], v[b]);
}

// libstdc++ heap helpers (stl_heap.h), on positions of v
static void push_heap_(std::vector<Resp>& v, int first, int hole, int top, Resp value) {
    int parent = (hole - 1) / 2;
    while (hole > top && greater_r(v[first + parent], value)) {
        v[first + hole] = v[first + parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    v[first + hole] = value;
}
static void adjust_heap_(std::vector<Resp>& v, int first, int hole, int len, Resp value) {
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (greater_r(v[first + second], v[first + second - 1])) second--;
        v[first + hole] = v[first + second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        v[first + hole] = v[first + second - 1];
        hole = second - 1;
    }
    push_heap_(v, first, hole, top, value);
}
static void heap_select_(std::vector<Resp>& v, int first, int middle, int last) {
    const int len = middle - first;
    if (len >= 2)
        for (int parent = (len - 2) / 2;; --parent) {
            adjust_heap_(v, first, parent, len, v[first + parent]);
            if (parent == 0) break;
        }
    for (int i = middle; i < last; ++i)
        if (greater_r(v[i], v[first])) {
            const Resp value = v[i];
            v[i] = v[first];
            adjust_heap_(v, first, 0, len, value);
        }
}
static void insertion_sort_(std::vector<Resp>& v, int first, int last) {
    if (first == last) return;
    for (int i = first + 1; i < last; ++i) {
        const Resp val = v[i];
        if (greater_r(val, v[first])) {
            for (int j = i; j > first; --j) v[j] = v[j - 1];
            v[first] = val;
        } else {
            int j = i;
            while (greater_r(val, v[j - 1])) { v[j] = v[j - 1]; --j; }
            v[j] = val;
        }
    }
}
static int lg_(int n) { return 31 - __builtin_clz(n); }

static void introselect_(std::vector<Resp>& v, int first, int nth, int last, int depth) {
    while (last - first > 3) {
        if (depth == 0) {
            heap_select_(v, first, nth + 1, last);
            std::swap(v[first], v[nth]);
            return;
        }
        --depth;
        const int mid = first + (last - first) / 2;
        move_median_to_first(v, first, first + 1, mid, last - 1);
        const int cut = hoare_step(v, first + 1, last, v[first].response);
        if (cut <= nth) first = cut;
        else last = cut;
    }
    insertion_sort_(v, first, last);
}

static void retain_sim(std::vector<Resp>& k, int n) {
    if (n >= 0 && (int)k.size() > n) {
        if (n == 0) { k.clear(); return; }
        introselect_(k, 0, n - 1, (int)k.size(), 2 * lg_((int)k.size()));
        const float amb = k[n - 1].response;
        k.resize(partition_step(k, n, (int)k.size(), amb));
    }
}
static void retain_ref(std::vector<Resp>& k, int n) {   // csrc/orb_features.hip retain_best (the r02 host form)
    if (n >= 0 && k.size() > (size_t)n) {
        if (n == 0) { k.clear(); return; }
        std::nth_element(k.begin(), k.begin() + n - 1, k.end(), greater_r);
        const float amb = k[n - 1].response;
        auto end = std::partition(k.begin() + n, k.end(), [amb](const Resp& p) { return p.response >= amb; });
        k.resize(end - k.begin());
    }
}

static bool same(const std::vector<Resp>& a, const std::vector<Resp>& b) {
    if (a.size() != b.size()) return false;
    for (size_t i = 0; i < a.size(); ++i)
        if (a[i].idx != b[i].idx || a[i].response != b[i].response) return false;
    return true;
}

int main(int argc, char** argv) {
    const int cases = argc > 1 ? atoi(argv[1]) : 3000;
    std::mt19937 rng(12345);
    int bad = 0;
    for (int t = 0; t < cases; ++t) {
        const int m = 1 + (int)(rng() % (t % 10 == 0 ? 60000 : 3000));
        const int range = 1 + (int)(rng() % (t % 3 == 0 ? 8 : t % 3 == 1 ? 256 : 1000000));
        std::vector<Resp> a(m);
        for (int i = 0; i < m; ++i) a[i] = Resp{(float)(rng() % range) * (t % 4 == 0 ? 0.37f : 1.f), i};
        const int n = (int)(rng() % (m + 2));
        std::vector<Resp> r1 = a, r2 = a;
        retain_ref(r1, n);
        retain_sim(r2, n);
        if (!same(r1, r2)) { ++bad; if (bad < 5) printf("retain mismatch: m %d n %d range %d\n", m, n, range); }
        // the heap_select fallback and small depth limits, against libstdc++'s own internals
        if (m >= 2) {
            const int nth = (int)(rng() % m), depth = (int)(rng() % 4);
            std::vector<Resp> h1 = a, h2 = a;
            std::__introselect(h1.begin(), h1.begin() + nth, h1.end(), depth, __gnu_cxx::__ops::__iter_comp_iter(greater_r));
            introselect_(h2, 0, nth, m, depth);
            if (!same(h1, h2)) { ++bad; if (bad < 5) printf("introselect(depth %d) mismatch: m %d nth %d\n", depth, m, nth); }
        }
    }
    printf("%d cases, %d mismatches\n", cases, bad);
    return bad ? 1 : 0;
}
