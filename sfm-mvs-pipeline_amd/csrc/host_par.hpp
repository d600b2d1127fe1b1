// Host-side parallel loop for the BA problem setup (sfmx_ba_create / _update / _solve): the
// reference adjusts a growing scene after every registered camera (SfM.cpp:235 / :371), so the
// O(observations) host work of every call is on the critical path.  Work is split into a FIXED
// number of ranges (independent of the machine's thread count), so every result is the same on
// every host; the ranges run on up to 16 std::threads.
#pragma once
#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

namespace sfmx {

inline int host_threads() {
    const unsigned h = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(16u, h ? h : 1u));
}

// f(i) for i in [0, n): items taken from a shared counter by up to host_threads() threads
template <class F>
void parallel_items(int n, F&& f) {
    const int nt = std::min(host_threads(), n);
    if (nt <= 1) {
        for (int i = 0; i < n; ++i) f(i);
        return;
    }
    std::atomic<int> next{0};
    auto work = [&]() {
        for (int i = next.fetch_add(1); i < n; i = next.fetch_add(1)) f(i);
    };
    std::vector<std::thread> th;
    th.reserve(nt - 1);
    for (int t = 1; t < nt; ++t) th.emplace_back(work);
    work();
    for (auto& t : th) t.join();
}

// f(begin, end) over [0, n) in `pieces` fixed ranges
template <class F>
void parallel_ranges(int64_t n, int pieces, F&& f) {
    pieces = (int)std::max<int64_t>(1, std::min<int64_t>(pieces, n));
    parallel_items(pieces, [&](int i) { f(n * i / pieces, n * (i + 1) / pieces); });
}

}  // namespace sfmx
