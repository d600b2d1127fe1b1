// Host-side parallel loop for the BA problem setup (sfmx_ba_create / _update / _solve): the
// reference adjusts a growing scene after every registered camera (SfM.cpp:235 / :371), so the
// O(observations) host work of every call is on the critical path.  Work is split into a FIXED
// number of ranges (independent of the machine's thread count), so every result is the same on
// every host; the ranges run on up to 16 threads (a persistent pool).
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace sfmx {

inline int host_threads() {
    const unsigned h = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(16u, h ? h : 1u));
}

// A persistent worker pool (host_threads() - 1 threads, started on first use): spawning and joining
// 15 std::threads per parallel loop cost ~0.1-0.2 ms each, and a BA call makes ~10 such loops.  One
// job at a time; a caller that finds the pool busy (another thread's loop) runs its loop serially.
class HostPool {
public:
    explicit HostPool(int workers) {
        for (int t = 0; t < workers; ++t) th_.emplace_back([this] { loop(); });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    // runs work() on every worker and on the caller; returns when all have returned. false: busy.
    template <class W>
    bool run(W& work) {
        std::unique_lock<std::mutex> busy(run_mu_, std::try_to_lock);
        if (!busy.owns_lock()) return false;
        std::function<void()> job = [&work] { work(); };
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &job;
            pending_ = (int)th_.size();
            ++gen_;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [this] { return pending_ == 0; });
        job_ = nullptr;
        return true;
    }

private:
    void loop() {
        unsigned seen = 0;
        for (;;) {
            std::function<void()>* job;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                job = job_;
            }
            (*job)();
            std::lock_guard<std::mutex> lk(mu_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_, run_mu_;
    std::condition_variable cv_, done_;
    std::function<void()>* job_ = nullptr;
    unsigned gen_ = 0;
    int pending_ = 0;
    bool stop_ = false;
};

inline HostPool& host_pool() {
    static HostPool p(host_threads() - 1);
    return p;
}

// f(i) for i in [0, n): items taken from a shared counter by the pool's threads and the caller
template <class F>
void parallel_items(int n, F&& f) {
    if (host_threads() <= 1 || n <= 1) {
        for (int i = 0; i < n; ++i) f(i);
        return;
    }
    std::atomic<int> next{0};
    auto work = [&]() {
        for (int i = next.fetch_add(1); i < n; i = next.fetch_add(1)) f(i);
    };
    if (!host_pool().run(work)) work();
}

// f(begin, end) over [0, n) in `pieces` fixed ranges
template <class F>
void parallel_ranges(int64_t n, int pieces, F&& f) {
    pieces = (int)std::max<int64_t>(1, std::min<int64_t>(pieces, n));
    parallel_items(pieces, [&](int i) { f(n * i / pieces, n * (i + 1) / pieces); });
}

}  // namespace sfmx
