// Host-side parallel loop for the BA problem setup (sfmx_ba_create / _update / _solve): the
// reference adjusts a growing scene after every registered camera (SfM.cpp:235 / :371), so the
// O(observations) host work of every call is on the critical path.  Work is split into a FIXED
// number of ranges (independent of the machine's thread count), so every result is the same on
// every host; the ranges run on up to 16 threads (a persistent pool).
#pragma once
#include "diag.hpp"
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace sfmx {

// diagnostic library only (diag.hpp): SFMX_HOST_THREADS (1 .. 64, default 16), SFMX_HOST_SPIN_US (0 .. 100000,
// default below); read once
inline int env_int(const char* v, int def, int lo, int hi) {
    return v ? std::max(lo, std::min(hi, std::atoi(v))) : def;
}
inline int host_threads() {
    static const int n = [] {
        const unsigned h = std::thread::hardware_concurrency();
        return std::min(env_int(SFMX_DIAG_ENV("SFMX_HOST_THREADS"), 16, 1, 64), (int)std::max(1u, h ? h : 1u));
    }();
    return n;
}

// A persistent worker pool (host_threads() - 1 threads, started on first use): spawning and joining
// 15 std::threads per parallel loop cost ~0.1-0.2 ms each, and a BA call makes ~15 such loops.  One
// job at a time; a caller that finds the pool busy (another thread's loop) runs its loop serially.
// r05: a worker spins on the job generation for SPIN_US after its last job before it blocks on the
// condition variable, and the caller spins on the completion count: a load's parallel loops come in
// bursts a few hundred us apart, and a condition-variable wake-up of every worker per loop (each loop
// waits for its slowest worker) cost 50-400 us per loop on a loaded host.
class HostPool {
public:
    static constexpr int SPIN_US = 1000;   // r06: 3000 before; CPU burn between calls
    const int spin_us = env_int(SFMX_DIAG_ENV("SFMX_HOST_SPIN_US"), SPIN_US, 0, 100000);
    explicit HostPool(int workers) {
        for (int t = 0; t < workers; ++t) th_.emplace_back([this] { loop(); });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_.store(true);
            gen_.fetch_add(1, std::memory_order_release);
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
        job_.store(&job, std::memory_order_relaxed);
        pending_.store((int)th_.size(), std::memory_order_relaxed);
        {
            std::lock_guard<std::mutex> lk(mu_);   // (a worker about to block re-checks the generation under it)
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        work();
        while (pending_.load(std::memory_order_acquire) != 0) cpu_relax();
        job_.store(nullptr, std::memory_order_relaxed);
        return true;
    }

private:
    static void cpu_relax() {
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
    }
    void loop() {
        unsigned seen = 0;
        for (;;) {
            unsigned g = gen_.load(std::memory_order_acquire);
            if (g == seen) {   // spin a while, then block
                const auto t0 = std::chrono::steady_clock::now();
                for (int i = 0; g == seen; ++i) {
                    cpu_relax();
                    g = gen_.load(std::memory_order_acquire);
                    if ((i & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us)) break;
                }
                if (g == seen) {
                    std::unique_lock<std::mutex> lk(mu_);
                    cv_.wait(lk, [&] { return gen_.load(std::memory_order_acquire) != seen; });
                    g = gen_.load(std::memory_order_acquire);
                }
            }
            seen = g;
            if (stop_.load()) return;
            std::function<void()>* job = job_.load(std::memory_order_relaxed);
            (*job)();
            pending_.fetch_sub(1, std::memory_order_acq_rel);
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_, run_mu_;
    std::condition_variable cv_;
    std::atomic<std::function<void()>*> job_{nullptr};
    std::atomic<unsigned> gen_{0};
    std::atomic<int> pending_{0};
    std::atomic<bool> stop_{false};
};

inline HostPool& host_pool() {
    static HostPool p(host_threads() - 1);
    return p;
}

// One persistent side thread for a job that runs beside the caller's parallel loops (the BA load's
// factorization plan): std::async spawned a thread per call (~30-50 us on the critical path).
class SideThread {
public:
    SideThread() : th_([this] { loop(); }) {}
    ~SideThread() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        th_.join();
    }
    void submit(std::function<void()> f) {
        wait();
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = std::move(f);
            busy_ = true;
        }
        cv_.notify_all();
    }
    void wait() {
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [this] { return !busy_; });
    }

private:
    void loop() {
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [this] { return stop_ || (busy_ && job_); });
                if (stop_) return;
                f = std::move(job_);
                job_ = nullptr;
            }
            f();
            {
                std::lock_guard<std::mutex> lk(mu_);
                busy_ = false;
            }
            done_.notify_all();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_, done_;
    std::function<void()> job_;
    bool busy_ = false, stop_ = false;
    std::thread th_;
};

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
