// mgp_pool.h — a small persistent thread pool for the host stages (libmgphost.so).
//
// run(n, fn) calls fn(0..n-1) on the pool's threads plus the caller's and returns when
// all have finished. The decoder's passes run several times per inflated chunk (one
// chunk is ~0.1-0.4 M records): spawning a fresh std::thread per pass cost ~20 us per
// thread per pass.
#pragma once
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace mgp_host {

class Pool {
  public:
    explicit Pool(int n_threads) {
        for (int t = 1; t < n_threads; ++t) th_.emplace_back([this] { loop(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    Pool(const Pool&) = delete;
    Pool& operator=(const Pool&) = delete;
    int size() const { return (int)th_.size() + 1; }
    // fn(i) for i in [0, n), every i once
    void run(int n, const std::function<void(int)>& fn) {
        if (n <= 0) return;
        if (n == 1 || th_.empty()) {
            for (int i = 0; i < n; ++i) fn(i);
            return;
        }
        {
            std::lock_guard<std::mutex> g(mu_);
            fn_ = &fn;
            n_ = n;
            next_ = 0;
            done_ = 0;
            ++gen_;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> g(mu_);
        done_cv_.wait(g, [&] { return done_ == n_; });
        fn_ = nullptr;
    }

  private:
    void work() {
        for (;;) {
            const int i = next_.fetch_add(1);
            if (i >= n_) return;
            (*fn_)(i);
            std::lock_guard<std::mutex> g(mu_);
            if (++done_ == n_) done_cv_.notify_all();
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
            }
            work();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(int)>* fn_ = nullptr;
    std::atomic<int> next_{0};
    int n_ = 0, done_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

}  // namespace mgp_host
