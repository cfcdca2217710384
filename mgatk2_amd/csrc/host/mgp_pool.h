// mgp_pool.h — a small persistent thread pool for the host stages (libmgphost.so).
//
// run(n, fn) calls fn(0..n-1) on the pool's threads plus the caller's and returns when
// all have finished. The decoder's passes run several times per inflated chunk (one
// chunk is ~0.1-0.4 M records): spawning a fresh std::thread per pass cost ~20 us per
// thread per pass.
//
// Every run has its own job state (fn, n, index counter, done and active counts) on
// the caller's stack. A worker joins a job under the mutex and only while the job is
// published; run() returns once every item is done AND no worker is still inside the
// job's work loop, so a worker late out of one run can never claim an index of the
// next run's counter against the previous run's bound (each job's bound is constant).
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
        Job job(&fn, n);
        {
            std::lock_guard<std::mutex> g(mu_);
            job_ = &job;
            ++gen_;
        }
        cv_.notify_all();
        work(job);
        std::unique_lock<std::mutex> g(mu_);
        done_cv_.wait(g, [&] { return job.done == job.n && job.active == 0; });
        job_ = nullptr;  // (under the lock: no worker can join it any more)
    }

  private:
    struct Job {
        Job(const std::function<void(int)>* f, int count) : fn(f), n(count) {}
        const std::function<void(int)>* const fn;
        const int n;
        std::atomic<int> next{0};
        int done = 0, active = 0;  // (under mu_)
    };
    void work(Job& j) {
        for (;;) {
            const int i = j.next.fetch_add(1);
            if (i >= j.n) return;
            (*j.fn)(i);
            std::lock_guard<std::mutex> g(mu_);
            if (++j.done == j.n) done_cv_.notify_all();
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            Job* j;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return stop_ || (job_ != nullptr && gen_ != seen); });
                if (stop_) return;
                seen = gen_;
                j = job_;
                ++j->active;
            }
            work(*j);
            std::lock_guard<std::mutex> g(mu_);
            if (--j->active == 0 && j->done == j->n) done_cv_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    Job* job_ = nullptr;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

}  // namespace mgp_host
