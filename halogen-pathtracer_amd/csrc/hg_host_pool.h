// hg_host_pool.h — a small persistent host thread pool for hg_upload_scene's byte compare, copies and repack (the
// moving-camera frame calls hg_upload_scene once per frame, so per-call thread creation would cost a good part of the
// ~1 ms compare).  Workers are started on first use and live for the process; one job runs at a time (callers are
// serialised by a mutex); the calling thread works on the job too.  Host-only.
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

class HgHostPool {
   public:
    static HgHostPool& get() {
        static HgHostPool pool(std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
        return pool;
    }
    int threads() const { return int(workers_.size()) + 1; }

    // fn(task) for task in [0, n_tasks), spread over the workers and the calling thread; returns when all are done
    void run(size_t n_tasks, const std::function<void(size_t)>& fn) {
        if (n_tasks == 0) return;
        if (n_tasks == 1 || workers_.empty()) {
            for (size_t t = 0; t < n_tasks; ++t) fn(t);
            return;
        }
        std::lock_guard<std::mutex> job_lock(job_mu_);  // one job at a time
        {
            std::lock_guard<std::mutex> lk(mu_);
            fn_ = &fn;
            n_tasks_ = n_tasks;
            next_.store(0);
            done_ = 0;
            ++generation_;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [&] { return done_ == workers_.size(); });
        fn_ = nullptr;
    }

    ~HgHostPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
            ++generation_;
        }
        cv_.notify_all();
        for (auto& w : workers_) w.join();
    }

   private:
    explicit HgHostPool(unsigned n) {
        for (unsigned i = 1; i < n; ++i) workers_.emplace_back([this] { loop(); });
    }
    void work() {
        for (size_t t = next_.fetch_add(1); t < n_tasks_; t = next_.fetch_add(1)) (*fn_)(t);
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return generation_ != seen; });
                seen = generation_;
                if (stop_) return;
            }
            work();
            {
                std::lock_guard<std::mutex> lk(mu_);
                ++done_;
            }
            done_cv_.notify_one();
        }
    }
    std::vector<std::thread> workers_;
    std::mutex job_mu_, mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(size_t)>* fn_ = nullptr;
    size_t n_tasks_ = 0, done_ = 0;
    std::atomic<size_t> next_{0};
    uint64_t generation_ = 0;
    bool stop_ = false;
};
