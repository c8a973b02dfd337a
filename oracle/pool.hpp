// TEST INFRASTRUCTURE ONLY (the all-cores CPU baseline legs of bench.py; see rsvio_oracle.h).
//
// A persistent worker pool with dynamic scheduling -- the rayon analogue the reference's
// par_iter calls run on (src/feature_tracker/feature_tracker.rs:213,260): the workers are created
// once and kept, tasks are claimed from an atomic counter (rayon's work stealing, for independent
// tasks), and the calling thread works too.  Idle workers spin briefly before they sleep, so a
// burst of small parallel regions (an LM iteration's several passes over a window's landmarks)
// does not pay a thread start or a futex wake each time.
#pragma once

#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace orc {

class Pool {
public:
    static Pool& get() {
        static Pool p;
        return p;
    }

    // f(task) for task in [0, n_tasks) on up to `threads` threads (the caller included); returns
    // when every task has run.  threads <= 1 or one task: inline, in task order.
    template <class F>
    void run(int n_tasks, int threads, F&& f) {
        if (n_tasks <= 0) return;
        if (threads <= 1 || n_tasks == 1) {
            for (int i = 0; i < n_tasks; ++i) f(i);
            return;
        }
        std::lock_guard<std::mutex> serial(run_mu_);  // one parallel region at a time
        ensure(threads - 1);
        const int a = std::min(threads - 1, (int)workers_.size());
        {
            std::lock_guard<std::mutex> lk(mu_);
            fn_ = [&f](int i) { f(i); };
            n_tasks_ = n_tasks;
            next_.store(0, std::memory_order_relaxed);
            done_.store(0, std::memory_order_relaxed);
            left_.store(0, std::memory_order_relaxed);
            active_ = a;
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        work();
        // every active worker has left this region's task loop before fn_ goes out of scope (and
        // before the next region starts: no worker can miss a region it is active in)
        while (done_.load(std::memory_order_acquire) < n_tasks || left_.load(std::memory_order_acquire) < a) pause();
    }

    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }

private:
    static void pause() {
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
    }

    void ensure(int n) {
        while ((int)workers_.size() < n) {
            const int id = (int)workers_.size();
            workers_.emplace_back([this, id] { loop(id); });
        }
    }

    void work() {
        for (;;) {
            const int i = next_.fetch_add(1, std::memory_order_relaxed);
            if (i >= n_tasks_) return;
            fn_(i);
            done_.fetch_add(1, std::memory_order_release);
        }
    }

    void loop(int id) {
        unsigned long long seen = 0;
        for (;;) {
            // spin ~50 us for the next region, then sleep on the condition variable; the region's
            // parameters are read under the mutex they were published under
            for (int s = 0; gen_.load(std::memory_order_acquire) == seen && s < 20000; ++s) pause();
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return gen_.load(std::memory_order_relaxed) != seen; });
            seen = gen_.load(std::memory_order_relaxed);
            const bool stop = stop_, active = id < active_;
            lk.unlock();
            if (stop) return;
            if (!active) continue;  // a region that asked for fewer threads
            work();
            left_.fetch_add(1, std::memory_order_release);
        }
    }

    std::vector<std::thread> workers_;
    std::mutex run_mu_, mu_;
    std::condition_variable cv_;
    std::atomic<unsigned long long> gen_{0};
    std::atomic<int> next_{0}, done_{0}, left_{0};
    std::function<void(int)> fn_;
    int n_tasks_ = 0, active_ = 0;
    bool stop_ = false;
};

}  // namespace orc
