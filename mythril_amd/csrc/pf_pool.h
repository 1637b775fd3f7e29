// Persistent host worker pool for the batch entry points of libpflower.so
// (pflt_lower_many, pflt_recheck_many).  The workers start on first use and then wait on a
// condition variable, so the fork-join over a single query's few buckets costs a wake-up, not
// a thread creation and join per call (std::thread per call was ~20-40 us each — as long as
// lowering a small bucket).  Host-only C++; the pool is never destroyed (its detached workers
// would otherwise wait on a destroyed condition variable at process exit).
// fork(): the child has none of the parent's workers, and the pool's mutexes may have been
// held by a parent thread at the fork — so a pthread_atfork child handler gives the child a
// fresh pool (the parent's is left untouched: its state is garbage in the child).  Without it
// a child of a process that had used the pool waited forever on busy_ for workers that do
// not exist (tools/full_pass.py's default-fork ProcessPoolExecutor).
#pragma once

#include <pthread.h>

#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace pfpool {

class Pool {
   public:
    // fn(0) .. fn(n - 1) on the caller and up to n_threads - 1 workers; returns when all ran.
    // fn must not throw (lower_job and the re-check report failures in their results) and
    // must not call run() itself (one fork-join at a time)
    void run(size_t n, size_t n_threads, const std::function<void(size_t)>& fn) {
        const size_t nt = n_threads < n ? n_threads : n;
        if (nt <= 1) {
            for (size_t j = 0; j < n; j++) fn(j);
            return;
        }
        std::lock_guard<std::mutex> serial(run_m_);  // one fork-join at a time
        {
            std::lock_guard<std::mutex> lk(m_);
            while (workers_.size() < nt - 1) {
                const size_t id = workers_.size();
                workers_.emplace_back([this, id] { work(id); });
                workers_.back().detach();
            }
            fn_ = &fn;
            n_ = n;
            next_.store(0);
            want_ = nt - 1;
            busy_ = nt - 1;
            ++gen_;
        }
        cv_work_.notify_all();
        for (size_t j; (j = next_.fetch_add(1)) < n;) fn(j);
        std::unique_lock<std::mutex> lk(m_);
        cv_done_.wait(lk, [this] { return busy_ == 0; });
        fn_ = nullptr;
    }

   private:
    void work(size_t id) {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(m_);
        for (;;) {
            cv_work_.wait(lk, [&] { return gen_ != seen; });
            seen = gen_;
            if (id >= want_) continue;  // not needed this round
            const std::function<void(size_t)>* f = fn_;
            const size_t n = n_;
            lk.unlock();
            for (size_t j; (j = next_.fetch_add(1)) < n;) (*f)(j);
            lk.lock();
            if (--busy_ == 0) cv_done_.notify_one();
        }
    }

    std::mutex run_m_, m_;
    std::condition_variable cv_work_, cv_done_;
    std::vector<std::thread> workers_;
    const std::function<void(size_t)>* fn_ = nullptr;
    size_t n_ = 0, want_ = 0, busy_ = 0;
    uint64_t gen_ = 0;
    std::atomic<size_t> next_{0};
};

inline Pool*& pool_ptr() {
    static Pool* p = new Pool();  // never destroyed (see above)
    return p;
}

inline Pool& pool() {
    static const int registered = pthread_atfork(nullptr, nullptr, [] { pool_ptr() = new Pool(); });
    (void)registered;
    return *pool_ptr();
}

inline void parallel_for(size_t n, size_t n_threads, const std::function<void(size_t)>& fn) {
    pool().run(n, n_threads ? n_threads : 1, fn);
}

}  // namespace pfpool
