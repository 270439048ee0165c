// Persistent host worker pool for the engine's per-pair host work (planning,
// staging, the log10 finish). Spawning threads per call cost more than the
// work itself on region-sized calls (tens of microseconds per thread), so the
// workers live for the life of the library and wait on a condition variable.
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstdint>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace hcphmm {

class WorkerPool {
public:
    static WorkerPool& get()
    {
        static WorkerPool pool;
        return pool;
    }
    int size() const { return int(workers_.size()) + 1; }   // + the calling thread

    // Run fn(t) for t in [0, ntasks) on the workers and the calling thread;
    // returns when all have finished. Safe to call from several threads at once.
    // A task that throws (e.g. std::bad_alloc in a planner) does not unwind
    // past the other tasks: every task still runs or is skipped, the batch
    // drains, and the first exception is rethrown here, in the caller.
    void run(int ntasks, const std::function<void(int)>& fn)
    {
        if (ntasks <= 1 || workers_.empty()) {
            for (int t = 0; t < ntasks; ++t) fn(t);
            return;
        }
        Batch b{&fn, ntasks};
        {
            std::lock_guard<std::mutex> lk(mu_);
            queue_.push_back(&b);
        }
        // No more wake-ups than the batch has tasks (the 415 x 128 region call
        // 1.00 -> 0.95 ms at 16 threads; workers spinning for the next batch
        // measured no faster and were removed).
        const int want = std::min(ntasks - 1, int(workers_.size()));
        if (want >= int(workers_.size()))
            cv_.notify_all();
        else
            for (int k = 0; k < want; ++k) cv_.notify_one();
        const int mine = drain(b);   // the caller works too
        std::unique_lock<std::mutex> lk(mu_);
        b.finished += mine;
        // b lives on this stack: wait until every task ran and no worker holds it.
        done_cv_.wait(lk, [&] { return b.finished == b.n && b.users == 0; });
        for (size_t k = 0; k < queue_.size(); ++k)
            if (queue_[k] == &b) {
                queue_.erase(queue_.begin() + long(k));
                break;
            }
        if (b.error) std::rethrow_exception(b.error);
    }

    ~WorkerPool()
    {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& w : workers_) w.join();
    }

private:
    struct Batch {
        const std::function<void(int)>* fn;
        int n;
        std::atomic<int> next{0};
        std::atomic<bool> failed{false};
        std::exception_ptr error;   // the first task exception, set once (failed)
        int finished = 0;   // tasks run, guarded by mu_
        int users = 0;      // workers inside drain(), guarded by mu_
        Batch(const std::function<void(int)>* f, int k) : fn(f), n(k) {}
    };

    WorkerPool()
    {
        // HC_PHMM_THREADS caps the pool (default: the hardware threads, at most 16).
        unsigned hw = std::max(1u, std::thread::hardware_concurrency());
        if (const char* e = std::getenv("HC_PHMM_THREADS"))
            if (std::atoi(e) > 0) hw = unsigned(std::atoi(e));
        const int nw = int(std::min(hw, 16u)) - 1;
        for (int k = 0; k < nw; ++k) workers_.emplace_back([this] { loop(); });
    }

    // Take tasks of b until none are left; returns how many this thread ran.
    static int drain(Batch& b)
    {
        int mine = 0;
        for (int t; (t = b.next.fetch_add(1)) < b.n; ++mine) {
            if (b.failed.load(std::memory_order_relaxed)) continue;   // skip the rest after a failure
            try {
                (*b.fn)(t);
            } catch (...) {
                bool expect = false;
                if (b.failed.compare_exchange_strong(expect, true)) b.error = std::current_exception();
            }
        }
        return mine;
    }

    // First queued batch with tasks left (exhausted ones are dropped); under mu_.
    Batch* pick()
    {
        while (!queue_.empty()) {
            Batch* b = queue_.front();
            if (b->next.load() < b->n) return b;
            queue_.erase(queue_.begin());
        }
        return nullptr;
    }

    void loop()
    {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            Batch* b = nullptr;
            cv_.wait(lk, [&] { return stop_ || (b = pick()) != nullptr; });
            if (stop_) return;
            ++b->users;
            lk.unlock();
            const int mine = drain(*b);
            lk.lock();
            b->finished += mine;
            --b->users;
            if (b->finished == b->n && b->users == 0) done_cv_.notify_all();
        }
    }

    std::vector<std::thread> workers_;
    std::vector<Batch*> queue_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    bool stop_ = false;
};

// f(lo, hi) over [0, n) in chunks of at least `grain`, on the pool.
template <typename F>
void parallel_for(int64_t n, F&& f, int64_t grain = 4096)
{
    if (n <= 0) return;
    WorkerPool& P = WorkerPool::get();
    const int64_t nt = std::min<int64_t>(P.size(), (n + grain - 1) / grain);
    if (nt <= 1) {
        f(int64_t(0), n);
        return;
    }
    const int64_t tasks = nt * 4 < (n + grain - 1) / grain ? nt * 4 : nt;   // some slack for imbalance
    const int64_t chunk = (n + tasks - 1) / tasks;
    P.run(int(tasks), [&](int t) {
        const int64_t b = int64_t(t) * chunk, e = std::min(n, b + chunk);
        if (b < e) f(b, e);
    });
}

// Parallel exclusive prefix sum of f(k), k in [0, n), into out[0..n].
template <typename F>
void prefix_sum(int64_t n, std::vector<int64_t>& out, F f)
{
    out.assign(size_t(n) + 1, 0);
    if (n <= 0) return;
    const int T = int(std::min<int64_t>(32, std::max<int64_t>(1, n / 16384)));
    const int64_t chunk = (n + T - 1) / T;
    std::vector<int64_t> part(static_cast<size_t>(T) + 1, 0);
    WorkerPool::get().run(T, [&](int t) {
        int64_t s = 0;
        for (int64_t k = t * chunk, e = std::min(n, k + chunk); k < e; ++k) {
            out[size_t(k) + 1] = s += f(k);
        }
        part[size_t(t) + 1] = s;
    });
    for (int t = 1; t <= T; ++t) part[size_t(t)] += part[size_t(t) - 1];
    WorkerPool::get().run(T, [&](int t) {
        const int64_t add = part[size_t(t)];
        if (add)
            for (int64_t k = t * chunk, e = std::min(n, k + chunk); k < e; ++k) out[size_t(k) + 1] += add;
    });
}

}  // namespace hcphmm
