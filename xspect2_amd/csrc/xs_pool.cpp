// xs_pool.cpp — the library's persistent host worker threads (xs::parallel_for,
// declared in xs_internal.h).  Host code only.
//
// The library's data-parallel host passes (hit rows copied out and widened,
// offsets rebased, files read and written in pieces, ids hashed, JSON
// formatted) used to start and join fresh std::threads every call -- up to ~90
// per 400 MB result and thousands per JSON save -- and an exception while
// starting one left joinable threads behind (std::terminate).  Now they hand
// their tasks to workers started once and kept for the process.
#include <pthread.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>

#include "xs_internal.h"

namespace {

class WorkerPool {
  public:
    void run(int n, const std::function<void(int)>& fn) {
        if (n <= 1) {
            if (n == 1) fn(0);
            return;
        }
        Job job;
        job.fn = &fn;
        job.n = n;
        job.left = n - 1;
        {
            std::lock_guard<std::mutex> g(mu_);
            grow(n - 1);
            jobs_.push_back(&job);
        }
        cv_.notify_all();
        std::exception_ptr mine;
        try {
            fn(0);
        } catch (...) {
            mine = std::current_exception();
        }
        std::unique_lock<std::mutex> g(mu_);
        while (job.next < job.n) {  // the caller takes its own job's unclaimed tasks (no worker free, or none started)
            const int t = job.next++;
            if (job.next == job.n) jobs_.erase(std::find(jobs_.begin(), jobs_.end(), &job));
            g.unlock();
            std::exception_ptr e;
            try {
                fn(t);
            } catch (...) {
                e = std::current_exception();
            }
            g.lock();
            finish(&job, e);
        }
        job.done.wait(g, [&] { return job.left == 0; });
        g.unlock();
        if (mine) std::rethrow_exception(mine);
        if (job.err) std::rethrow_exception(job.err);
    }

  private:
    struct Job {
        const std::function<void(int)>* fn = nullptr;
        int n = 0, next = 1, left = 0;  // tasks 1..n-1 go to workers; left = those not finished
        std::exception_ptr err;
        std::condition_variable done;
    };
    static constexpr int kMaxWorkers = 31;

    // under mu_: the next task of the oldest job that has one
    bool claim(Job** j, int* t) {
        while (!jobs_.empty()) {
            Job* f = jobs_.front();
            if (f->next < f->n) {
                *j = f;
                *t = f->next++;
                if (f->next == f->n) jobs_.pop_front();
                return true;
            }
            jobs_.pop_front();
        }
        return false;
    }
    // under mu_
    void finish(Job* j, std::exception_ptr e) {
        if (e && !j->err) j->err = e;
        if (--j->left == 0) j->done.notify_all();
    }
    // under mu_: at least `want` workers (as many as the system lets us start, at most kMaxWorkers)
    void grow(int want) {
        want = std::min(want, kMaxWorkers);
        while (workers_ < want) {
            try {
                std::thread([this] { loop(); }).detach();
            } catch (...) {
                return;  // fewer workers: the callers run the remaining tasks themselves
            }
            ++workers_;
        }
    }
    void loop() {
        std::unique_lock<std::mutex> g(mu_);
        for (;;) {
            Job* j = nullptr;
            int t = 0;
            while (!claim(&j, &t)) cv_.wait(g);
            g.unlock();
            std::exception_ptr e;
            try {
                (*j->fn)(t);
            } catch (...) {
                e = std::current_exception();
            }
            g.lock();
            finish(j, e);
        }
    }

    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<Job*> jobs_;
    int workers_ = 0;
};

// Never destroyed: its detached workers outlive static destruction at exit.  A
// forked child (Python multiprocessing with the fork start method) has none of
// the parent's workers and maybe a mutex a vanished worker held: it starts
// from a fresh pool (the old one is left behind, unused).
std::atomic<WorkerPool*> g_pool{nullptr};
std::once_flag g_pool_once;

WorkerPool& pool() {
    std::call_once(g_pool_once, [] {
        g_pool.store(new WorkerPool);
        (void)pthread_atfork(nullptr, nullptr, [] { g_pool.store(new WorkerPool); });
    });
    return *g_pool.load();
}
}  // namespace

void xs::parallel_for(int n, const std::function<void(int)>& fn) { pool().run(n, fn); }
