// Persistent host thread pool (see threadpool.h).
#include "threadpool.h"

#include <algorithm>
#include <cstdlib>

namespace dcnn_native {

namespace {
thread_local bool tl_in_region = false;

int default_threads() {
  if (const char* e = std::getenv("DCNN_NUM_THREADS")) {
    const int v = std::atoi(e);
    if (v > 0) return v;
  }
  if (const char* e = std::getenv("OMP_NUM_THREADS")) {
    const int v = std::atoi(e);
    if (v > 0) return v;
  }
  const unsigned hc = std::thread::hardware_concurrency();
  return hc ? (int)std::min(hc, 64u) : 1;
}
}  // namespace

ThreadPool& ThreadPool::instance() {
  static ThreadPool pool;
  return pool;
}

ThreadPool::ThreadPool() { start(default_threads()); }

ThreadPool::~ThreadPool() { stop(); }

void ThreadPool::start(int n) {
  nthreads_ = std::max(1, n);
  quit_ = false;
  quit_atomic_.store(false, std::memory_order_relaxed);
  for (int i = 1; i < nthreads_; ++i) workers_.emplace_back(&ThreadPool::worker, this, i);
}

void ThreadPool::stop() {
  {
    std::lock_guard<std::mutex> g(mu_);
    quit_ = true;
    quit_atomic_.store(true, std::memory_order_relaxed);
  }
  cv_.notify_all();
  for (auto& t : workers_) t.join();
  workers_.clear();
}

void ThreadPool::set_num_threads(int n) {
  n = std::max(1, n);
  std::lock_guard<std::mutex> r(run_mu_);
  if (n == nthreads_) return;
  stop();
  start(n);
}

// No spin-before-block: on virtualised hosts PAUSE loops trap to the hypervisor and spinning
// threads steal the vCPUs the work needs (measured: 8 spinning workers made a 100 us loop take
// 3 ms), so workers and the caller sleep on the condition variables right away.
namespace {
constexpr int spin_iters() { return 0; }
inline void cpu_relax() { __builtin_ia32_pause(); }
}  // namespace

void ThreadPool::worker(int) {
  long seen = 0;
  for (;;) {
    for (int i = 0, n = spin_iters(); i < n && gen_atomic_.load(std::memory_order_acquire) == seen &&
                    !quit_atomic_.load(std::memory_order_relaxed);
         ++i)
      cpu_relax();
    const std::function<void(long)>* job;
    long ntasks;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return quit_ || generation_ != seen; });
      if (quit_) return;
      seen = generation_;
      job = job_;
      ntasks = ntasks_;
    }
    tl_in_region = true;
    for (long t; (t = next_.fetch_add(1, std::memory_order_relaxed)) < ntasks;) (*job)(t);
    tl_in_region = false;
    if (active_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
      std::lock_guard<std::mutex> g(mu_);
      done_cv_.notify_all();
    }
  }
}

void ThreadPool::run(long ntasks, const std::function<void(long)>& fn, Schedule sched) {
  if (ntasks <= 0) return;
  if (tl_in_region || nthreads_ == 1 || ntasks == 1) {
    for (long t = 0; t < ntasks; ++t) fn(t);
    return;
  }
  (void)sched;  // tasks are sized by the callers to fixed index ranges: dynamic dispatch of them
                // never changes results, whichever thread runs a task
  std::lock_guard<std::mutex> r(run_mu_);
  {
    std::lock_guard<std::mutex> g(mu_);
    job_ = &fn;
    ntasks_ = ntasks;
    next_.store(0, std::memory_order_relaxed);
    active_.store((int)workers_.size(), std::memory_order_relaxed);
    ++generation_;
    gen_atomic_.store(generation_, std::memory_order_release);
  }
  cv_.notify_all();
  tl_in_region = true;
  for (long t; (t = next_.fetch_add(1, std::memory_order_relaxed)) < ntasks;) fn(t);
  tl_in_region = false;
  for (int i = 0, n = spin_iters(); i < n && active_.load(std::memory_order_acquire) != 0; ++i) cpu_relax();
  if (active_.load(std::memory_order_acquire) != 0) {
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return active_.load(std::memory_order_acquire) == 0; });
  }
  job_ = nullptr;
}

int get_num_threads() { return ThreadPool::instance().num_threads(); }
void set_num_threads(int n) { ThreadPool::instance().set_num_threads(n); }
bool in_parallel_region() { return tl_in_region; }

long reduction_chunks(long len, long grain) {
  if (len <= 0) return 0;
  grain = std::max(1L, grain);
  const long by_grain = (len + grain - 1) / grain;
  return std::max(1L, std::min(by_grain, 256L));  // independent of the thread count: deterministic
}

void parallel_for(long begin, long end, long grain, const std::function<void(long, long)>& fn, Schedule sched) {
  const long len = end - begin;
  if (len <= 0) return;
  const long nchunks = reduction_chunks(len, grain);
  if (nchunks == 1) {
    fn(begin, end);
    return;
  }
  ThreadPool::instance().run(
      nchunks,
      [&](long k) {
        const long lo = begin + k * len / nchunks, hi = begin + (k + 1) * len / nchunks;
        if (lo < hi) fn(lo, hi);
      },
      sched);
}

void parallel_for_2d(long n0, long n1, const std::function<void(long, long)>& fn, Schedule sched) {
  parallel_for(
      0, n0 * n1, 1,
      [&](long lo, long hi) {
        for (long k = lo; k < hi; ++k) fn(k / n1, k % n1);
      },
      sched);
}

}  // namespace dcnn_native
