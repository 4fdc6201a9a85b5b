// Host thread pool for the CPU compute backend: parallel_for / parallel_for_2d with static or
// dynamic (work-stealing counter) scheduling, and a ThreadArena that runs a callable with a given
// number of compute threads.
//
// Reference: include/threading/thread_handler.hpp:25-173 (parallel_for over TBB / OpenMP /
// serial with static, auto and affinity partitioners) and include/threading/thread_wrapper.hpp:18-47
// (TBB task_arena of N threads). Here: one persistent pool of std::threads (no TBB/OpenMP
// dependency), the calling thread takes part in every loop, nested loops run serially on the
// calling worker (no oversubscription), and chunk boundaries depend only on (range, grain,
// threads) — so reductions written per chunk and combined in chunk order are deterministic.
#pragma once
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace dcnn_native {

enum class Schedule { Static = 0, Dynamic = 1 };

class ThreadPool {
 public:
  static ThreadPool& instance();
  int num_threads() const { return nthreads_; }
  void set_num_threads(int n);
  // Run fn(task) for task in [0, ntasks) on up to num_threads() threads (caller included).
  // Blocks until every task finished. Re-entrant calls from a worker run serially.
  void run(long ntasks, const std::function<void(long)>& fn, Schedule sched = Schedule::Dynamic);
  ~ThreadPool();

 private:
  ThreadPool();
  void start(int n);
  void stop();
  void worker(int id);

  int nthreads_ = 1;
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(long)>* job_ = nullptr;
  long ntasks_ = 0;
  Schedule sched_ = Schedule::Dynamic;
  std::atomic<long> next_{0};
  std::atomic<int> active_{0};
  long generation_ = 0;
  std::atomic<long> gen_atomic_{0};   // mirrors generation_ for lock-free spinning
  bool quit_ = false;
  std::atomic<bool> quit_atomic_{false};
  std::mutex run_mu_;  // one parallel region at a time from outside the pool
};

int get_num_threads();
void set_num_threads(int n);
bool in_parallel_region();

// fn(lo, hi) over [begin, end) in chunks of >= grain elements (at most ~4 chunks per thread).
void parallel_for(long begin, long end, long grain, const std::function<void(long, long)>& fn,
                  Schedule sched = Schedule::Static);
// fn(i, j) over [0, n0) x [0, n1), flattened and chunked.
void parallel_for_2d(long n0, long n1, const std::function<void(long, long)>& fn,
                     Schedule sched = Schedule::Static);

// Deterministic chunking used by reductions: chunk k covers [k*len/nchunks, (k+1)*len/nchunks).
long reduction_chunks(long len, long grain);

// ThreadWrapper analog: run `fn` with the pool resized to `threads` compute threads, then restore.
class ThreadArena {
 public:
  explicit ThreadArena(int threads) : threads_(threads) {}
  template <typename F>
  void execute(F&& fn) {
    const int prev = get_num_threads();
    set_num_threads(threads_);
    try {
      fn();
    } catch (...) {
      set_num_threads(prev);
      throw;
    }
    set_num_threads(prev);
  }

 private:
  int threads_;
};

}  // namespace dcnn_native
