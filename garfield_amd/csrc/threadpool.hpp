// Process-wide CPU worker pool for the CPU (gloo / plumbing) aggregation path.
//
// Reference counterpart: so_threadpool (pytorch_impl/libs/native/so_threadpool/
// threadpool.cpp:80-149, include/threadpool.hpp:52-222) — a FIFO job queue and a
// parallel_for that splits a range into <= nbworkers chunks. This pool keeps the
// same contract but splits into a FIXED number of chunks (independent of the
// thread count), so reductions that combine per-chunk partials in chunk order are
// bitwise reproducible on any machine.
#pragma once
#include <condition_variable>
#include <cstddef>
#include <functional>
#include <mutex>
#include <queue>
#include <thread>
#include <vector>

namespace garfield {
namespace cpu {

class ThreadPool {
 public:
  explicit ThreadPool(size_t nthreads);
  ~ThreadPool();
  ThreadPool(const ThreadPool&) = delete;
  ThreadPool& operator=(const ThreadPool&) = delete;

  size_t size() const { return workers_.size(); }

  // Run fn(chunk_index) for chunk_index in [0, nchunks) and wait for all of them.
  // Exceptions thrown by fn are re-thrown (first one wins) on the calling thread.
  void run_chunks(size_t nchunks, const std::function<void(size_t)>& fn);

 private:
  void loop();
  std::vector<std::thread> workers_;
  std::queue<std::function<void()>> jobs_;
  std::mutex mutex_;
  std::condition_variable cv_;
  bool stop_ = false;
};

// Global pool (size: GARFIELD_NUM_THREADS or hardware concurrency).
ThreadPool& pool();

// Split [begin, end) into `nchunks` contiguous pieces (fixed, data-size based)
// and call fn(chunk, lo, hi) for each non-empty piece in parallel.
void parallel_for(size_t begin, size_t end, size_t nchunks,
                  const std::function<void(size_t, size_t, size_t)>& fn);

// Convenience: chunk count derived from the range only (never from the thread count).
size_t default_chunks(size_t range, size_t min_per_chunk = 4096);

}  // namespace cpu
}  // namespace garfield
