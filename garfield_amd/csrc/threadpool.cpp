#include "threadpool.hpp"

#include <atomic>
#include <cstdlib>
#include <exception>

namespace garfield {
namespace cpu {

ThreadPool::ThreadPool(size_t nthreads) {
  if (nthreads == 0) nthreads = 1;
  workers_.reserve(nthreads);
  for (size_t i = 0; i < nthreads; ++i) workers_.emplace_back([this] { loop(); });
}

ThreadPool::~ThreadPool() {
  {
    std::lock_guard<std::mutex> g(mutex_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : workers_) t.join();
}

void ThreadPool::loop() {
  for (;;) {
    std::function<void()> job;
    {
      std::unique_lock<std::mutex> lk(mutex_);
      cv_.wait(lk, [this] { return stop_ || !jobs_.empty(); });
      if (stop_ && jobs_.empty()) return;
      job = std::move(jobs_.front());
      jobs_.pop();
    }
    job();
  }
}

void ThreadPool::run_chunks(size_t nchunks, const std::function<void(size_t)>& fn) {
  if (nchunks == 0) return;
  if (nchunks == 1 || workers_.size() <= 1) {
    for (size_t c = 0; c < nchunks; ++c) fn(c);
    return;
  }
  std::atomic<size_t> next{0};
  size_t done = 0;  // guarded by wmx: the waiter may only return (and destroy these locals)
                    // once the last task has left its critical section
  std::mutex emx;
  std::exception_ptr err;
  std::mutex wmx;
  std::condition_variable wcv;
  const size_t ntasks = nchunks < workers_.size() ? nchunks : workers_.size();
  auto task = [&] {
    for (;;) {
      const size_t c = next.fetch_add(1);
      if (c >= nchunks) break;
      try {
        fn(c);
      } catch (...) {
        std::lock_guard<std::mutex> g(emx);
        if (!err) err = std::current_exception();
      }
    }
    std::lock_guard<std::mutex> g(wmx);
    if (++done == ntasks) wcv.notify_all();
  };
  {
    std::lock_guard<std::mutex> g(mutex_);
    for (size_t i = 0; i < ntasks; ++i) jobs_.push(task);
  }
  cv_.notify_all();
  {
    std::unique_lock<std::mutex> lk(wmx);
    wcv.wait(lk, [&] { return done == ntasks; });
  }
  if (err) std::rethrow_exception(err);
}

ThreadPool& pool() {
  static ThreadPool p([] {
    const char* env = std::getenv("GARFIELD_NUM_THREADS");
    long v = env ? std::strtol(env, nullptr, 10) : 0;
    if (v <= 0) v = static_cast<long>(std::thread::hardware_concurrency());
    if (v <= 0) v = 1;
    return static_cast<size_t>(v);
  }());
  return p;
}

void parallel_for(size_t begin, size_t end, size_t nchunks,
                  const std::function<void(size_t, size_t, size_t)>& fn) {
  if (end <= begin) return;
  const size_t range = end - begin;
  if (nchunks == 0) nchunks = 1;
  if (nchunks > range) nchunks = range;
  const size_t per = (range + nchunks - 1) / nchunks;
  pool().run_chunks(nchunks, [&](size_t c) {
    const size_t lo = begin + c * per;
    size_t hi = lo + per;
    if (hi > end) hi = end;
    if (lo < hi) fn(c, lo, hi);
  });
}

size_t default_chunks(size_t range, size_t min_per_chunk) {
  size_t c = range / (min_per_chunk ? min_per_chunk : 1);
  if (c < 1) c = 1;
  if (c > 256) c = 256;
  return c;
}

}  // namespace cpu
}  // namespace garfield
