// Host-side self-test of the native CPU runtime, built with -fsanitize=thread or
// -fsanitize=address by tests/test_native_sanitizers.py (race / memory-error
// detection: the reference had none). Exercises:
//  * ThreadPool::run_chunks from several caller threads at once (the completion
//    protocol that once let a waiter destroy its condvar under a notifier);
//  * the CPU GARs (pairwise distances, Krum / Bulyan / Brute selections,
//    coordinate-wise rules) against simple serial recomputations;
//  * Mailbox: concurrent writers publishing tagged slots while a reader waits.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <random>
#include <thread>
#include <vector>

#include "gar_common.hpp"
#include "gar_cpu.hpp"
#include "mailbox.hpp"
#include "threadpool.hpp"

using namespace garfield;

static int failures = 0;
#define CHECK(c)                                                    \
  do {                                                              \
    if (!(c)) {                                                     \
      std::fprintf(stderr, "CHECK failed: %s (line %d)\n", #c, __LINE__); \
      ++failures;                                                   \
    }                                                               \
  } while (0)

static void test_pool() {
  std::vector<std::thread> callers;
  std::atomic<long> total{0};
  for (int c = 0; c < 6; ++c) {
    callers.emplace_back([&total] {
      for (int rep = 0; rep < 200; ++rep) {
        std::vector<long> part(37, 0);
        cpu::parallel_for(0, 10000, 37, [&](size_t chunk, size_t lo, size_t hi) {
          long s = 0;
          for (size_t i = lo; i < hi; ++i) s += static_cast<long>(i);
          part[chunk] = s;
        });
        long s = 0;
        for (long p : part) s += p;
        total += s;
      }
    });
  }
  for (auto& t : callers) t.join();
  CHECK(total.load() == 6L * 200L * (9999L * 10000L / 2));
}

static void test_gars() {
  std::mt19937 rng(7);
  std::normal_distribution<float> nd;
  const size_t n = 11, d = 3001, f = 2;
  std::vector<std::vector<float>> data(n, std::vector<float>(d));
  for (size_t i = 0; i < n; ++i)
    for (size_t x = 0; x < d; ++x) data[i][x] = nd(rng) * (1.0f + 0.3f * static_cast<float>(i));
  cpu::Rows<float> r;
  r.n = n;
  r.d = d;
  for (auto& v : data) r.p.push_back(v.data());
  auto D = cpu::pairwise_sqdist(r);
  for (size_t i = 0; i < n; ++i)
    for (size_t j = 0; j < n; ++j) {
      if (i == j) continue;
      double s = 0;
      for (size_t x = 0; x < d; ++x) {
        const double a = static_cast<double>(data[i][x]) - data[j][x];
        s += a * a;
      }
      CHECK(std::fabs(D[i * n + j] - s) <= 1e-9 * s);
    }
  auto w = cpu::krum_weights(D, n, f, n - f - 2);
  float tot = 0;
  for (float x : w) tot += x;
  CHECK(std::fabs(tot - 1.f) < 1e-5f);
  auto W = cpu::bulyan_weights(D, n - 2, f, n - 2 - f - 2, n - 2 - 2 * f - 2);
  CHECK(!W.empty());
  auto wb = cpu::brute_weights(D, n, f);
  size_t sel = 0;
  for (float x : wb) sel += x != 0.f;
  CHECK(sel == n - f);
  std::vector<float> out(d);
  cpu::coordwise<float>(r, kMedian, 0, 0, {}, 0, 0, 0, out.data());
  for (size_t x = 0; x < d; x += 97) {
    std::vector<float> col;
    for (size_t i = 0; i < n; ++i) col.push_back(data[i][x]);
    std::sort(col.begin(), col.end());
    CHECK(out[x] == col[n / 2]);
  }
  cpu::coordwise<float>(r, kTrimmedMean, f, 0, {}, 0, 0, 0, out.data());
  cpu::combine<float>(r, w, out.data());
}

static void test_mailbox() {
  mailbox::Mailbox mb(8, 4096, false);
  std::vector<std::thread> writers;
  for (int it = 1; it <= 50; ++it) {
    writers.clear();
    for (int s = 0; s < 8; ++s) {
      writers.emplace_back([&mb, s, it] {
        std::vector<float> buf(1024, static_cast<float>(it * 100 + s));
        mb.write(static_cast<size_t>(s), it, buf.data(), buf.size() * sizeof(float));
      });
    }
    auto ids = mb.wait(it, 6, 5.0);
    CHECK(ids.size() >= 6);
    for (auto& t : writers) t.join();
    auto all = mb.ready(it);
    CHECK(all.size() == 8);
    for (size_t id : all) CHECK(static_cast<const float*>(mb.slot(id))[1023] == static_cast<float>(it * 100 + id));
  }
}

int main() {
  test_pool();
  test_gars();
  test_mailbox();
  if (failures) {
    std::fprintf(stderr, "selftest: %d failure(s)\n", failures);
    return 1;
  }
  std::printf("selftest: ok\n");
  return 0;
}
